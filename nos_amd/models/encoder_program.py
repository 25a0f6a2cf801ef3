"""A pre-LN transformer encoder (ViT / BERT-style trunk) as a pod-server
program, numpy only.

Any tenant whose model is a stack of ``torch.nn.TransformerEncoderLayer``
(``norm_first=True``, GELU, batch-first) ships it to the pod server with this
builder: the weight names are the module's ``state_dict`` keys
(``layers.{i}.self_attn.in_proj_weight`` ...), the input is the float token
embeddings ``[batch, seq, hidden]`` (embedding lookups stay in the client),
and the server's compiler lowers every layer onto the same fused kernels as
YOLOS -- LN folded into the QKV and FC1 GEMMs, QKV + attention fused,
residual adds and GELU in the GEMM epilogues.  Heads must be 64 wide and the
widths multiples of 64 for the gfx950 kernels (checked at parse time).
"""
from __future__ import annotations

import numpy as np

from ..podserver.program import Builder


def encoder_program(weights: dict[str, np.ndarray], num_layers: int, heads: int, input_shape: tuple[int, int, int],
                    dtype: str = "fp32", eps: float = 1e-5, final_norm: bool = True,
                    prefix: str = "layers.") -> tuple[dict, bytes]:
    """(program, payload) for ``num_layers`` encoder layers named
    ``{prefix}{i}.*`` (and ``norm.weight`` / ``norm.bias`` if
    ``final_norm``) on an fp32 input of ``input_shape``."""
    b = Builder(f"encoder-l{num_layers}-h{input_shape[-1]}-{dtype}")
    P = {k: b.param(k, v, dtype) for k, v in weights.items()}
    x = b.input("x", list(input_shape), "fp32")
    h = b.op("cast", x, dtype=dtype) if dtype != "fp32" else x
    for i in range(num_layers):
        L = f"{prefix}{i}."
        y = b.op("layernorm", h, P[L + "norm1.weight"], P[L + "norm1.bias"], eps=eps)
        qkv = b.op("linear", y, P[L + "self_attn.in_proj_weight"], P[L + "self_attn.in_proj_bias"])
        a = b.op("attention", qkv, heads=heads)
        h = b.op("add", h, b.op("linear", a, P[L + "self_attn.out_proj.weight"], P[L + "self_attn.out_proj.bias"]))
        y = b.op("layernorm", h, P[L + "norm2.weight"], P[L + "norm2.bias"], eps=eps)
        y = b.op("gelu", b.op("linear", y, P[L + "linear1.weight"], P[L + "linear1.bias"]))
        h = b.op("add", h, b.op("linear", y, P[L + "linear2.weight"], P[L + "linear2.bias"]))
    if final_norm:
        h = b.op("layernorm", h, P["norm.weight"], P["norm.bias"], eps=eps)
    if dtype != "fp32":
        h = b.op("cast", h, dtype="fp32")
    return b.build([h])


def random_encoder_weights(num_layers: int, hidden: int, mlp: int, seed: int = 0,
                           final_norm: bool = True) -> dict[str, np.ndarray]:
    """Random-init weights under ``nn.TransformerEncoder`` state-dict names."""
    rng = np.random.default_rng(seed)

    def n(*shape, s):
        return (rng.standard_normal(shape, dtype=np.float32) * s).astype(np.float32)

    w: dict[str, np.ndarray] = {}
    for i in range(num_layers):
        L = f"layers.{i}."
        w.update({L + "self_attn.in_proj_weight": n(3 * hidden, hidden, s=hidden ** -0.5),
                  L + "self_attn.in_proj_bias": n(3 * hidden, s=0.02),
                  L + "self_attn.out_proj.weight": n(hidden, hidden, s=hidden ** -0.5),
                  L + "self_attn.out_proj.bias": n(hidden, s=0.02),
                  L + "linear1.weight": n(mlp, hidden, s=hidden ** -0.5), L + "linear1.bias": n(mlp, s=0.02),
                  L + "linear2.weight": n(hidden, mlp, s=mlp ** -0.5), L + "linear2.bias": n(hidden, s=0.02),
                  L + "norm1.weight": 1 + n(hidden, s=0.1), L + "norm1.bias": n(hidden, s=0.1),
                  L + "norm2.weight": 1 + n(hidden, s=0.1), L + "norm2.bias": n(hidden, s=0.1)})
    if final_norm:
        w["norm.weight"], w["norm.bias"] = 1 + n(hidden, s=0.1), n(hidden, s=0.1)
    return w


__all__ = ["encoder_program", "random_encoder_weights"]
