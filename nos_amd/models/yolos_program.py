"""YOLOS as a pod-server program (numpy only: the client pod never imports torch).

A pod on a pod-server slice ships its model to the GPU's server as a program
(nos_amd/podserver/program/): this module writes the YOLOS detector of the
reference demo (``demos/gpu-sharing-comparison/client/main.py:14-25``) as that
op graph, with random-init weights drawn by numpy (no network, no
checkpoints).  The graph spells the model out op by op -- patchify,
patch-embedding GEMM, token concat, the bicubic position-embedding
interpolation, 12 pre-LN encoder layers, the final LayerNorm and the two MLP
heads -- and the server's compiler folds and fuses it back onto the same 5
kernels per layer :class:`nos_amd.models.yolos.YolosDetector` runs; the
parameter names are the detector's, so :meth:`YolosDetector.load_numpy`
loads the same weights for parity tests.
"""
from __future__ import annotations

import numpy as np

from ..podserver.program import Builder
from .yolos_config import YolosConfig, demo_input_hw


def yolos_weights(cfg: YolosConfig, seed: int = 0, hw0: tuple[int, int] | None = None) -> dict[str, np.ndarray]:
    """Random-init fp32 weights named like YolosDetector's parameters:
    N(0, initializer_range) matrices and token/position embeddings, and
    LayerNorm scales / biases near 1 / 0 (perturbed, so LN folding and bias
    epilogues are exercised, not multiplied by ones and zeros)."""
    rng = np.random.default_rng(seed)
    std = cfg.initializer_range
    h, m, nd = cfg.hidden_size, cfg.intermediate_size, cfg.num_detection_tokens
    pd = cfg.num_channels * cfg.patch_size ** 2
    gh0, gw0 = (hw0 or cfg.image_size)[0] // cfg.patch_size, (hw0 or cfg.image_size)[1] // cfg.patch_size

    def n(*shape, s=std):
        return (rng.standard_normal(shape, dtype=np.float32) * s).astype(np.float32)

    w = {"patch_w": n(h, pd), "patch_b": n(h), "cls_token": n(1, 1, h), "det_tokens": n(1, nd, h),
         "pos_embed": n(1, 1 + gh0 * gw0 + nd, h)}
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}."
        w.update({p + "ln1_w": 1 + n(h, s=0.1), p + "ln1_b": n(h), p + "qkv_w": n(3 * h, h), p + "qkv_b": n(3 * h),
                  p + "proj_w": n(h, h), p + "proj_b": n(h), p + "ln2_w": 1 + n(h, s=0.1), p + "ln2_b": n(h),
                  p + "fc1_w": n(m, h), p + "fc1_b": n(m), p + "fc2_w": n(h, m), p + "fc2_b": n(h)})
    w["ln_f_w"], w["ln_f_b"] = 1 + n(h, s=0.1), n(h)
    for head, out in (("cls_head", cfg.num_labels + 1), ("box_head", 4)):
        for i, (n_in, n_out) in enumerate(((h, h), (h, h), (h, out))):
            w[f"{head}.{2 * i}"] = n(n_out, n_in)
            w[f"{head}.{2 * i + 1}"] = n(n_out)
    return w


def yolos_program(cfg: YolosConfig, weights: dict[str, np.ndarray], hw: tuple[int, int] | None = None,
                  dtype: str = "fp32", batch: int = 1) -> tuple[dict, bytes]:
    """(program, payload) of YOLOS inference on a ``[batch, 3, *hw]`` fp32
    image; weights and activations in ``dtype`` (fp32: the reference demo's
    precision; bf16)."""
    hw = hw or demo_input_hw()
    b = Builder(f"yolos-h{cfg.hidden_size}-l{cfg.num_hidden_layers}-{dtype}")
    P = {k: b.param(k, v, dtype) for k, v in weights.items()}
    h_, p, nd = cfg.hidden_size, cfg.patch_size, cfg.num_detection_tokens
    C = cfg.num_channels
    gh, gw = hw[0] // p, hw[1] // p
    S0 = weights["pos_embed"].shape[1]
    g0 = S0 - 1 - nd
    gh0 = cfg.image_size[0] // p
    gw0 = g0 // gh0
    eps = cfg.layer_norm_eps

    x = b.input("pixel_values", [batch, C, hw[0], hw[1]], "fp32")
    if dtype != "fp32":
        x = b.op("cast", x, dtype=dtype)
    if hw[0] != gh * p:
        x = b.op("slice", x, dim=2, start=0, end=gh * p)
    if hw[1] != gw * p:
        x = b.op("slice", x, dim=3, start=0, end=gw * p)
    x = b.op("reshape", x, shape=[batch, C, gh, p, gw, p])
    x = b.op("permute", x, dims=[0, 2, 4, 1, 3, 5])
    x = b.op("reshape", x, shape=[batch, gh * gw, C * p * p])
    emb = b.op("linear", x, P["patch_w"], P["patch_b"])
    cls, det = P["cls_token"], P["det_tokens"]
    if batch > 1:
        cls = b.op("expand", cls, shape=[batch, -1, -1])
        det = b.op("expand", det, shape=[batch, -1, -1])
    tok = b.op("cat", cls, emb, det, dim=1)
    # position embeddings interpolated to the input's patch grid (a function
    # of the weights only: the server folds it once at load time)
    pe = b.op("cast", P["pos_embed"], dtype="fp32") if dtype != "fp32" else P["pos_embed"]
    cls_pe = b.op("slice", pe, dim=1, start=0, end=1)
    patch_pe = b.op("slice", pe, dim=1, start=1, end=1 + g0)
    det_pe = b.op("slice", pe, dim=1, start=1 + g0, end=S0)
    pp = b.op("permute", patch_pe, dims=[0, 2, 1])
    pp = b.op("reshape", pp, shape=[1, h_, gh0, gw0])
    pp = b.op("interpolate", pp, size=[gh, gw], mode="bicubic")
    pp = b.op("reshape", pp, shape=[1, h_, gh * gw])
    pp = b.op("permute", pp, dims=[0, 2, 1])
    pos = b.op("cat", cls_pe, pp, det_pe, dim=1)
    if dtype != "fp32":
        pos = b.op("cast", pos, dtype=dtype)
    h = b.op("add", tok, pos)
    for i in range(cfg.num_hidden_layers):
        L = f"layers.{i}."
        y = b.op("layernorm", h, P[L + "ln1_w"], P[L + "ln1_b"], eps=eps)
        qkv = b.op("linear", y, P[L + "qkv_w"], P[L + "qkv_b"])
        a = b.op("attention", qkv, heads=cfg.num_attention_heads)
        h = b.op("add", b.op("linear", a, P[L + "proj_w"], P[L + "proj_b"]), h)
        y = b.op("layernorm", h, P[L + "ln2_w"], P[L + "ln2_b"], eps=eps)
        mm = b.op("gelu", b.op("linear", y, P[L + "fc1_w"], P[L + "fc1_b"]))
        h = b.op("add", b.op("linear", mm, P[L + "fc2_w"], P[L + "fc2_b"]), h)
    S = 1 + gh * gw + nd
    det_h = b.op("slice", h, dim=1, start=S - nd, end=S)
    y = b.op("layernorm", det_h, P["ln_f_w"], P["ln_f_b"], eps=eps)
    outs = []
    for head in ("cls_head", "box_head"):
        z = y
        for i in range(3):
            z = b.op("linear", z, P[f"{head}.{2 * i}"], P[f"{head}.{2 * i + 1}"])
            if i < 2:
                z = b.op("relu", z)
        outs.append(z)
    boxes = b.op("cast", outs[1], dtype="fp32") if dtype != "fp32" else outs[1]
    boxes = b.op("sigmoid", boxes, out="pred_boxes")
    logits = outs[0]
    return b.build([logits, boxes])


def demo_tenant(dtype: str = "fp32", seed: int = 0, small: bool = True,
                hw: tuple[int, int] | None = None) -> tuple[dict, bytes]:
    """The demo pod's program: YOLOS-small at the demo's 800x1066 input
    (``small=False``: the tiny test config at its own 64x96 input)."""
    cfg = YolosConfig.small() if small else YolosConfig.test()
    hw = hw or (demo_input_hw() if small else cfg.image_size)
    return yolos_program(cfg, yolos_weights(cfg, seed), hw, dtype)


__all__ = ["yolos_weights", "yolos_program", "demo_tenant"]
