"""Decoder-LLM tenants: a ``transformers`` Llama as a pod-server program.

The MPS clients of the reference are arbitrary CUDA programs
(``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:29-34``);
this builder makes the canonical decoder LLM one: a random-init
``LlamaForCausalLM`` (no checkpoints: there is no network) is written as the
program op graph -- token-id input, embedding gather, per layer RMSNorm ->
Q / K / V projections -> rotary -> causal grouped-query attention -> output
projection + residual -> RMSNorm -> SwiGLU MLP + residual, final RMSNorm and
the LM head -- with the module's own weights, so the program's logits are
compared against the HF module's forward (tests/test_llama_tenant.py, GPU:
tests/test_tenant_programs_gpu.py).  On the server the compiler merges the
Q / K / V (and gate / up) projections into one GEMM each, folds every
RMSNorm into the GEMM after it (``linear_rms``), moves the rotary embedding
into the attention (``nos_attn_h3g``: causal, head_dim 128, GQA) and the
residual adds into GEMM epilogues.

The rotary tables are the HF default rope (``rope_theta``, no scaling) for
positions 0..S-1, computed in float64 and stored as fp32 weights.
"""
from __future__ import annotations

import numpy as np

from ..podserver.program import Builder


def llama_config(small: bool = True, **kw):
    """A LlamaConfig: ``small`` -- the fleet tenant (1024 hidden, 8 layers,
    8 heads of 128, 2 KV heads, 2816 MLP, 32000 vocab); else the tests' tiny
    variant.  Keyword arguments override fields."""
    from transformers import LlamaConfig

    base = dict(hidden_size=1024, num_hidden_layers=8, num_attention_heads=8, num_key_value_heads=2,
                intermediate_size=2816, vocab_size=32000, max_position_embeddings=4096, rms_norm_eps=1e-5,
                rope_theta=10000.0, tie_word_embeddings=False) if small else \
        dict(hidden_size=256, num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1,
             intermediate_size=512, vocab_size=512, max_position_embeddings=512, rms_norm_eps=1e-5,
             rope_theta=10000.0, tie_word_embeddings=False)
    base.update(kw)
    return LlamaConfig(**base)


def llama_model(cfg, seed: int = 0):
    """A random-init HF LlamaForCausalLM in fp32, eval mode (eager attention)."""
    import torch
    from transformers import LlamaForCausalLM

    torch.manual_seed(seed)
    cfg._attn_implementation = "eager"
    m = LlamaForCausalLM(cfg).float().eval()
    with torch.no_grad():  # non-trivial norm weights (HF initialises them to ones)
        g = torch.Generator().manual_seed(seed + 1)
        for name, p in m.named_parameters():
            if name.endswith("norm.weight"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g))
    return m


def rope_tables(seq: int, head_dim: int, theta: float) -> tuple[np.ndarray, np.ndarray]:
    inv = 1.0 / theta ** (np.arange(0, head_dim, 2, dtype=np.float64) / head_dim)
    f = np.outer(np.arange(seq, dtype=np.float64), inv)
    emb = np.concatenate([f, f], axis=1)
    return np.cos(emb).astype(np.float32), np.sin(emb).astype(np.float32)


def llama_program(model, seq: int, batch: int = 1, dtype: str = "fp32",
                  rope_len: int | None = None) -> tuple[dict, bytes]:
    """(program, weights) of causal-LM logits [batch, seq, vocab] for token
    ids [batch, seq] (i32).  ``rope_len`` (>= seq): the rotary tables' rows
    in the weights, sliced to ``seq`` in the graph (folded at load) -- the
    programs of several sequence lengths then share one weight payload (the
    pod server's shape variants)."""
    rope_len = seq if rope_len is None else rope_len
    if rope_len < seq:
        raise ValueError(f"rope_len {rope_len} < seq {seq}")
    cfg = model.config
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    d, nh = cfg.hidden_size, cfg.num_attention_heads
    nkv = cfg.num_key_value_heads
    hd = getattr(cfg, "head_dim", None) or d // nh
    eps = float(cfg.rms_norm_eps)
    b = Builder(f"llama-h{d}-l{cfg.num_hidden_layers}-{dtype}")
    ids = b.input("input_ids", [batch, seq], "i32")
    P = lambda k: b.param(k, sd[k], dtype)  # noqa: E731
    cos, sin = rope_tables(rope_len, hd, float(getattr(cfg, "rope_theta", 10000.0)))
    rc, rs = b.param("rope.cos", cos, "fp32"), b.param("rope.sin", sin, "fp32")
    if rope_len > seq:
        rc, rs = (b.op("slice", t, dim=0, start=0, end=seq) for t in (rc, rs))
    h = b.op("embedding", ids, P("model.embed_tokens.weight"))
    for i in range(cfg.num_hidden_layers):
        p = f"model.layers.{i}."
        y = b.op("rmsnorm", h, P(p + "input_layernorm.weight"), eps=eps)
        q = b.op("reshape", b.op("linear", y, P(p + "self_attn.q_proj.weight")), shape=[batch, seq, nh, hd])
        k = b.op("reshape", b.op("linear", y, P(p + "self_attn.k_proj.weight")), shape=[batch, seq, nkv, hd])
        v = b.op("reshape", b.op("linear", y, P(p + "self_attn.v_proj.weight")), shape=[batch, seq, nkv, hd])
        q, k = b.op("rotary", q, rc, rs), b.op("rotary", k, rc, rs)
        o = b.op("reshape", b.op("sdpa", q, k, v, causal=True), shape=[batch, seq, nh * hd])
        h = b.op("add", b.op("linear", o, P(p + "self_attn.o_proj.weight")), h)
        y = b.op("rmsnorm", h, P(p + "post_attention_layernorm.weight"), eps=eps)
        g = b.op("linear", y, P(p + "mlp.gate_proj.weight"))
        u = b.op("linear", y, P(p + "mlp.up_proj.weight"))
        h = b.op("add", b.op("linear", b.op("mul", b.op("silu", g), u), P(p + "mlp.down_proj.weight")), h)
    h = b.op("rmsnorm", h, P("model.norm.weight"), eps=eps)
    head = "lm_head.weight" if "lm_head.weight" in sd else "model.embed_tokens.weight"
    logits = b.op("linear", h, P(head), out="logits")
    return b.build([logits])


def llama_decode_programs(model, prompt_len: int, max_len: int, batch: int = 1, dtype: str = "fp32",
                          extend: tuple[int, ...] = ()) -> tuple[list[dict], bytes]:
    """A STATEFUL generation tenant: ``[prefill, decode, *extends]`` programs
    over one weight payload and one state -- per layer a K and a V cache
    ``[batch, max_len, kv_heads, head_dim]`` plus the position counter
    ``pos`` [batch] (i32) -- registered as shape variants (the server routes
    by the input's shape):

    * prefill, input ids ``[batch, prompt_len]``: starts a sequence
      (``pos_set`` 0), writes the prompt's K / V into the caches, attends
      causally (the compiler sees position 0 and runs the flash kernel on the
      fresh keys), advances ``pos`` by ``prompt_len``;
    * decode, input ids ``[batch, 1]``: one token at the device-side position
      -- rotary at ``pos``, ``kv_write`` of its K / V, ``sdpa_cache`` over the
      cache (decode.hip), ``pos`` += 1;
    * ``extend`` lengths: like decode for chunks of that many tokens (a longer
      prompt = prefill + extends + decode steps).

    Every program outputs the last token's logits ``[batch, 1, vocab]`` and
    the greedy next ids ``[batch, 1]`` (i32, ``argmax``), so a client's
    generation loop sends back one id per step.  The caches' bytes count
    against the slice at registration; a replay never allocates state."""
    if not 0 < prompt_len <= max_len:
        raise ValueError(f"prompt_len must be in [1, {max_len}]")
    cfg = model.config
    sd = {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}
    d, nh = cfg.hidden_size, cfg.num_attention_heads
    nkv = cfg.num_key_value_heads
    hd = getattr(cfg, "head_dim", None) or d // nh
    eps = float(cfg.rms_norm_eps)
    cos, sin = rope_tables(max_len, hd, float(getattr(cfg, "rope_theta", 10000.0)))
    head = "lm_head.weight" if "lm_head.weight" in sd else "model.embed_tokens.weight"
    cache_dt = "bf16" if dtype == "bf16" else "fp32"
    progs = []
    chunks = [(prompt_len, True), (1, False)] + [(n, False) for n in extend]
    weights = b""
    for seq, reset in chunks:
        b = Builder(f"llama-h{d}-l{cfg.num_hidden_layers}-{dtype}-{'prefill' if reset else 'step'}{seq}")
        ids = b.input("input_ids", [batch, seq], "i32")
        P = lambda k: b.param(k, sd[k], dtype)  # noqa: E731
        rc, rs = b.param("rope.cos", cos, "fp32"), b.param("rope.sin", sin, "fp32")
        b.state("pos", [batch], "i32")
        caches = [(b.state(f"kc{i}", [batch, max_len, nkv, hd], cache_dt),
                   b.state(f"vc{i}", [batch, max_len, nkv, hd], cache_dt)) for i in range(cfg.num_hidden_layers)]
        p = b.op("pos_set", "pos", value=0) if reset else "pos"
        h = b.op("embedding", ids, P("model.embed_tokens.weight"))
        for i in range(cfg.num_hidden_layers):
            pf = f"model.layers.{i}."
            y = b.op("rmsnorm", h, P(pf + "input_layernorm.weight"), eps=eps)
            q = b.op("reshape", b.op("linear", y, P(pf + "self_attn.q_proj.weight")), shape=[batch, seq, nh, hd])
            k = b.op("reshape", b.op("linear", y, P(pf + "self_attn.k_proj.weight")), shape=[batch, seq, nkv, hd])
            v = b.op("reshape", b.op("linear", y, P(pf + "self_attn.v_proj.weight")), shape=[batch, seq, nkv, hd])
            q, k = b.op("rotary_at", q, rc, rs, p), b.op("rotary_at", k, rc, rs, p)
            kc = b.op("kv_write", caches[i][0], k, p)
            vc = b.op("kv_write", caches[i][1], v, p)
            o = b.op("reshape", b.op("sdpa_cache", q, kc, vc, p), shape=[batch, seq, nh * hd])
            h = b.op("add", b.op("linear", o, P(pf + "self_attn.o_proj.weight")), h)
            y = b.op("rmsnorm", h, P(pf + "post_attention_layernorm.weight"), eps=eps)
            g = b.op("linear", y, P(pf + "mlp.gate_proj.weight"))
            u = b.op("linear", y, P(pf + "mlp.up_proj.weight"))
            h = b.op("add", b.op("linear", b.op("mul", b.op("silu", g), u), P(pf + "mlp.down_proj.weight")), h)
        if seq > 1:   # only the last token's logits: the LM head runs on one row
            h = b.op("slice", h, dim=1, start=seq - 1, end=seq)
        h = b.op("rmsnorm", h, P("model.norm.weight"), eps=eps)
        logits = b.op("linear", h, P(head), out="logits")
        nxt = b.op("argmax", logits, out="next_ids")
        b.op("pos_add", p, n=seq)
        prog, w = b.build([logits, nxt])
        progs.append(prog)
        weights = w
    return progs, weights


def llama_tenant(dtype: str = "fp32", seed: int = 0, small: bool = True, seq: int = 512,
                 batch: int = 1) -> tuple[dict, bytes]:
    """(program, weights) of the decoder-LLM tenant (``small=False``: the
    tiny test config at seq 64)."""
    m = llama_model(llama_config(small), seed)
    return llama_program(m, seq if small else 64, batch, dtype)


__all__ = ["llama_config", "llama_model", "llama_program", "llama_decode_programs", "llama_tenant", "rope_tables"]
