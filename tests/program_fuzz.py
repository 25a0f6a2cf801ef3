"""Random pod-server programs for property-based tests (hypothesis).

:func:`programs` draws a program the way a tenant could write one -- MLP
chains (linear / norms / activations / residuals / strided slices /
softmax), attention blocks (fused-QKV ``attention`` or ``sdpa`` with causal
masking, grouped-query ratios and rotary), conv nets (grouped, depthwise,
strided, dilated convs, BatchNorm, pooling), activation x activation
``matmul`` and stateful decoders (K / V caches, device positions) -- with dimensions drawn around the kernels' tile edges (1, 31,
33, 127, 129, ...), in fp32 or bf16.  Whatever the validator accepts must run
on the server and agree with the program's eager fp32 reference; whatever it
refuses must be refused before anything is allocated (``ProgramError``).
Numpy only: the programs are built like a pod builds them.
"""
from __future__ import annotations

import math

import numpy as np
from hypothesis import strategies as st

from nos_amd.podserver.program import Builder

EDGE = (1, 2, 31, 33, 63, 65, 127, 129)
WIDTH = (32, 64, 96, 160)
OUT = (1, 3, 31, 33, 64, 96, 127, 129, 160)


class _Builder(Builder):
    def op(self, op: str, *inputs, out=None, **attrs) -> str:   # optional operands given as None are left out
        return super().op(op, *[i for i in inputs if i is not None], out=out, **attrs)


@st.composite
def programs(draw, gpu: bool = True):
    """(program, weights, input array, description)."""
    fam = draw(st.sampled_from(["mlp", "mlp", "attn", "sdpa", "conv", "matmul", "decode"]))
    dt = draw(st.sampled_from(["fp32", "fp32", "bf16"]))
    seed = draw(st.integers(0, 2 ** 16))
    rng = np.random.default_rng(seed)
    b = _Builder(f"fuzz-{fam}-{dt}")
    W = lambda *shape, scale=None: b.param(f"w{len(b.params)}",   # noqa: E731
                                           rng.standard_normal(shape) * (scale if scale is not None else
                                                                         1 / math.sqrt(shape[-1])), dt)
    if fam == "conv":
        N = draw(st.sampled_from((1, 2)))
        C = draw(st.sampled_from((3, 4, 8, 16)))
        H = draw(st.sampled_from((9, 16, 33)))
        Wd = draw(st.sampled_from((8, 17, 31)))
        x = b.input("x", [N, C, H, Wd])
        h = b.op("cast", x, dtype=dt) if dt != "fp32" else x
        c = C
        for _ in range(draw(st.integers(1, 3))):
            k = draw(st.sampled_from((1, 3, 5)))
            groups = draw(st.sampled_from((1, 1, c)))  # dense or depthwise
            oc = c if groups == c else draw(st.sampled_from((8, 32, 33, 64)))
            stride, dil = draw(st.sampled_from((1, 2))), draw(st.sampled_from((1, 1, 2)))
            pad = draw(st.sampled_from((0, k // 2)))
            h = b.op("conv2d", h, W(oc, c // groups, k, k, scale=1 / math.sqrt(c // groups * k * k)),
                     W(oc, scale=0.1), stride=[stride, stride], padding=[pad, pad], dilation=[dil, dil],
                     groups=groups)
            c = oc
            if draw(st.booleans()):
                h = b.op("batchnorm", h, W(c, scale=0.1), W(c, scale=0.1), W(c, scale=0.1),
                         b.param(f"w{len(b.params)}", 1 + rng.random(c), dt), eps=1e-5)
            h = b.op(draw(st.sampled_from(("relu", "gelu", "silu"))), h)
            if draw(st.booleans()):
                op = draw(st.sampled_from(("max_pool2d", "avg_pool2d")))
                h = b.op(op, h, kernel=[2, 2], stride=[2, 2])
        h = b.op("mean", h, dims=[2, 3])
        if draw(st.booleans()):
            n = draw(st.sampled_from(OUT))
            h = b.op("linear", h, W(n, c), W(n, scale=0.1) if draw(st.booleans()) else None)
        data = rng.standard_normal((N, C, H, Wd)).astype(np.float32)
        return (*b.build([h]), data, fam)

    B = draw(st.sampled_from((1, 2)))
    S = draw(st.sampled_from(EDGE))
    D = draw(st.sampled_from(WIDTH))
    x = b.input("x", [B, S, D])
    h = b.op("cast", x, dtype=dt) if dt != "fp32" else x
    data = rng.standard_normal((B, S, D)).astype(np.float32)
    if fam == "attn":   # a fused QKV projection + attention (YOLOS / BERT style), head_dim 64
        heads = draw(st.sampled_from((1, 2, 3)))
        qkv = b.op("linear", h, W(3 * heads * 64, D), W(3 * heads * 64, scale=0.1))
        h = b.op("attention", qkv, heads=heads, causal=draw(st.booleans()))
        h = b.op("linear", h, W(D, heads * 64), None)
        return (*b.build([h]), data, fam)
    if fam == "sdpa":   # decoder attention: grouped-query heads, causal, rotary
        hd = draw(st.sampled_from((64, 128)))
        hkv = draw(st.sampled_from((1, 2)))
        nh = hkv * draw(st.sampled_from((1, 2, 4)))
        q = b.op("reshape", b.op("linear", h, W(nh * hd, D)), shape=[B, S, nh, hd])
        k = b.op("reshape", b.op("linear", h, W(hkv * hd, D)), shape=[B, S, hkv, hd])
        v = b.op("reshape", b.op("linear", h, W(hkv * hd, D)), shape=[B, S, hkv, hd])
        if draw(st.booleans()):
            inv = 1.0 / 10000 ** (np.arange(0, hd, 2) / hd)
            f = np.outer(np.arange(S), inv)
            e = np.concatenate([f, f], 1)
            cs, sn = b.param("cos", np.cos(e), "fp32"), b.param("sin", np.sin(e), "fp32")
            q, k = b.op("rotary", q, cs, sn), b.op("rotary", k, cs, sn)
        o = b.op("sdpa", q, k, v, causal=draw(st.booleans()))
        h = b.op("linear", b.op("reshape", o, shape=[B, S, nh * hd]), W(D, nh * hd))
        return (*b.build([h]), data, fam)
    if fam == "decode":   # stateful: K / V caches + a position counter, written and attended at the positions
        hd = draw(st.sampled_from((64, 128)))
        hkv = draw(st.sampled_from((1, 2)))
        nh = hkv * draw(st.sampled_from((1, 2, 4)))
        L = max(S, draw(st.sampled_from((16, 100, 300))))
        cdt = draw(st.sampled_from(("fp32", "bf16")))
        pos = b.state("pos", [B], "i32")
        kc, vc = b.state("kc", [B, L, hkv, hd], cdt), b.state("vc", [B, L, hkv, hd], cdt)
        q = b.op("reshape", b.op("linear", h, W(nh * hd, D)), shape=[B, S, nh, hd])
        k = b.op("reshape", b.op("linear", h, W(hkv * hd, D)), shape=[B, S, hkv, hd])
        v = b.op("reshape", b.op("linear", h, W(hkv * hd, D)), shape=[B, S, hkv, hd])
        if draw(st.booleans()):
            inv = 1.0 / 10000 ** (np.arange(0, hd, 2) / hd)
            e = np.concatenate([np.outer(np.arange(L), inv)] * 2, 1)
            cs, sn = b.param("cos", np.cos(e), "fp32"), b.param("sin", np.sin(e), "fp32")
            q, k = b.op("rotary_at", q, cs, sn, pos), b.op("rotary_at", k, cs, sn, pos)
        kc2, vc2 = b.op("kv_write", kc, k, pos), b.op("kv_write", vc, v, pos)
        o = b.op("sdpa_cache", q, kc2, vc2, pos)
        h = b.op("linear", b.op("reshape", o, shape=[B, S, nh * hd]), W(D, nh * hd))
        b.op("pos_add", pos, n=S)
        return (*b.build([h]), data, fam)
    if fam == "matmul":   # activation x activation (scores-like), softmax, back through a linear
        a = b.op("linear", h, W(64, D))
        at = b.op("permute", a, dims=[0, 2, 1])
        s_ = b.op("matmul", a, at)                                    # [B, S, S]
        p = b.op("softmax", b.op("mul", s_, b.param("sc", np.full([1], 0.125), dt)))
        h = b.op("matmul", p, a)                                      # [B, S, 64]
        h = b.op(draw(st.sampled_from(("sum", "mean"))), h, dims=[1], keepdim=draw(st.booleans()))
        return (*b.build([h]), data, fam)
    # mlp: a random chain over [B, S, width]
    width = D
    shape = {h: (S, width)}
    for _ in range(draw(st.integers(1, 5))):
        kind = draw(st.sampled_from(("linear", "linear", "norm", "unary", "residual", "slice", "softmax", "scale")))
        if kind == "linear":
            n = draw(st.sampled_from(OUT + (width,)))
            act = draw(st.sampled_from((None, "gelu", "relu")))
            h = b.op("linear", h, W(n, width), W(n, scale=0.1) if draw(st.booleans()) else None, act=act)
            width = n
        elif kind == "norm":
            if draw(st.booleans()):
                h = b.op("layernorm", h, W(width, scale=0.1), W(width, scale=0.1), eps=1e-5)
            else:
                h = b.op("rmsnorm", h, b.param(f"w{len(b.params)}", 1 + 0.1 * rng.standard_normal(width), dt),
                         eps=1e-5)
        elif kind == "unary":
            h = b.op(draw(st.sampled_from(("gelu", "relu", "silu", "sigmoid", "tanh", "neg"))), h)
        elif kind == "residual":
            same = sorted(v for v, sh in shape.items() if sh == (S, width) and v != h)
            if not same:
                continue
            h = b.op("add", h, draw(st.sampled_from(same)))
        elif kind == "slice":
            dim = draw(st.sampled_from((1, 2)))
            n = S if dim == 1 else width
            if n < 2:
                continue
            s0 = draw(st.integers(0, n - 1))
            s1 = draw(st.integers(s0 + 1, n))
            h = b.op("slice", h, dim=dim, start=s0, end=s1)
            if dim == 1:
                S = s1 - s0
            else:
                width = s1 - s0
        elif kind == "softmax":
            h = b.op("softmax", h)
        else:
            h = b.op("mul", h, b.param(f"w{len(b.params)}", 1 + 0.1 * rng.standard_normal(width), dt))
        shape[h] = (S, width)
    if not b.nodes:
        h = b.op("relu", h)
    return (*b.build([h]), data, fam)


def tolerance(dtype: str) -> tuple[float, float]:
    """(relative-to-max, absolute) error an output may have against the fp32
    reference: fp32 programs run at fp32-class precision (h3 / exact
    kernels); bf16 programs round every intermediate to 8 bits."""
    return (2e-3, 1e-4) if dtype == "fp32" else (6e-2, 1e-2)
