"""Tenant programs: what a fractional pod ships to the pod server.

MPS runs any CUDA client program in the server's context
(``/root/reference/docs/en/docs/dynamic-gpu-partitioning/partitioning-modes-comparison.md:34-35``,
``getting-started-mps.md:22-55``).  The MI355X pod server (server.py) cannot
run foreign machine code safely in its one HIP context, so a tenant ships a
*program* instead: a static op graph over a whitelisted set of nos-amd ops
plus its weights as raw tensor bytes.  Nothing in it is executable -- no
pickle, no code -- and every op lowers onto the gfx950 kernels of
``libnos_hip.so`` (``nos_amd.ops``), so native kernels run by construction.

Wire form (JSON object; the weights travel as the message payload)::

    {"format": "nos-amd.program/v1", "name": "yolos-small",
     "inputs":  [{"name": "x", "shape": [1, 3, 800, 1066], "dtype": "fp32"}],
     "params":  [{"name": "w0", "shape": [384, 768], "dtype": "fp32", "offset": 0, "nbytes": 1179648}, ...],
     "nodes":   [{"op": "linear", "inputs": ["x", "w0", "b0"], "output": "h0", "attrs": {"act": "gelu"}}, ...],
     "outputs": ["logits", "boxes"]}

Values are SSA names; nodes are listed in execution order.  Wire dtypes are
``fp32`` (IEEE float32, little endian) and ``bf16`` (the upper 16 bits of a
float32, little-endian uint16).

:func:`parse` validates a program completely before anything is allocated:
the op whitelist, every attribute, the topological order and the exact shape
and dtype of every value (shape inference), the native kernels' constraints
on a GPU (head_dim 64, K % 64 for bf16 GEMMs, ...), the payload layout, and
an upper bound of the device bytes it needs (:attr:`Program.bytes_estimate`)
that the server checks against the tenant's slice before building.

:meth:`Program.compile` is a small graph compiler:

1. **constant folding** -- every node whose inputs are all weights runs once
   at load time on the device (e.g. YOLOS's bicubic position-embedding
   interpolation), its result becomes a weight;
2. **LayerNorm folding** -- ``layernorm -> linear`` becomes one
   ``linear_ln`` GEMM (the norm folded into the weight,
   :func:`nos_amd.ops.fold_layernorm`, statistics in the GEMM prologue);
3. **epilogue fusion** -- an activation (``gelu``/``relu``) and then a
   residual ``add`` after a GEMM go into its epilogue;
4. **QKV-attention fusion** -- ``linear_ln`` producing a fused QKV consumed
   only by ``attention`` becomes one node that, for fp32 tenants under the
   bf16x6 math, writes K/V straight into the attention's bf16 planes
   (``nos_gemm_ln_f32x6_qkv`` + ``nos_attn_fwd_f32x6_presplit_d64``);
5. **dead-value elimination and last-use release**: intermediates are
   dropped after their last consumer, so a HIP graph captured from the
   compiled program reuses their memory.

Later passes (round 4-5), each trimming launches or memory round trips (the
full order is in :class:`CompiledProgram`; ``NOS_AMD_SKIP_PASSES=name,...``
leaves the switchable ones out for A/B runs): ``add`` over ``cat``
distribution (position embeddings become the patch GEMM's residual), ViT
patch extraction as one strided im2col (``patchify``; bf16: the cast folded
in), cast + reshape / permute chains as one ``relayout``, row-slice
pushdown (YOLOS's last layer on its detection tokens only), BatchNorm
folding, parallel linears merged (Q / K / V, gate / up, the detection heads'
first layers), small linears over adjacent column slices merged into
block-diagonal GEMMs (``blockdiag``), RMSNorm folding, cast + activation as
one ``unary`` pass (``cast_unary``), rotary fused into ``sdpa``, a cat
written in place by its GEMM (``cat_buffer``), fp16-plane and LayerNorm
hand-offs between h3 kernels (``cat_stats``: layer 0's statistics from the
patch GEMM plus build-time constant rows), conv weight preparation.

The compiled program is a callable ``(x) -> tuple(outputs)``, captured into a
HIP graph by the server exactly like a built-in model.  :meth:`Program.reference`
runs the unfused graph eagerly in fp32 (the numerics reference of tests).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

FORMAT = "nos-amd.program/v1"
WIRE_DTYPES = {"fp32": 4, "bf16": 2, "i32": 4}   # i32: token ids (an input only; consumed by embedding)
FLOAT_DTYPES = ("fp32", "bf16")
MAX_NODES = 8192
MAX_PARAMS = 8192
MAX_NUMEL = 1 << 31          # elements of one value
MAX_RANK = 8
MAX_VARIANTS = 8             # input shapes one tenant may register (parse_variants)
UNARY = ("gelu", "relu", "sigmoid", "silu", "tanh", "exp", "neg", "rsqrt")
BINARY = ("add", "mul", "sub", "div")
ACTS = (None, "gelu", "relu")
INTERP_MODES = ("bicubic", "bilinear", "nearest")


class ProgramError(ValueError):
    """The program is malformed or uses something the server does not run."""


@dataclass(frozen=True)
class Value:
    name: str
    shape: tuple[int, ...]
    dtype: str
    kind: str                 # "input" | "param" | "node"

    @property
    def numel(self) -> int:
        return math.prod(self.shape)

    @property
    def nbytes(self) -> int:
        return self.numel * WIRE_DTYPES[self.dtype]


@dataclass
class Node:
    op: str
    inputs: list[str]
    output: str
    attrs: dict = field(default_factory=dict)


# ---------------------------------------------------------------- validation
def _req(cond: bool, msg: str) -> None:
    if not cond:
        raise ProgramError(msg)


def _int(v, what: str, lo: int | None = None) -> int:
    _req(isinstance(v, int) and not isinstance(v, bool), f"{what} must be an integer, got {v!r}")
    if lo is not None:
        _req(v >= lo, f"{what} must be >= {lo}, got {v}")
    return v


def _dim(d, what: str) -> int:
    """One dimension: an int in [1, MAX_NUMEL] (products are then taken on
    Python ints, which cannot wrap)."""
    d = _int(d, what, 1)
    _req(d <= MAX_NUMEL, f"{what} {d} is over {MAX_NUMEL}")
    return d


def _shape(v, what: str) -> tuple[int, ...]:
    _req(isinstance(v, list) and len(v) <= MAX_RANK, f"{what} must be a list of at most {MAX_RANK} dims")
    s = tuple(_dim(d, f"{what} dim") for d in v)
    _req(math.prod(s) <= MAX_NUMEL, f"{what} has more than {MAX_NUMEL} elements")
    return s


def _name(v, what: str) -> str:
    _req(isinstance(v, str) and 0 < len(v) <= 128, f"{what} must be a non-empty string of <= 128 chars")
    return v


def _broadcast(a: tuple, b: tuple, what: str) -> tuple:
    n = max(len(a), len(b))
    a2, b2 = (1,) * (n - len(a)) + a, (1,) * (n - len(b)) + b
    out = []
    for x, y in zip(a2, b2):
        _req(x == y or x == 1 or y == 1, f"{what}: shapes {a} and {b} do not broadcast")
        out.append(max(x, y))
    return tuple(out)


def _infer(node: Node, ins: list[Value], gpu: bool) -> tuple[tuple[int, ...], str]:
    """Output (shape, dtype) of a node; raises ProgramError on any mismatch,
    including the native kernels' constraints when the program runs on a GPU."""
    op, a = node.op, node.attrs
    what = f"node {node.output!r} ({op})"

    def arity(lo: int, hi: int) -> None:
        _req(lo <= len(ins) <= hi, f"{what}: takes {lo}..{hi} inputs, got {len(ins)}")

    def same_dtype() -> str:
        _req(len({v.dtype for v in ins}) == 1, f"{what}: inputs must share one dtype, got {[v.dtype for v in ins]}")
        return ins[0].dtype

    def only(*keys: str) -> None:
        extra = set(a) - set(keys)
        _req(not extra, f"{what}: unknown attributes {sorted(extra)}")

    if op == "linear":
        only("act")
        arity(2, 3)
        dt = same_dtype()
        x, w = ins[0], ins[1]
        _req(len(w.shape) == 2 and len(x.shape) >= 1 and x.shape[-1] == w.shape[1] and dt in FLOAT_DTYPES,
             f"{what}: float x [..., K] and weight [N, K] required, got {x.shape} and {w.shape}")
        if len(ins) == 3:
            _req(ins[2].shape == (w.shape[0],), f"{what}: bias must be [{w.shape[0]}], got {ins[2].shape}")
        _req(a.get("act") in ACTS, f"{what}: act must be one of {ACTS}")
        if gpu:
            k_mult = 64 if dt == "bf16" else 32
            _req(x.shape[-1] % k_mult == 0, f"{what}: the {dt} GEMM kernels need K % {k_mult} == 0, K = {x.shape[-1]}")
        return x.shape[:-1] + (w.shape[0],), dt
    if op == "layernorm":
        only("eps")
        arity(3, 3)
        dt = same_dtype()
        d = ins[0].shape[-1] if ins[0].shape else 0
        _req(ins[1].shape == (d,) and ins[2].shape == (d,) and dt in FLOAT_DTYPES, f"{what}: gamma/beta must be [{d}]")
        eps = a.get("eps", 1e-5)
        _req(isinstance(eps, (int, float)) and 0 < eps < 1, f"{what}: eps must be in (0, 1)")
        return ins[0].shape, dt
    if op == "attention":
        only("heads", "scale", "causal")
        arity(1, 1)
        x = ins[0]
        h = _int(a.get("heads"), f"{what}: heads", 1)
        _req(len(x.shape) == 3 and x.shape[2] % (3 * h) == 0 and x.dtype in FLOAT_DTYPES,
             f"{what}: qkv must be a float [B, S, 3*heads*D], got {x.shape} with {h} heads")
        d = x.shape[2] // (3 * h)
        if "scale" in a:
            _req(isinstance(a["scale"], (int, float)) and a["scale"] > 0, f"{what}: scale must be > 0")
        _req(isinstance(a.get("causal", False), bool), f"{what}: causal must be a bool")
        if gpu:
            _req(d in (64, 128), f"{what}: the attention kernels take head_dim 64 or 128, got {d}")
        return (x.shape[0], x.shape[1], h * d), x.dtype
    if op in BINARY:
        only()
        arity(2, 2)
        dt = same_dtype()
        _req(dt in FLOAT_DTYPES, f"{what}: takes float tensors")
        return _broadcast(ins[0].shape, ins[1].shape, what), dt
    if op in UNARY:
        only()
        arity(1, 1)
        _req(ins[0].dtype in FLOAT_DTYPES, f"{what}: takes a float tensor")
        return ins[0].shape, ins[0].dtype
    if op == "cat":
        only("dim")
        arity(1, 64)
        dt = same_dtype()
        r = len(ins[0].shape)
        dim = _int(a.get("dim"), f"{what}: dim")
        dim = dim + r if dim < 0 else dim
        _req(0 <= dim < r, f"{what}: dim out of range")
        for v in ins[1:]:
            _req(len(v.shape) == r and all(v.shape[i] == ins[0].shape[i] for i in range(r) if i != dim),
                 f"{what}: shapes {[v.shape for v in ins]} differ outside dim {dim}")
        s = list(ins[0].shape)
        s[dim] = sum(v.shape[dim] for v in ins)
        return tuple(s), dt
    if op == "slice":
        only("dim", "start", "end")
        arity(1, 1)
        s = list(ins[0].shape)
        dim = _int(a.get("dim"), f"{what}: dim")
        dim = dim + len(s) if dim < 0 else dim
        _req(0 <= dim < len(s), f"{what}: dim out of range")
        start, end = _int(a.get("start"), f"{what}: start", 0), _int(a.get("end"), f"{what}: end", 1)
        _req(start < end <= s[dim], f"{what}: need 0 <= start < end <= {s[dim]}, got {start}:{end}")
        s[dim] = end - start
        return tuple(s), ins[0].dtype
    if op == "reshape":
        only("shape")
        arity(1, 1)
        want = a.get("shape")
        _req(isinstance(want, list) and len(want) <= MAX_RANK and all(isinstance(d, int) for d in want),
             f"{what}: shape must be a list of integers")
        _req(sum(1 for d in want if d == -1) <= 1 and all(d == -1 or d >= 1 for d in want),
             f"{what}: shape dims must be >= 1, at most one -1")
        _req(all(d <= MAX_NUMEL for d in want), f"{what}: shape dims must be <= {MAX_NUMEL}")
        n = ins[0].numel
        known = math.prod(d for d in want if d != -1)
        if -1 in want:
            _req(known > 0 and n % known == 0, f"{what}: cannot reshape {ins[0].shape} to {want}")
            want = [n // known if d == -1 else d for d in want]
        _req(math.prod(want) == n, f"{what}: cannot reshape {ins[0].shape} to {want}")
        return tuple(want), ins[0].dtype
    if op == "permute":
        only("dims")
        arity(1, 1)
        dims = a.get("dims")
        _req(isinstance(dims, list) and all(isinstance(d, int) and not isinstance(d, bool) for d in dims)
             and sorted(dims) == list(range(len(ins[0].shape))),
             f"{what}: dims must be a permutation of 0..{len(ins[0].shape) - 1}")
        return tuple(ins[0].shape[d] for d in dims), ins[0].dtype
    if op == "expand":
        only("shape")
        arity(1, 1)
        want = a.get("shape")
        s = ins[0].shape
        _req(isinstance(want, list) and len(want) == len(s), f"{what}: shape must have rank {len(s)}")
        out = []
        for src, d in zip(s, want):
            _req(isinstance(d, int) and (d == -1 or d == src or (src == 1 and 1 <= d <= MAX_NUMEL)),
                 f"{what}: cannot expand {s} to {want}")
            out.append(src if d == -1 else d)
        return tuple(out), ins[0].dtype
    if op == "cast":
        only("dtype")
        arity(1, 1)
        _req(a.get("dtype") in FLOAT_DTYPES and ins[0].dtype in FLOAT_DTYPES,
             f"{what}: casts between {FLOAT_DTYPES} only")
        return ins[0].shape, a["dtype"]
    if op == "interpolate":
        only("size", "mode")
        arity(1, 1)
        x = ins[0]
        _req(len(x.shape) == 4 and x.dtype == "fp32", f"{what}: takes an fp32 [N, C, H, W] tensor")
        size = a.get("size")
        _req(isinstance(size, list) and len(size) == 2 and all(isinstance(d, int) and 1 <= d <= 65536 for d in size),
             f"{what}: size must be [H, W]")
        _req(a.get("mode", "bicubic") in INTERP_MODES, f"{what}: mode must be one of {INTERP_MODES}")
        return (x.shape[0], x.shape[1], size[0], size[1]), x.dtype
    if op == "conv2d":
        only("stride", "padding", "dilation", "groups")
        arity(2, 3)
        dt = same_dtype()
        x, w = ins[0], ins[1]
        g = a.get("groups", 1)
        _req(isinstance(g, int) and not isinstance(g, bool) and 1 <= g <= 65536, f"{what}: groups must be an int >= 1")
        _req(len(x.shape) == 4 and len(w.shape) == 4 and x.shape[1] == w.shape[1] * g and w.shape[0] % g == 0,
             f"{what}: x [N, C, H, W] and weight [OC, C / groups, KH, KW] (OC % groups == 0) required, got "
             f"{x.shape} and {w.shape} for groups = {g}")
        if len(ins) == 3:
            _req(ins[2].shape == (w.shape[0],), f"{what}: bias must be [{w.shape[0]}]")
        st = _pair(a.get("stride", [1, 1]), f"{what}: stride", 1)
        pd = _pair(a.get("padding", [0, 0]), f"{what}: padding", 0)
        dl = _pair(a.get("dilation", [1, 1]), f"{what}: dilation", 1)
        oh = (x.shape[2] + 2 * pd[0] - dl[0] * (w.shape[2] - 1) - 1) // st[0] + 1
        ow = (x.shape[3] + 2 * pd[1] - dl[1] * (w.shape[3] - 1) - 1) // st[1] + 1
        _req(oh >= 1 and ow >= 1, f"{what}: empty output for input {x.shape}")
        return (x.shape[0], w.shape[0], oh, ow), dt
    if op == "batchnorm":
        only("eps")
        arity(5, 5)
        dt = same_dtype()
        x = ins[0]
        _req(len(x.shape) >= 2 and all(v.shape == (x.shape[1],) for v in ins[1:]),
             f"{what}: x [N, C, ...] and gamma / beta / mean / var [C] required")
        _eps(a, what)
        return x.shape, dt
    if op in ("max_pool2d", "avg_pool2d"):
        only("kernel", "stride", "padding")
        arity(1, 1)
        x = ins[0]
        _req(len(x.shape) == 4 and x.dtype in FLOAT_DTYPES, f"{what}: takes a float [N, C, H, W] tensor")
        k = _pair(a.get("kernel"), f"{what}: kernel", 1)
        st = _pair(a.get("stride", list(k)), f"{what}: stride", 1)
        pd = _pair(a.get("padding", [0, 0]), f"{what}: padding", 0)
        _req(pd[0] <= k[0] // 2 and pd[1] <= k[1] // 2, f"{what}: padding must be <= kernel / 2")
        oh, ow = (x.shape[2] + 2 * pd[0] - k[0]) // st[0] + 1, (x.shape[3] + 2 * pd[1] - k[1]) // st[1] + 1
        _req(oh >= 1 and ow >= 1, f"{what}: empty output")
        return (x.shape[0], x.shape[1], oh, ow), x.dtype
    if op in ("mean", "sum"):
        only("dims", "keepdim")
        arity(1, 1)
        x = ins[0]
        r = len(x.shape)
        dims = a.get("dims")
        _req(isinstance(dims, list) and dims and all(isinstance(d, int) and not isinstance(d, bool) and -r <= d < r
                                                      for d in dims), f"{what}: dims must be a list of axes")
        dd = sorted({d % r for d in dims})
        keep = a.get("keepdim", False)
        _req(isinstance(keep, bool), f"{what}: keepdim must be a bool")
        _req(x.dtype in FLOAT_DTYPES, f"{what}: takes a float tensor")
        return tuple((1 if i in dd else n) for i, n in enumerate(x.shape) if keep or i not in dd), x.dtype
    if op == "matmul":
        only()
        arity(2, 2)
        dt = same_dtype()
        x, y = ins
        _req(len(x.shape) >= 2 and len(y.shape) >= 2 and x.shape[-1] == y.shape[-2],
             f"{what}: [..., M, K] @ [..., K, N] required, got {x.shape} and {y.shape}")
        bx, by = x.shape[:-2], y.shape[:-2]
        _req(not bx or not by or bx == by, f"{what}: batch dims must match or one side be 2-D")
        return (bx or by) + (x.shape[-2], y.shape[-1]), dt
    if op == "softmax":
        only("dim")
        arity(1, 1)
        _req(a.get("dim", -1) in (-1, len(ins[0].shape) - 1), f"{what}: softmax runs over the last dim")
        _req(ins[0].dtype in FLOAT_DTYPES, f"{what}: takes a float tensor")
        return ins[0].shape, ins[0].dtype
    if op == "embedding":
        only()
        arity(2, 2)
        ids, table = ins
        _req(ids.dtype == "i32", f"{what}: ids must be i32, got {ids.dtype}")
        _req(len(table.shape) == 2 and table.dtype in FLOAT_DTYPES, f"{what}: table must be a float [V, D]")
        if gpu:
            _req(table.shape[1] * WIRE_DTYPES[table.dtype] % 16 == 0, f"{what}: table rows must be 16-byte multiples")
        return ids.shape + (table.shape[1],), table.dtype
    if op == "rmsnorm":
        only("eps")
        arity(2, 2)
        dt = same_dtype()
        _req(len(ins[0].shape) >= 1 and ins[1].shape == (ins[0].shape[-1],), f"{what}: weight must be [D]")
        _eps(a, what)
        return ins[0].shape, dt
    if op == "rotary":
        only()
        arity(3, 3)
        x, c, sn = ins
        _req(len(x.shape) == 4 and x.shape[3] % 2 == 0 and x.dtype in FLOAT_DTYPES,
             f"{what}: x must be [B, S, H, D] with D even")
        _req(c.shape == sn.shape == (x.shape[1], x.shape[3]) and c.dtype == sn.dtype == "fp32",
             f"{what}: cos / sin must be fp32 [S, D] = [{x.shape[1]}, {x.shape[3]}]")
        return x.shape, x.dtype
    if op == "sdpa":
        only("causal", "scale")
        arity(3, 3)
        dt = same_dtype()
        q, k, v = ins
        _req(len(q.shape) == 4 and len(k.shape) == 4 and k.shape == v.shape and q.shape[0] == k.shape[0]
             and q.shape[3] == k.shape[3] and q.shape[2] % k.shape[2] == 0,
             f"{what}: q [B, Sq, H, D], k / v [B, Skv, Hkv, D] with H % Hkv == 0 required, got {q.shape}, {k.shape}")
        _req(isinstance(a.get("causal", False), bool), f"{what}: causal must be a bool")
        if a.get("causal"):
            _req(q.shape[1] <= k.shape[1], f"{what}: causal attention needs Sq <= Skv")
        if "scale" in a:
            _req(isinstance(a["scale"], (int, float)) and a["scale"] > 0, f"{what}: scale must be > 0")
        if gpu:
            _req(q.shape[3] in (64, 128), f"{what}: the attention kernels take head_dim 64 or 128, got {q.shape[3]}")
        return q.shape, dt
    raise ProgramError(f"{what}: op {op!r} is not one the pod server runs (whitelist: {' '.join(OPS)})")


def _pair(v, what: str, lo: int) -> tuple[int, int]:
    if isinstance(v, int) and not isinstance(v, bool):
        v = [v, v]
    _req(isinstance(v, list) and len(v) == 2, f"{what} must be an int or [h, w]")
    return (_int(v[0], what, lo), _int(v[1], what, lo))


def _eps(a: dict, what: str) -> None:
    eps = a.get("eps", 1e-5)
    _req(isinstance(eps, (int, float)) and not isinstance(eps, bool) and 0 < eps < 1, f"{what}: eps must be in (0, 1)")


OPS = ("linear", "layernorm", "attention", *BINARY, *UNARY, "cat", "slice", "reshape", "permute", "expand",
       "cast", "interpolate",
       # general tenants: conv nets and decoder LLMs (nos_amd/ops/tenant.py)
       "conv2d", "batchnorm", "max_pool2d", "avg_pool2d", "mean", "sum", "matmul", "softmax", "embedding",
       "rmsnorm", "rotary", "sdpa")
NEVER_FOLD = ("attention", "sdpa")
# step kinds that run a gfx950 kernel of libnos_hip.so (CompiledProgram.stats["kernels"])
NATIVE_KINDS = ("linear", "linear_ln", "linear_rms", "ln_qkv_attention", "attention", "layernorm", "conv2d", "matmul",
                "softmax", "embedding", "rmsnorm", "rotary", "sdpa", "patches", "unary")
GEMM_OPS = ("linear", "conv2d")


def _workspace(node: Node, ins: list[Value], out: Value, f32_math: str) -> int:
    """Transient device bytes one op allocates while it runs, beyond its
    inputs and output (an upper bound; :meth:`Program.bytes_estimate_for`)."""
    op = node.op
    if op == "linear" and ins[0].dtype == "fp32" and f32_math == "h3":
        m = ins[0].numel // ins[0].shape[-1]
        return ins[0].nbytes + 4 * m                       # A's fp16 planes + row scales
    if op == "linear_rms" or (op == "linear" and ins[0].dtype == "bf16" and f32_math == "h3"):
        m = ins[0].numel // ins[0].shape[-1]
        return 2 * m * ins[0].shape[-1] * 4 + 4 * m + out.numel * 4
    if op == "attention":
        b, s, three_hd = ins[0].shape
        h = node.attrs["heads"]
        return _attn_ws(b, s, s, h, h, three_hd // (3 * h)) + ins[0].nbytes + out.numel * 4
    if op == "sdpa":
        (b, sq, h, d), (_, skv, hkv, _) = ins[0].shape, ins[1].shape
        copies = sum(v.numel * 4 for v in ins[:3]) if ins[0].dtype != "fp32" else 0
        return _attn_ws(b, sq, skv, h, hkv, d) + copies + out.numel * 4
    if op == "conv2d":
        n, c, _, _ = ins[0].shape
        oc, cg, kh, kw = ins[1].shape
        p = out.numel // (n * oc)
        kp = -(-(cg * kh * kw) // 32) * 32
        return n * (c // cg) * p * (kp * 4 + 4) + ins[0].numel * 4 + out.numel * 4
    if op == "matmul":
        k = ins[0].shape[-1]
        kp = -(-k // 32) * 32
        rows = ins[0].numel // k + ins[1].numel // k
        return rows * kp * 12 + out.numel * 4          # padded fp32 copies + planes + the fp32 result
    return 0


def _attn_ws(b: int, sq: int, skv: int, h: int, hkv: int, d: int) -> int:
    """Upper bound of both attention kernels' workspaces (attention_f32x.hip
    nos_attn_f32x6_workspace, attention_h3g.hip nos_attn_h3g_workspace)."""
    skvp = -(-skv // 32) * 32
    return b * max(h, hkv) * skvp * 6 * d * 2 + 4 * b * sq * h * (d + 2) * 4 + b * hkv * (skv // 256 + 2) * 8 + 4096


@dataclass
class Program:
    name: str
    inputs: list[Value]
    params: dict[str, Value]
    param_layout: dict[str, tuple[int, int]]     # name -> (offset, nbytes) in the payload
    nodes: list[Node]
    outputs: list[str]
    values: dict[str, Value]
    payload: bytes | memoryview = b""

    # ------------------------------------------------------------ accounting
    @property
    def param_bytes(self) -> int:
        return sum(v.nbytes for v in self.params.values())

    @property
    def bytes_estimate(self) -> int:
        return self.bytes_estimate_for(None)

    def foldable(self) -> set[str]:
        """Node outputs the compiler folds to constants at load time (every
        input a weight or another folded value; never attention)."""
        const = set(self.params)
        out = set()
        for n in self.nodes:
            if n.op not in NEVER_FOLD and all(i in const for i in n.inputs):
                const.add(n.output)
                out.add(n.output)
        return out

    def bytes_estimate_for(self, kernel_config: dict | None = None) -> int:
        """Device bytes a build needs, bounded before anything is allocated:

        * the weights, plus their split planes under the server's fp32 math
          (``kernel_config["f32_math"]``; h3: two fp16 planes = 1x an fp32
          matrix + row scales; x6: three bf16 planes = 1.5x; exact: none) and
          the folded copy LayerNorm / RMSNorm folding makes of a weight
          (+ its two bias vectors);
        * constant-folded values, which are weights too: they are counted as
          persistent (they are materialised at load time and live
          for the tenant's lifetime), never released;
        * the input, and the peak of the unfused graph's live activations
          when every value is released after its last consumer (what the
          compiled program does; fusion only removes intermediates) plus the
          largest per-op workspace live at that point (GEMM A planes, the
          attention's K/V planes, conv im2col planes, ...; :func:`_workspace`),
          twice over: one graph plus the solo graph's private buffers.

        The measured peak of the real build is checked again after it."""
        f32_math = (kernel_config or {}).get("f32_math", "h3")
        folded = self.foldable()
        persistent = sum(self.values[o].nbytes for o in folded)
        last = {}
        for k, n in enumerate(self.nodes):
            for i in n.inputs:
                last[i] = k
        keep = set(self.outputs)
        live = peak = 0
        for k, n in enumerate(self.nodes):
            if n.output in folded:
                continue
            ws = _workspace(n, [self.values[i] for i in n.inputs], self.values[n.output], f32_math)
            live += self.values[n.output].nbytes
            peak = max(peak, live + ws)
            for i in set(n.inputs):
                v = self.values[i]
                if v.kind == "node" and i not in folded and last.get(i) == k and i not in keep:
                    live -= v.nbytes
        plane_mult = {"h3": 1.0, "x6": 1.5}.get(f32_math, 0.0)
        planes = 0
        by_out = {n.output: n for n in self.nodes}
        for n in self.nodes:
            if n.op not in GEMM_OPS or len(n.inputs) < 2 or n.inputs[1] not in self.params:
                continue
            w = self.values[n.inputs[1]]
            if w.dtype == "fp32":
                planes += int(w.nbytes * plane_mult) + 4 * w.shape[0]
            src = by_out.get(n.inputs[0])
            if src is not None and src.op in ("layernorm", "rmsnorm"):  # the folded copy + c1 / c2
                planes += w.nbytes + 8 * w.shape[0]
        return self.param_bytes + planes + persistent + sum(v.nbytes for v in self.inputs) + 2 * peak

    # ------------------------------------------------------------ tensors
    def tensors(self, device) -> dict:
        """The weights as device tensors (copied out of the payload)."""
        import torch

        out = {}
        buf = memoryview(self.payload)
        for name, v in self.params.items():
            off, nb = self.param_layout[name]
            raw = np.frombuffer(buf[off:off + nb], dtype=np.float32 if v.dtype == "fp32" else np.int16)
            t = torch.from_numpy(raw.copy()).view(v.shape)
            if v.dtype == "bf16":
                t = t.view(torch.bfloat16)
            out[name] = t.to(device)
        return out

    def input_tensor(self, device, data: np.ndarray | None = None):
        import torch

        v = self.inputs[0]
        if data is None:
            x = torch.zeros(v.shape, dtype=torch_dtype(v.dtype))
        elif v.dtype == "i32":
            x = torch.from_numpy(np.ascontiguousarray(data, dtype=np.int32)).view(v.shape)
        else:
            x = torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32)).view(v.shape).to(torch_dtype(v.dtype))
        return x.to(device)

    def id_bound(self) -> int | None:
        """For an i32 (token id) input: the smallest embedding table it
        indexes -- ids must lie in [0, bound) (checked per request)."""
        if self.inputs[0].dtype != "i32":
            return None
        vs = [self.values[n.inputs[1]].shape[0] for n in self.nodes if n.op == "embedding"]
        return min(vs) if vs else None

    # ------------------------------------------------------------ execution
    def compile(self, device, params: dict | None = None) -> "CompiledProgram":
        return CompiledProgram(self, device, params)

    def reference(self, x, params: dict | None = None) -> tuple:
        """Eager, unfused, fp32 evaluation of the graph on the CPU (the
        numerics reference: every op in plain PyTorch)."""
        import torch

        ps = params if params is not None else self.tensors("cpu")
        env = {k: t.float().cpu() for k, t in ps.items()}
        env[self.inputs[0].name] = x.cpu() if self.inputs[0].dtype == "i32" else x.float().cpu()
        with torch.no_grad():
            for n in self.nodes:
                args = [env[i] for i in n.inputs]
                if n.op == "cast":
                    env[n.output] = args[0]
                else:
                    env[n.output] = _eager(n.op, args, n.attrs, ref=True)
        return tuple(env[o] for o in self.outputs)


def torch_dtype(dt: str):
    import torch

    return {"fp32": torch.float32, "bf16": torch.bfloat16, "i32": torch.int32}[dt]


def parse_variants(objs: list, payload: bytes | memoryview = b"", gpu: bool = False) -> list[Program]:
    """A tenant's programs for several input shapes (sequence-length or image
    size buckets) over ONE weight payload: each is parsed like :func:`parse`;
    all must declare the same weights (names, shapes, dtypes, payload spans)
    and input dtype, and their input shapes must differ.  The server builds
    one graph per shape on shared weight tensors and routes each request by
    its input shape."""
    _req(isinstance(objs, list) and 1 <= len(objs) <= MAX_VARIANTS,
         f"a tenant registers 1 to {MAX_VARIANTS} program variants")
    progs = [parse(o, payload, gpu=gpu) for o in objs]
    p0 = progs[0]
    seen = set()
    for p in progs:
        sig = {k: (v.shape, v.dtype) for k, v in p.params.items()}
        _req(sig == {k: (v.shape, v.dtype) for k, v in p0.params.items()} and p.param_layout == p0.param_layout,
             f"variant {p.name!r} declares other weights than {p0.name!r}: variants share one weight payload")
        _req(p.inputs[0].dtype == p0.inputs[0].dtype, "variants take the same input dtype")
        _req(p.inputs[0].shape not in seen, f"two variants take the input shape {list(p.inputs[0].shape)}")
        seen.add(p.inputs[0].shape)
    return progs


def parse(obj: dict, payload: bytes | memoryview = b"", gpu: bool = False) -> Program:
    """Validate a wire program (see the module docstring) against its payload;
    ``gpu``: also check the native kernels' shape constraints."""
    _req(isinstance(obj, dict), "program must be a JSON object")
    _req(obj.get("format") == FORMAT, f"program format must be {FORMAT!r}")
    extra = set(obj) - {"format", "name", "inputs", "params", "nodes", "outputs", "meta"}
    _req(not extra, f"unknown program keys {sorted(extra)}")
    name = str(obj.get("name", "program"))[:128]
    values: dict[str, Value] = {}

    def define(v: Value) -> None:
        _req(v.name not in values, f"value {v.name!r} is defined twice")
        values[v.name] = v

    ins = obj.get("inputs")
    _req(isinstance(ins, list) and len(ins) == 1, "a program takes exactly one input")
    inputs = []
    for d in ins:
        _req(isinstance(d, dict), "inputs must be objects")
        dt = d.get("dtype", "fp32")
        _req(dt in WIRE_DTYPES, f"input dtype must be one of {sorted(WIRE_DTYPES)}")
        v = Value(_name(d.get("name"), "input name"), _shape(d.get("shape"), "input shape"), dt, "input")
        define(v)
        inputs.append(v)
    ps = obj.get("params", [])
    _req(isinstance(ps, list) and len(ps) <= MAX_PARAMS, f"params must be a list of at most {MAX_PARAMS}")
    params: dict[str, Value] = {}
    layout: dict[str, tuple[int, int]] = {}
    spans = []
    for d in ps:
        _req(isinstance(d, dict), "params must be objects")
        dt = d.get("dtype", "fp32")
        _req(dt in FLOAT_DTYPES, f"param dtype must be one of {FLOAT_DTYPES}")
        v = Value(_name(d.get("name"), "param name"), _shape(d.get("shape"), "param shape"), dt, "param")
        off, nb = _int(d.get("offset"), "param offset", 0), _int(d.get("nbytes"), "param nbytes", 0)
        _req(nb == v.nbytes, f"param {v.name!r}: nbytes {nb} != {v.nbytes} for {v.shape} {dt}")
        _req(off % WIRE_DTYPES[dt] == 0, f"param {v.name!r}: offset must be {dt}-aligned")
        _req(off + nb <= len(payload), f"param {v.name!r} lies outside the {len(payload)}-byte payload")
        define(v)
        params[v.name] = v
        layout[v.name] = (off, nb)
        spans.append((off, off + nb, v.name))
    spans.sort()
    for (a0, a1, an), (b0, _b1, bn) in zip(spans, spans[1:]):
        _req(b0 >= a1, f"params {an!r} and {bn!r} overlap in the payload")
    ns = obj.get("nodes")
    _req(isinstance(ns, list) and 0 < len(ns) <= MAX_NODES, f"nodes must be a list of 1..{MAX_NODES}")
    nodes = []
    for d in ns:
        _req(isinstance(d, dict) and set(d) <= {"op", "inputs", "output", "attrs"}, "a node is {op, inputs, output, attrs}")
        op = d.get("op")
        _req(op in OPS, f"op {op!r} is not one the pod server runs (whitelist: {' '.join(OPS)})")
        refs = d.get("inputs")
        _req(isinstance(refs, list) and refs, f"node of op {op}: inputs must be a non-empty list")
        for r in refs:
            _req(isinstance(r, str) and r in values, f"node of op {op}: input {r!r} is not defined before it")
        attrs = d.get("attrs") or {}
        _req(isinstance(attrs, dict), "attrs must be an object")
        n = Node(op, list(refs), _name(d.get("output"), "node output"), dict(attrs))
        shape, dt = _infer(n, [values[r] for r in refs], gpu)
        _req(math.prod(shape) <= MAX_NUMEL, f"node {n.output!r}: output too large")
        define(Value(n.output, shape, dt, "node"))
        nodes.append(n)
    outs = obj.get("outputs")
    _req(isinstance(outs, list) and outs and all(isinstance(o, str) and o in values for o in outs),
         "outputs must name defined values")
    return Program(name, inputs, params, layout, nodes, list(outs), values, payload)


# ---------------------------------------------------------------- execution
def _eager(op: str, args: list, attrs: dict, ref: bool = False):
    """One unfused op in PyTorch (constant folding, and :meth:`Program.reference`)."""
    import torch
    import torch.nn.functional as F

    from .. import ops

    if op == "linear":
        y = F.linear(args[0], args[1], args[2] if len(args) > 2 else None)
        act = attrs.get("act")
        return F.gelu(y) if act == "gelu" else (F.relu(y) if act == "relu" else y)
    if op == "layernorm":
        x = args[0]
        return F.layer_norm(x, (x.shape[-1],), args[1], args[2], attrs.get("eps", 1e-5))
    if op == "attention":
        # fp32 under h3 math: the h3 flash kernel with per-row scales (a bare
        # attention has no LN-folded weights to bound K / V; the x6 kernel it
        # replaces spends six MFMAs per product instead of three)
        h3 = (args[0].is_cuda and args[0].dtype == torch.float32 and ops.f32_math() == "h3" and not ref
              and os.environ.get("NOS_AMD_BARE_ATTN_X6") != "1")   # (=1: the x6 kernel, for A/B)
        if (attrs.get("causal") or args[0].shape[-1] // (3 * attrs["heads"]) != 64 or not args[0].is_cuda
                or h3):
            from ..ops import tenant as T

            q, k, v = _qkv_views(args[0], attrs["heads"])
            if "q_start" in attrs:
                q = q[:, attrs["q_start"]:attrs["q_end"]]
            return T.sdpa(q, k, v, causal=attrs.get("causal", False), scale=attrs.get("scale")).flatten(2)
        y = ops.attention_qkv(args[0].contiguous(), attrs["heads"], scale=attrs.get("scale"))
        return y[:, attrs["q_start"]:attrs["q_end"]] if "q_start" in attrs else y
    if op == "add":
        return args[0] + args[1]
    if op == "mul":
        return args[0] * args[1]
    if op == "gelu":
        return F.gelu(args[0])
    if op == "relu":
        return F.relu(args[0])
    if op == "sigmoid":
        return torch.sigmoid(args[0])
    if op == "silu":
        return F.silu(args[0])
    if op == "cat":
        return torch.cat(args, dim=attrs["dim"])
    if op == "slice":
        d = attrs["dim"]
        return args[0].narrow(d, attrs["start"], attrs["end"] - attrs["start"])
    if op == "reshape":
        return args[0].reshape(attrs["shape"])
    if op == "permute":
        return args[0].permute(attrs["dims"])
    if op == "expand":
        return args[0].expand(attrs["shape"])
    if op == "cast":
        return args[0].to(torch_dtype(attrs["dtype"]))
    if op == "interpolate":
        mode = attrs.get("mode", "bicubic")
        return F.interpolate(args[0], size=tuple(attrs["size"]), mode=mode,
                             align_corners=None if mode == "nearest" else False)
    if op == "sub":
        return args[0] - args[1]
    if op == "div":
        return args[0] / args[1]
    if op == "tanh":
        return torch.tanh(args[0])
    if op == "exp":
        return torch.exp(args[0])
    if op == "neg":
        return -args[0]
    if op == "rsqrt":
        return torch.rsqrt(args[0])
    if op == "conv2d":
        return F.conv2d(args[0], args[1], args[2] if len(args) > 2 else None, _pair2(attrs, "stride", 1),
                        _pair2(attrs, "padding", 0), _pair2(attrs, "dilation", 1), attrs.get("groups", 1))
    if op == "batchnorm":
        return F.batch_norm(args[0], args[3], args[4], args[1], args[2], False, 0.0, attrs.get("eps", 1e-5))
    if op == "max_pool2d":
        k = _pair2(attrs, "kernel", 1)
        return F.max_pool2d(args[0], k, attrs.get("stride") and _pair2(attrs, "stride", 1) or k,
                            _pair2(attrs, "padding", 0))
    if op == "avg_pool2d":
        k = _pair2(attrs, "kernel", 1)
        return F.avg_pool2d(args[0], k, attrs.get("stride") and _pair2(attrs, "stride", 1) or k,
                            _pair2(attrs, "padding", 0))
    if op == "mean":
        return args[0].mean(dim=attrs["dims"], keepdim=attrs.get("keepdim", False))
    if op == "sum":
        return args[0].sum(dim=attrs["dims"], keepdim=attrs.get("keepdim", False))
    if op == "matmul":
        return args[0] @ args[1]
    if op == "softmax":
        return torch.softmax(args[0].float(), dim=-1).to(args[0].dtype)
    if op == "embedding":
        return F.embedding(args[0].long(), args[1])
    from ..ops import tenant as T

    if op == "rmsnorm":
        return T.rmsnorm_ref(args[0], args[1], attrs.get("eps", 1e-5))
    if op == "rotary":
        return T.rope_ref(args[0], args[1], args[2])
    if op == "sdpa":
        return T.sdpa_ref(args[0], args[1], args[2], attrs.get("causal", False), attrs.get("scale"))
    raise ProgramError(f"op {op!r}")


def _pair2(attrs: dict, key: str, default: int) -> tuple[int, int]:
    v = attrs.get(key, default)
    return (v, v) if isinstance(v, int) else (v[0], v[1])


def _qkv_views(qkv, heads: int):
    """q, k, v [B, S, H, D] views of a fused projection [B, S, 3*H*D]."""
    B, S, n = qkv.shape
    return qkv.view(B, S, 3, heads, n // (3 * heads)).unbind(2)


@dataclass
class _Step:
    kind: str                     # op name or a fused kind: linear_ln | ln_qkv_attention
    inputs: list[str]
    output: str
    attrs: dict
    release: list[str] = field(default_factory=list)   # values whose last use this is


class CompiledProgram:
    """A parsed program lowered onto the nos-amd ops for one device (see the
    module docstring for the passes).  ``__call__(x)`` returns the outputs as
    a tuple; it launches only stream-ordered work, so it can be captured into
    a HIP graph."""

    def __init__(self, prog: Program, device, params: dict | None = None):
        import torch

        self.program = prog
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.consts: dict[str, object] = dict(params) if params is not None else prog.tensors(self.device)
        self.input_name = prog.inputs[0].name
        self.outputs = list(prog.outputs)
        self.stats: dict[str, int] = {}
        self.aux: dict[str, object] = {}   # derived weights a kernel reads (e.g. conv weights as padded matrices)
        self._new_shapes: dict[str, tuple] = {}   # values the passes create or re-shape
        self._new_dtypes: dict[str, str] = {}
        with torch.no_grad():
            # NOS_AMD_SKIP_PASSES=name,...: leave launch-trimming passes out (A/B runs)
            skip = self._skip = set(os.environ.get("NOS_AMD_SKIP_PASSES", "").split(","))
            steps = self._fold_constants(prog)
            if "add_over_cat" not in skip:
                steps = self._distribute_add_over_cat(steps)
            if "patchify" not in skip:
                steps = self._fuse_patchify(steps)
            if "cast_relayout" not in skip:
                steps = self._fuse_cast_relayout(steps)
            steps = self._pushdown_row_slices(steps)
            steps = self._fold_batchnorm(steps)
            steps = self._merge_parallel_linears(steps)
            if "blockdiag" not in skip:
                steps = self._merge_blockdiag_linears(steps)
            steps = self._fold_layernorm(steps)
            steps = self._fold_rmsnorm(steps)
            steps = self._fuse_epilogues(steps)
            if "cast_unary" not in skip:
                steps = self._fuse_cast_unary(steps)
            steps = self._fuse_qkv_attention(steps)
            steps = self._fuse_rotary_sdpa(steps)
            if "cat_buffer" not in skip:
                steps = self._cat_into_buffer(steps)
            steps = self._mark_plane_handoffs(steps)
            steps = self._mark_ln_handoffs(steps)
            self._prep_conv_weights(steps)
            self.steps = self._plan_releases(steps)
            used = {i for s in self.steps for i in s.inputs} | set(self.outputs)
            for k in [k for k in self.consts if k not in used]:  # e.g. weights replaced by their LN-folded form
                del self.consts[k]
        self.stats["kernels"] = sum(1 for s in self.steps if s.kind in NATIVE_KINDS)

    # ------------------------------------------------------------ passes
    def _fold_constants(self, prog: Program) -> list[_Step]:
        """Run every all-constant node once at load time.  A constant is freed
        as soon as no later node (folded or not) and no output uses it, so a
        chain of large folded values never holds more than its live links
        (:meth:`Program.bytes_estimate_for` counts them as weights)."""
        last: dict[str, int] = {}
        for k, n in enumerate(prog.nodes):
            for i in n.inputs:
                last[i] = k
        keep = set(self.outputs)
        steps = []
        folded = 0
        for k, n in enumerate(prog.nodes):
            if all(i in self.consts for i in n.inputs) and n.op not in NEVER_FOLD:
                self.consts[n.output] = _eager(n.op, [self.consts[i] for i in n.inputs], n.attrs).contiguous()
                folded += 1
                for i in set(n.inputs):
                    if last.get(i) == k and i not in keep:
                        self.consts.pop(i, None)
            else:
                steps.append(_Step(n.op, list(n.inputs), n.output, dict(n.attrs)))
        # weights only feeding folded nodes are dead now
        live = {i for s in steps for i in s.inputs} | set(self.outputs)
        for k in [k for k in self.consts if k not in live]:
            del self.consts[k]
        self.stats["constant_folded"] = folded
        return steps

    def _cat_into_buffer(self, steps: list[_Step]) -> list[_Step]:
        """A cat whose parts are constants plus one GEMM output (YOLOS's [cls,
        patches, detection tokens]) needs no copy kernel: the constant parts go
        into a persistent buffer once, at build, and the GEMM writes its rows
        straight into the buffer's slab (``out=``).  Only where the slab is
        contiguous (every dim before the cat dim of size 1)."""
        import torch

        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        n = 0
        for c in steps:
            if c.kind != "cat" or c.output in self.outputs:
                continue
            dyn = [i for i in c.inputs if i not in self.consts]
            if len(dyn) != 1 or c.inputs.count(dyn[0]) != 1:
                continue
            p = by_out.get(dyn[0])
            shape = tuple(self._shape(c.output))
            d = c.attrs.get("dim", 0) % len(shape)
            if (p is None or p.kind != "linear" or uses.get(p.output) != 1 or p.attrs.get("row_stats")
                    or math.prod(shape[:d]) != 1 or self._dtype(p.output) not in ("fp32", "bf16")):
                continue
            buf = torch.empty(shape, dtype=torch_dtype(self._dtype(c.output)), device=self.device)
            off = 0
            for i in c.inputs:
                ln = self._shape(i)[d]
                if i != p.output:
                    buf.narrow(d, off, ln).copy_(self.consts[i])
                else:
                    p.attrs["out_into"] = (c.output + "::buf", d, off)
                off += ln
            self.aux[c.output + "::buf"] = buf
            c.kind, c.inputs, c.attrs = "cat_buffer", [p.output], {"buf": c.output + "::buf"}
            n += 1
        self.stats["cats_in_place"] = n
        return steps

    def _fuse_patchify(self, steps: list[_Step]) -> list[_Step]:
        """[cast fp32 -> bf16] -> [crop slices] -> reshape [N, C, H/ph, ph,
        W/pw, pw] -> permute (0, 2, 4, 1, 3, 5) -> reshape [N, P, C ph pw] of
        an fp32 image, read only by linears: a ViT's patch extraction.  One
        ``patches`` step on the image itself: the im2col kernel reads the
        top-left (H/ph)ph x (W/pw)pw window through the image's strides (the
        crop is free) and writes the patch rows straight as the GEMM's h3
        planes (fp32 under h3 math: no copy, no split pass) or as bf16 rows
        (the cast folded in); elsewhere the same views in PyTorch."""
        uses = self._consumers(steps, self.outputs)
        by_in: dict[str, list[_Step]] = {}
        by_out = {s.output: s for s in steps}
        for s in steps:
            for i in s.inputs:
                by_in.setdefault(i, []).append(s)
        drop: set[int] = set()
        n = 0
        for r1 in steps:
            if r1.kind != "reshape" or uses.get(r1.output) != 1:
                continue
            dt = self._dtype(r1.inputs[0])
            if dt not in ("fp32", "bf16"):
                continue
            # the image behind the crops (and the cast of a bf16 tenant)
            src, pre = r1.inputs[0], []
            while (src in by_out and by_out[src].kind == "slice" and uses.get(src) == 1
                   and by_out[src].attrs["dim"] % 4 in (2, 3) and by_out[src].attrs["start"] == 0):
                pre.append(by_out[src])
                src = by_out[src].inputs[0]
            if dt == "bf16":
                c = by_out.get(src)
                if c is None or c.kind != "cast" or uses.get(src) != 1 or self._dtype(c.inputs[0]) != "fp32":
                    continue
                pre.append(c)
                src = c.inputs[0]
            xs = tuple(self._shape(r1.inputs[0]))
            sh = tuple(r1.attrs["shape"])
            if len(xs) != 4 or len(sh) != 6 or sh[0] != xs[0] or sh[1] != xs[1] or sh[2] * sh[3] != xs[2] \
                    or sh[4] * sh[5] != xs[3]:
                continue
            pm = by_in[r1.output][0]
            if pm.kind != "permute" or list(pm.attrs["dims"]) != [0, 2, 4, 1, 3, 5] or uses.get(pm.output) != 1:
                continue
            r2 = by_in[pm.output][0]
            N, C, hp, ph, wp, pw = sh
            if (r2.kind != "reshape" or list(r2.attrs["shape"]) != [N, hp * wp, C * ph * pw]
                    or (dt == "fp32" and (C * ph * pw) % 32) or r2.output in self.outputs
                    or not all(c.kind == "linear" and c.inputs[0] == r2.output for c in by_in.get(r2.output, []))):
                continue
            drop.update(id(x) for x in (r1, pm, *pre))
            r2.kind, r2.inputs = "patches", [src]
            r2.attrs = {"ph": ph, "pw": pw, "hp": hp, "wp": wp, "dtype": dt}
            n += 1
        self.stats["patchify_fused"] = n
        return [s for s in steps if id(s) not in drop]

    def _fuse_cast_unary(self, steps: list[_Step]) -> list[_Step]:
        """cast -> activation, or activation -> cast (each value read once):
        one ``unary`` step that evaluates the activation in fp32 and writes
        the cast's dtype (a bf16 head's fp32 sigmoid boxes: one launch, not
        two).  Runs after the epilogue fusion, so only activations no GEMM
        absorbed are left."""
        from ..ops.tenant import UNARY_CODES

        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop: set[int] = set()
        n = 0
        for s in steps:
            if id(s) in drop:
                continue
            if s.kind in UNARY_CODES:
                p = by_out.get(s.inputs[0])
                if (p is None or p.kind != "cast" or id(p) in drop or uses.get(p.output) != 1
                        or p.output in self.outputs):
                    continue
                src, act, dt = p.inputs[0], s.kind, self._dtype(s.output)
            elif s.kind == "cast":
                p = by_out.get(s.inputs[0])
                if (p is None or p.kind not in UNARY_CODES or id(p) in drop or uses.get(p.output) != 1
                        or p.output in self.outputs):
                    continue
                src, act, dt = p.inputs[0], p.kind, s.attrs["dtype"]
            else:
                continue
            if self._dtype(src) not in ("fp32", "bf16") or dt not in ("fp32", "bf16"):
                continue
            drop.add(id(p))
            s.kind, s.inputs, s.attrs = "unary", [src], {"op": act, "dtype": dt}
            n += 1
        self.stats["cast_unary_fused"] = n
        return [s for s in steps if id(s) not in drop]

    def _fuse_cast_relayout(self, steps: list[_Step]) -> list[_Step]:
        """cast -> reshape / permute chain (each value read once) -> ONE
        relayout step: the chain's views, and the one copy a non-viewable
        reshape needs done as the cast (strided read, converted contiguous
        write) -- a bf16 tenant's image cast and its patch extraction are one
        launch instead of two."""
        uses = self._consumers(steps, self.outputs)
        by_in: dict[str, list[_Step]] = {}
        for s in steps:
            for i in s.inputs:
                by_in.setdefault(i, []).append(s)
        drop: set[int] = set()
        n = 0
        for s in steps:
            if s.kind != "cast" or uses.get(s.output) != 1 or s.output in self.outputs:
                continue
            chain, cur = [], s.output
            while uses.get(cur) == 1 and cur not in self.outputs:
                nxt = by_in[cur][0]
                if nxt.kind not in ("reshape", "permute"):
                    break
                chain.append(nxt)
                cur = nxt.output
            if not chain:
                continue
            ops_ = [("reshape", list(c.attrs["shape"])) if c.kind == "reshape" else ("permute", list(c.attrs["dims"]))
                    for c in chain]
            last = chain[-1]
            for c in chain[:-1]:
                drop.add(id(c))
            drop.add(id(s))
            last.kind, last.inputs, last.attrs = "relayout", [s.inputs[0]], {"chain": ops_, "dtype": s.attrs["dtype"]}
            n += 1
        self.stats["cast_relayouts_fused"] = n
        return [s for s in steps if id(s) not in drop]

    def _distribute_add_over_cat(self, steps: list[_Step]) -> list[_Step]:
        """add(cat(parts), c) with c a constant -> cat(add(part_i, c_i)): the
        constant parts fold here and the add on a GEMM's part becomes that
        GEMM's residual (YOLOS: the position embeddings added to [cls, patches,
        detection tokens] -- the patch-embedding GEMM absorbs its slice, the
        cls / detection slices fold; one elementwise launch fewer)."""
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop: set[int] = set()
        before: dict[int, list[_Step]] = {}
        n = 0
        for s in steps:
            if s.kind != "add":
                continue
            for catn, cn in ((s.inputs[0], s.inputs[1]), (s.inputs[1], s.inputs[0])):
                c = by_out.get(catn)
                if c is None or c.kind != "cat" or uses.get(catn) != 1 or cn not in self.consts or catn == cn:
                    continue
                cst = self.consts[cn]
                cshape = tuple(self._shape(catn))
                if tuple(self._shape(s.output)) != cshape or cst.dim() > len(cshape):
                    continue  # the constant must not broadcast the cat's output up
                r = len(cshape)
                d = c.attrs.get("dim", 0) % r
                dc = d - (r - cst.dim())  # the constant's dim aligned with d (< 0: broadcast)
                full = dc >= 0 and cst.shape[dc] == cshape[d]
                if dc >= 0 and not full and cst.shape[dc] != 1:
                    continue
                parts, new, off = [], [], 0
                for k, pi in enumerate(c.inputs):
                    ln = self._shape(pi)[d]
                    ci = cst.narrow(dc, off, ln).contiguous() if full else cst
                    off += ln
                    name = f"{s.output}::cat{k}"
                    if pi in self.consts:
                        self.consts[name] = (self.consts[pi] + ci).contiguous()
                    else:
                        cname = f"{s.output}::c{k}"
                        self.consts[cname] = ci
                        new.append(_Step("add", [pi, cname], name, {}))
                        self._new_shapes[name] = tuple(self._shape(pi))
                        self._new_dtypes[name] = self._dtype(pi)
                    parts.append(name)
                c.inputs, c.output = parts, s.output
                before[id(c)] = new
                drop.add(id(s))
                n += 1
                break
        out = []
        for s in steps:
            out.extend(before.get(id(s), []))
            if id(s) not in drop:
                out.append(s)
        # constants only the distributed adds read are dead now
        live = {i for s in out for i in s.inputs} | set(self.outputs)
        for k in [k for k in self.consts if k not in live]:
            del self.consts[k]
        self.stats["adds_distributed"] = n
        return out

    def _pushdown_row_slices(self, steps: list[_Step]) -> list[_Step]:
        """Dead-row elimination: a slice along a row (non-feature) dim of a value
        only it consumes moves above the row-wise op that made it -- elementwise
        ops, linears, norms -- and into an attention as a query range (its keys
        and values still cover every row).  YOLOS keeps only its 100 detection
        tokens after the last layer: that layer's attention, projection and MLP
        then run on those 100 rows instead of 3401."""
        n = 0
        while True:
            steps = self._dedupe_slices(steps)
            uses = self._consumers(steps, self.outputs)
            by_out = {s.output: s for s in steps}
            hit = None
            for s in steps:
                if s.kind != "slice":
                    continue
                src = s.inputs[0]
                p = by_out.get(src)
                if p is None or uses.get(src) != 1:
                    continue
                shp = self._shape(src)
                r = len(shp)
                d = s.attrs["dim"] % r
                if d == r - 1:
                    continue  # a feature-column slice: not row-wise
                plan = self._slice_plan(p, d, r, shp)
                if plan is not None:
                    hit = (s, p, d, plan)
                    break
            if hit is None:
                break
            s, p, d, plan = hit
            st, en = s.attrs["start"], s.attrs["end"]
            new_steps = []
            for idx, dim in plan:  # slice these inputs of p
                name = p.inputs[idx]
                nn_ = f"{name}::rows{st}_{en}_{n}"
                sh = list(self._shape(name))
                sh[dim] = en - st
                self._new_shapes[nn_] = tuple(sh)
                self._new_dtypes[nn_] = self._dtype(name)
                new_steps.append(_Step("slice", [name], nn_, {"dim": dim, "start": st, "end": en}))
                p.inputs[idx] = nn_
            if p.kind in ("attention",):  # a query range on top of any earlier one
                q0 = p.attrs.get("q_start", 0)
                p.attrs["q_start"], p.attrs["q_end"] = q0 + st, q0 + en
            p.output = s.output
            self._new_shapes[s.output] = self._shape(s.output)
            i = steps.index(p)
            steps = [x for x in steps if x is not s]
            steps[i:i] = new_steps
            n += 1
        self.stats["row_slices_pushed"] = n
        return steps

    def _dedupe_slices(self, steps: list[_Step]) -> list[_Step]:
        """Identical slices of one value (the same rows pushed up two paths,
        e.g. a residual and the norm after it) become one."""
        seen: dict[tuple, str] = {}
        rename: dict[str, str] = {}
        out = []
        for s in steps:
            s.inputs = [rename.get(i, i) for i in s.inputs]
            if s.kind == "slice" and s.output not in self.outputs:
                key = (s.inputs[0], s.attrs["dim"] % len(self._shape(s.inputs[0])), s.attrs["start"], s.attrs["end"])
                if key in seen:
                    rename[s.output] = seen[key]
                    continue
                seen[key] = s.output
            out.append(s)
        return out

    def _slice_plan(self, p: _Step, d: int, r: int, out_shape) -> list[tuple[int, int]] | None:
        """Which inputs of row-wise step ``p`` (output rank ``r``) to slice along
        output dim ``d``, as (input index, input dim); None: not row-wise in d."""
        if p.kind in UNARY or p.kind == "cast":
            return [(0, d)]
        if p.kind in ("linear", "layernorm", "rmsnorm"):
            return [(0, d)] if len(self._shape(p.inputs[0])) == r else None
        if p.kind in BINARY:
            plan = []
            for i, name in enumerate(p.inputs):
                sh = self._shape(name)
                di = d - (r - len(sh))
                if di < 0 or sh[di] == 1:
                    continue  # broadcast along d: every row uses the same values
                if sh[di] != out_shape[d]:
                    return None
                plan.append((i, di))
            return plan
        if p.kind == "attention" and d == 1 and not p.attrs.get("causal"):
            return []  # the query range; keys / values still read every row
        return None

    def _fold_batchnorm(self, steps: list[_Step]) -> list[_Step]:
        """conv2d -> batchnorm (inference statistics, all weights constant)
        becomes one conv2d with W' = W gamma / sqrt(var + eps) and
        b' = (b - mean) gamma / sqrt(var + eps) + beta."""
        import torch

        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "batchnorm":
                continue
            c = by_out.get(s.inputs[0])
            if (c is None or c.kind != "conv2d" or uses.get(c.output) != 1
                    or not all(i in self.consts for i in c.inputs[1:] + s.inputs[1:])):
                continue
            w = self.consts[c.inputs[1]]
            b = self.consts[c.inputs[2]].float() if len(c.inputs) > 2 else 0.0
            g, be, mu, var = (self.consts[i].float() for i in s.inputs[1:])
            inv = g * torch.rsqrt(var + s.attrs.get("eps", 1e-5))
            base = f"{s.output}::bn"
            self.consts[base + ".w"] = (w.float() * inv[:, None, None, None]).to(w.dtype).contiguous()
            self.consts[base + ".b"] = ((b - mu) * inv + be).to(w.dtype).contiguous()
            c.inputs = [c.inputs[0], base + ".w", base + ".b"]
            drop.add(c.output)
            c.output = s.output
            by_out[s.output] = c
            s.kind = "__dropped__"
            n += 1
        self.stats["batchnorm_folded"] = n
        return [s for s in steps if s.kind != "__dropped__"]

    def _merge_parallel_linears(self, steps: list[_Step]) -> list[_Step]:
        """Linears that read the same activation with constant weights (Q / K /
        V projections, an MLP's gate / up) become ONE GEMM over the
        concatenated weights, each original output a column slice (a view) of
        it: fewer, wider launches, and the norm before them gets a single
        consumer, which lets it fold into the GEMM."""
        import torch

        # a linear whose output feeds a GELU / ReLU merges only with linears
        # whose outputs feed the same activation (and nothing else): the merged
        # GEMM gets that activation (fused into its epilogue) and each original
        # activation becomes a column slice of it -- YOLOS's two detection
        # heads; mixed groups would lose the fusion
        uses = self._consumers(steps, self.outputs)
        act_of: dict[str, _Step] = {}
        for s in steps:
            if s.kind in ("gelu", "relu") and uses.get(s.inputs[0]) == 1:
                act_of[s.inputs[0]] = s
        act_fed = {s.inputs[0] for s in steps if s.kind in ("gelu", "relu")}
        groups: dict[tuple, list[_Step]] = {}
        for s in steps:
            if (s.kind == "linear" and s.inputs[0] not in self.consts and not s.attrs
                    and all(i in self.consts for i in s.inputs[1:])):
                if s.output in act_of:
                    key = (s.inputs[0], act_of[s.output].kind)
                elif s.output not in act_fed:
                    key = (s.inputs[0], None)
                else:
                    continue
                groups.setdefault(key, []).append(s)
        first: dict[int, list[_Step]] = {}
        dead: set[int] = set()
        n = 0
        for (x, act), g in groups.items():
            if len(g) < 2 or len({self.consts[m.inputs[1]].dtype for m in g}) != 1:
                continue
            ws = [self.consts[m.inputs[1]] for m in g]
            name = f"{g[0].output}::merged"
            self.consts[name + ".w"] = torch.cat(ws, dim=0).contiguous()
            ins = [x, name + ".w"]
            if any(len(m.inputs) > 2 for m in g):
                self.consts[name + ".b"] = torch.cat([self.consts[m.inputs[2]] if len(m.inputs) > 2 else
                                                      torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
                                                      for m, w in zip(g, ws)]).contiguous()
                ins.append(name + ".b")
            new_steps = [_Step("linear", ins, name, {})]
            self._new_shapes[name] = tuple(self._shape(x)[:-1]) + (sum(w.shape[0] for w in ws),)
            self._new_dtypes[name] = self._dtype(g[0].output)
            src = name
            if act is not None:
                src = name + "::" + act
                new_steps.append(_Step(act, [name], src, {}))
                self._new_shapes[src], self._new_dtypes[src] = self._new_shapes[name], self._new_dtypes[name]
            first[id(g[0])] = new_steps
            off = 0
            for m, w in zip(g, ws):
                tgt = act_of[m.output] if act is not None else m
                tgt.kind, tgt.inputs, tgt.attrs = "slice", [src], {"dim": -1, "start": off, "end": off + w.shape[0]}
                if act is not None:
                    dead.add(id(m))
                off += w.shape[0]
            n += len(g)
        out = []
        for s in steps:
            if id(s) in first:
                out.extend(first[id(s)])
            if id(s) not in dead:
                out.append(s)
        self.stats["linears_merged"] = n
        return out

    def _merge_blockdiag_linears(self, steps: list[_Step], max_rows: int = 1024) -> list[_Step]:
        """Small linears over ADJACENT column slices of one activation, with
        the same activation after them (YOLOS's two detection heads after
        their merged first layer: 384 -> 384 -> 92 classes and 384 -> 384 ->
        4 boxes) become ONE GEMM over the block-diagonal weight
        [[W1, 0], [0, W2]] on the joined slice, each original output a column
        slice of it -- a chain of such layers collapses level by level.  Only
        for at most ``max_rows`` rows: the zero blocks double the GEMM's
        FLOPs, which only a launch-bound GEMM does not notice."""
        import torch

        total = 0
        while True:
            uses = self._consumers(steps, self.outputs)
            by_out = {s.output: s for s in steps}
            act_of = {s.inputs[0]: s for s in steps if s.kind in ("gelu", "relu") and uses.get(s.inputs[0]) == 1}
            act_fed = {s.inputs[0] for s in steps if s.kind in ("gelu", "relu")}
            groups: dict[tuple, list[tuple[int, int, _Step]]] = {}
            for s in steps:
                sl = by_out.get(s.inputs[0]) if s.kind == "linear" else None
                if (sl is None or sl.kind != "slice" or s.attrs or not all(i in self.consts for i in s.inputs[1:])
                        or uses.get(sl.output) != 1):
                    continue
                shape = tuple(self._shape(sl.inputs[0]))
                if sl.attrs["dim"] % len(shape) != len(shape) - 1 or math.prod(shape[:-1]) > max_rows:
                    continue
                if s.output in act_of:
                    act = act_of[s.output].kind
                elif s.output not in act_fed:
                    act = None
                else:
                    continue
                key = (sl.inputs[0], act, str(self.consts[s.inputs[1]].dtype))
                groups.setdefault(key, []).append((sl.attrs["start"], sl.attrs["end"], s))
            first: dict[int, list[_Step]] = {}
            dead: set[int] = set()
            n = 0
            for (x, act, _), g in groups.items():
                g.sort(key=lambda t: t[0])
                runs, cur = [], [g[0]]
                for t in g[1:]:
                    if t[0] == cur[-1][1]:
                        cur.append(t)
                    else:
                        runs.append(cur)
                        cur = [t]
                runs.append(cur)
                for run in runs:
                    if len(run) < 2:
                        continue
                    ws = [self.consts[m.inputs[1]] for _, _, m in run]
                    nrow, ncol = sum(w.shape[0] for w in ws), sum(w.shape[1] for w in ws)
                    wbd = torch.zeros((nrow, ncol), dtype=ws[0].dtype, device=ws[0].device)
                    r = c = 0
                    for w in ws:
                        wbd[r:r + w.shape[0], c:c + w.shape[1]] = w
                        r, c = r + w.shape[0], c + w.shape[1]
                    m0 = run[0][2]
                    name = f"{m0.output}::blockdiag"
                    self.consts[name + ".w"] = wbd
                    lo, hi = run[0][0], run[-1][1]
                    new_steps = []
                    src = x
                    if lo != 0 or hi != self._shape(x)[-1]:
                        src = name + "::in"
                        new_steps.append(_Step("slice", [x], src, {"dim": -1, "start": lo, "end": hi}))
                        self._new_shapes[src] = tuple(self._shape(x)[:-1]) + (hi - lo,)
                        self._new_dtypes[src] = self._dtype(x)
                    ins = [src, name + ".w"]
                    if any(len(m.inputs) > 2 for _, _, m in run):
                        self.consts[name + ".b"] = torch.cat(
                            [self.consts[m.inputs[2]] if len(m.inputs) > 2 else
                             torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
                             for (_, _, m), w in zip(run, ws)]).contiguous()
                        ins.append(name + ".b")
                    new_steps.append(_Step("linear", ins, name, {}))
                    self._new_shapes[name] = tuple(self._shape(x)[:-1]) + (nrow,)
                    self._new_dtypes[name] = self._dtype(m0.output)
                    out = name
                    if act is not None:
                        out = name + "::" + act
                        new_steps.append(_Step(act, [name], out, {}))
                        self._new_shapes[out], self._new_dtypes[out] = self._new_shapes[name], self._new_dtypes[name]
                    first[id(m0)] = new_steps
                    off = 0
                    for (_, _, m), w in zip(run, ws):
                        dead.add(id(by_out[m.inputs[0]]))   # the input slice
                        tgt = act_of[m.output] if act is not None else m
                        tgt.kind, tgt.inputs, tgt.attrs = "slice", [out], {"dim": -1, "start": off,
                                                                           "end": off + w.shape[0]}
                        if act is not None:
                            dead.add(id(m))
                        off += w.shape[0]
                    n += len(run)
            if not n:
                break
            total += n
            merged = []
            for s in steps:
                if id(s) in first:
                    merged.extend(first[id(s)])
                if id(s) not in dead:
                    merged.append(s)
            steps = merged
        self.stats["linears_blockdiag_merged"] = total
        return steps

    @staticmethod
    def _consumers(steps: list[_Step], outputs: list[str]) -> dict[str, int]:
        c: dict[str, int] = {}
        for s in steps:
            for i in s.inputs:
                c[i] = c.get(i, 0) + 1
        for o in outputs:
            c[o] = c.get(o, 0) + 1
        return c

    def _fold_layernorm(self, steps: list[_Step]) -> list[_Step]:
        from .. import ops

        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "linear" or s.inputs[0] not in by_out:
                continue
            ln = by_out[s.inputs[0]]
            if ln.kind != "layernorm" or uses.get(ln.output) != 1 or not all(i in self.consts for i in
                                                                                s.inputs[1:] + ln.inputs[1:]):
                continue
            w, b = self.consts[s.inputs[1]], (self.consts[s.inputs[2]] if len(s.inputs) > 2 else None)
            g, be = self.consts[ln.inputs[1]], self.consts[ln.inputs[2]]
            wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
            base = f"{s.output}::ln"
            self.consts[base + ".w"], self.consts[base + ".c1"], self.consts[base + ".c2"] = wg, c1, c2
            s.kind = "linear_ln"
            s.inputs = [ln.inputs[0], base + ".w", base + ".c1", base + ".c2"]
            s.attrs = {"act": s.attrs.get("act"), "eps": ln.attrs.get("eps", 1e-5)}
            drop.add(ln.output)
            n += 1
        self.stats["layernorm_folded"] = n
        return [s for s in steps if s.output not in drop]

    def _fold_rmsnorm(self, steps: list[_Step]) -> list[_Step]:
        """rmsnorm -> linear (its only consumer, constant weights) becomes one
        ``linear_rms``: gamma folded into the weight, the row statistics in
        the h3 split pre-pass (ops.tenant.linear_rms)."""
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "linear" or s.inputs[0] not in by_out:
                continue
            rn = by_out[s.inputs[0]]
            if rn.kind != "rmsnorm" or uses.get(rn.output) != 1 or not all(i in self.consts for i in
                                                                              s.inputs[1:] + rn.inputs[1:]):
                continue
            w, g = self.consts[s.inputs[1]], self.consts[rn.inputs[1]]
            base = f"{s.output}::rms"
            self.consts[base + ".w"] = (w.float() * g.float()[None, :]).to(w.dtype).contiguous()
            s.kind = "linear_rms"
            s.inputs = [rn.inputs[0], base + ".w"] + s.inputs[2:]
            s.attrs = {"act": s.attrs.get("act"), "eps": rn.attrs.get("eps", 1e-5)}
            drop.add(rn.output)
            n += 1
        self.stats["rmsnorm_folded"] = n
        return [s for s in steps if s.output not in drop]

    def _fuse_epilogues(self, steps: list[_Step]) -> list[_Step]:
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        rename: dict[str, str] = {}
        keep = []
        n_act = n_res = 0
        for s in steps:
            orig = list(s.inputs)
            s.inputs = [rename.get(i, i) for i in s.inputs]
            src = by_out.get(s.inputs[0]) if s.inputs else None
            if (s.kind in ("gelu", "relu") and src is not None and src.kind in ("linear", "linear_ln", "linear_rms")
                    and uses.get(src.output) == 1 and not src.attrs.get("act") and "residual" not in src.attrs):
                src.attrs["act"] = s.kind
                rename[s.output] = src.output
                n_act += 1
                continue
            if (s.kind in ("gelu", "relu") and src is not None and src.kind == "conv2d" and uses.get(orig[0]) == 1
                    and not src.attrs.get("act")):
                # conv -> act, or conv + residual -> act (a ResNet block's tail: the
                # residual goes in before the activation)
                src.attrs["act"] = s.kind
                if src.attrs.get("residual"):
                    src.attrs["residual_first"] = True
                rename[s.output] = src.output
                n_act += 1
                continue
            if s.kind == "add":
                a, b = s.inputs
                for prod, other in ((a, b), (b, a)):
                    p = by_out.get(prod)
                    if (p is not None and p.kind in ("linear", "conv2d") and uses.get(prod) == 1
                            and "residual" not in p.attrs
                            and self._shape(prod) == self._shape(s.output) == self._shape(other)
                            and self._dtype(prod) == self._dtype(other) and other != prod):
                        p.attrs["residual"] = True
                        p.inputs = p.inputs + [other]
                        rename[s.output] = p.output
                        n_res += 1
                        break
                else:
                    keep.append(s)
                continue
            keep.append(s)
        # an output that was renamed into its producer
        self.outputs = [rename.get(o, o) for o in self.outputs]
        self.stats["activation_fused"], self.stats["residual_fused"] = n_act, n_res
        return self._reorder(keep)

    def _reorder(self, steps: list[_Step]) -> list[_Step]:
        """A fused residual may come from a value defined after the producer:
        re-sort topologically (stable)."""
        defined = set(self.consts) | {self.input_name}
        out, pending = [], list(steps)
        while pending:
            for i, s in enumerate(pending):
                if all(x in defined for x in s.inputs):
                    out.append(s)
                    defined.add(s.output)
                    pending.pop(i)
                    break
            else:
                raise ProgramError("program graph has a cycle after fusion")
        return out

    def _fuse_qkv_attention(self, steps: list[_Step]) -> list[_Step]:
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "attention":
                continue
            p = by_out.get(s.inputs[0])
            if p is None or p.kind != "linear_ln" or uses.get(p.output) != 1 or p.attrs.get("act"):
                continue
            d = self._shape(s.output)[-1] // s.attrs["heads"]
            if "scale" in s.attrs and s.attrs["scale"] != 1.0 / math.sqrt(d):
                continue  # the fused kernels use the default 1/sqrt(head_dim)
            if s.attrs.get("causal") or d != 64:
                continue  # the general attention (ops.tenant.sdpa) runs it
            s.kind = "ln_qkv_attention"
            s.attrs = {"heads": s.attrs["heads"], "eps": p.attrs["eps"],
                       **{k: s.attrs[k] for k in ("q_start", "q_end") if k in s.attrs}}
            s.inputs = list(p.inputs)
            drop.add(p.output)
            n += 1
        self.stats["qkv_attention_fused"] = n
        return [s for s in steps if s.output not in drop]

    def _fuse_rotary_sdpa(self, steps: list[_Step]) -> list[_Step]:
        """rotary(q), rotary(k) -> sdpa with the same constant tables: the
        rotation moves into the attention (Q on load, K in its split pass)."""
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "sdpa":
                continue
            pq, pk = by_out.get(s.inputs[0]), by_out.get(s.inputs[1])
            if (pq is None or pk is None or pq is pk or pq.kind != "rotary" or pk.kind != "rotary"
                    or uses.get(pq.output) != 1 or uses.get(pk.output) != 1 or pq.inputs[1:] != pk.inputs[1:]
                    or not all(i in self.consts for i in pq.inputs[1:])
                    or self._shape(pq.inputs[1])[0] != self._shape(s.inputs[1])[1]):
                continue
            s.inputs = [pq.inputs[0], pk.inputs[0], s.inputs[2]] + pq.inputs[1:]
            s.attrs = {**s.attrs, "rope": True}
            drop |= {pq.output, pk.output}
            n += 1
        self.stats["rotary_fused"] = n
        return [s for s in steps if s.output not in drop]

    def _prep_conv_weights(self, steps: list[_Step]) -> None:
        """GPU: every conv weight [OC, C, KH, KW] also as the fp32 [OC, Kp]
        matrix the h3 GEMM reads (K = C KH KW zero-padded to 32), kept so its
        split planes are cached across replays."""
        import torch.nn.functional as F

        if not self.gpu:
            return
        for s in steps:
            if s.kind != "conv2d" or s.inputs[1] not in self.consts:
                continue
            w = self.consts[s.inputs[1]]
            k = w[0].numel()
            w2 = w.float().reshape(w.shape[0], k)
            kp = -(-k // 32) * 32
            name = s.inputs[1] + "::mat"
            self.aux[name] = (F.pad(w2, (0, kp - k)) if kp != k else w2).contiguous()
            s.attrs["w2"] = name

    def _mark_plane_handoffs(self, steps: list[_Step]) -> list[_Step]:
        """A fused LN-QKV attention or LN-GEMM whose only consumer is a
        linear's A operand may, under h3 math, hand its output over as that
        GEMM's fp16 planes (ops.H3Planes): marked here, decided per run."""
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        n = 0
        for s in steps:
            if s.kind != "linear" or s.inputs[0] in s.inputs[1:]:
                continue
            p = by_out.get(s.inputs[0])
            if p is not None and p.kind in ("ln_qkv_attention", "linear_ln") and uses.get(p.output) == 1:
                p.attrs["planes_out"] = True
                n += 1
        self.stats["plane_handoffs"] = n
        return steps

    def _mark_ln_handoffs(self, steps: list[_Step]) -> list[_Step]:
        """A pre-LN residual GEMM (fp32 linear + residual) whose output exactly
        one LN-GEMM (``linear_ln`` / ``ln_qkv_attention``) normalises writes,
        under h3 math with ``ops.set_ln_handoff``, that output's row statistics
        in its epilogue (``nos_gemm_f32h3_stats``); the LN-GEMM then applies
        the LayerNorm in its own A load (``nos_gemm_f32h3_lna``) -- no split
        pass.  Marked here, decided per run."""
        by_out = {s.output: s for s in steps}
        consumers: dict[str, int] = {}
        for s in steps:
            if s.kind in ("linear_ln", "ln_qkv_attention") and s.inputs[0] in by_out:
                consumers[s.inputs[0]] = consumers.get(s.inputs[0], 0) + 1
        n = 0
        for name, k in consumers.items():
            p = by_out[name]
            if (p.kind == "linear" and p.attrs.get("residual") and k == 1 and self._dtype(name) == "fp32"
                    and self._shape(name)[-1] % 32 == 0):
                p.attrs["row_stats"] = True
                n += 1
            elif p.kind == "cat_buffer" and k == 1 and "cat_stats" not in self._skip and self._mark_cat_stats(p, by_out):
                n += 1
        self.stats["ln_handoffs"] = n
        return steps

    def _mark_cat_stats(self, c: _Step, by_out: dict) -> bool:
        """An LN-GEMM reading a cat written in place by its GEMM part (YOLOS's
        [cls, patches, detection tokens] before layer 0): the GEMM writes its
        rows' statistics into a stats buffer whose constant rows are computed
        here, once -- the LN-GEMM then needs no statistics pass.  Row-wise
        cats of fp32 rows whose width is whole 128-column parts only."""
        import torch

        p = by_out.get(c.inputs[0])
        buf = self.aux[c.attrs["buf"]]
        shape = tuple(buf.shape)
        into = p.attrs.get("out_into") if p is not None else None
        if (p is None or p.kind != "linear" or into is None or buf.dtype != torch.float32 or len(shape) < 2
                or into[1] % len(shape) != len(shape) - 2 or shape[-1] % 128 or math.prod(shape[:-2]) != 1):
            return False
        rows = buf.reshape(-1, shape[-1]).double().view(shape[-2], shape[-1] // 128, 128)
        mean = rows.mean(-1)
        st = torch.stack([mean, ((rows - mean[..., None]) ** 2).sum(-1)], dim=-1).float().contiguous()
        name = c.attrs["buf"] + "::stats"
        self.aux[name] = st
        c.attrs["stats"] = name
        p.attrs["row_stats"] = True
        p.attrs["stats_into"] = name
        return True

    def _plan_releases(self, steps: list[_Step]) -> list[_Step]:
        last: dict[str, int] = {}
        for k, s in enumerate(steps):
            for i in s.inputs:
                last[i] = k
        keep = set(self.outputs) | set(self.consts) | {self.input_name}
        for name, k in last.items():
            if name not in keep:
                steps[k].release.append(name)
        return steps

    def _shape(self, name: str):
        if name in self._new_shapes:
            return self._new_shapes[name]
        v = self.program.values.get(name)
        return v.shape if v is not None else tuple(self.consts[name].shape)

    def _dtype(self, name: str):
        v = self.program.values.get(name)
        if v is None and name in self._new_dtypes:
            return self._new_dtypes[name]
        if v is not None:
            return v.dtype
        t = str(self.consts[name].dtype)  # a constant: its wire name, as program values carry
        return {"torch.float32": "fp32", "torch.bfloat16": "bf16", "torch.int32": "i32"}.get(t, t)

    # ------------------------------------------------------------ run
    def __call__(self, x) -> tuple:
        from .. import ops
        from ..ops import tenant as T

        env = dict(self.consts)
        env[self.input_name] = x
        for s in self.steps:
            a = [env[i] for i in s.inputs]
            k = s.kind
            if k == "linear":
                res = a.pop() if s.attrs.get("residual") else None
                rs = bool(s.attrs.get("row_stats")) and ops.ln_handoff_active() and (
                    isinstance(a[0], ops.H3Planes) or (a[0].is_cuda and a[0].dtype.itemsize == 4))
                into = s.attrs.get("out_into")  # (buffer, dim, offset): a slab of a cat's buffer
                # rows with unit inner stride go in as they are (a merged GEMM's
                # column slice: the kernels take the row stride); others are copied
                xa = a[0] if isinstance(a[0], ops.H3Planes) else _rows(a[0])
                if isinstance(a[0], ops.H3Planes):
                    dst = self.aux[into[0]].narrow(into[1], into[2], self._shape(s.output)[into[1]]) if into else None
                    sto = None
                    if rs and into and s.attrs.get("stats_into"):   # the cat buffer's row statistics (slab rows)
                        sto = self.aux[s.attrs["stats_into"]].narrow(0, into[2], a[0].planes.shape[1])
                    y = ops.linear_planes(a[0], a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                          residual=res, row_stats=rs, out=dst, stats_out=sto)
                    if dst is not None:
                        y = (dst, y[1]) if rs else dst
                elif into is not None:
                    dst = self.aux[into[0]].narrow(into[1], into[2], self._shape(s.output)[into[1]])
                    y = ops.linear(xa, a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                   residual=res, out=dst if dst.is_cuda else None)
                    if y.data_ptr() != dst.data_ptr():
                        dst.copy_(y)
                    y = dst
                else:
                    y = ops.linear(xa, a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                   residual=res, row_stats=rs)
                if rs:
                    y, env[s.output + "::lnp"] = y
            elif k == "linear_ln":
                xx = a[0].contiguous()
                pre = env.pop(s.inputs[0] + "::lnp", None)  # its producer's row statistics (_mark_ln_handoffs)
                if (s.attrs.get("planes_out") and xx.is_cuda and xx.dtype.itemsize == 4
                        and ops.h3_planes_active()):
                    y = ops.linear_ln_to_planes(xx, a[1], a[2], a[3], act=s.attrs.get("act"), eps=s.attrs["eps"],
                                                pre=pre)
                else:
                    y = ops.linear_ln(xx, a[1], a[2], a[3], act=s.attrs.get("act"), eps=s.attrs["eps"], pre=pre)
            elif k == "ln_qkv_attention":
                h = a[0].contiguous()
                pre = env.pop(s.inputs[0] + "::lnp", None)
                qr = (s.attrs["q_start"], s.attrs["q_end"]) if "q_start" in s.attrs else None
                if ops.ln_qkv_fusable(h):
                    y = ops.ln_qkv_attention(h, a[1], a[2], a[3], s.attrs["heads"], eps=s.attrs["eps"],
                                             planes_out=bool(s.attrs.get("planes_out"))
                                             and ops.h3_planes_active(attention=True), pre=pre, q_range=qr)
                else:
                    qkv = ops.linear_ln(h, a[1], a[2], a[3], eps=s.attrs["eps"])
                    y = ops.attention_qkv(qkv, s.attrs["heads"])
                    if qr is not None:
                        y = y[:, qr[0]:qr[1]]
            elif k == "attention":
                y = _eager("attention", [a[0].contiguous()], s.attrs)
            elif k == "conv2d":
                res = a.pop() if s.attrs.get("residual") else None
                y = T.conv2d(a[0], a[1], a[2] if len(a) > 2 else None, _pair2(s.attrs, "stride", 1),
                             _pair2(s.attrs, "padding", 0), _pair2(s.attrs, "dilation", 1), act=s.attrs.get("act"),
                             residual=res, w2=self.aux.get(s.attrs.get("w2")),
                             residual_first=bool(s.attrs.get("residual_first")), groups=s.attrs.get("groups", 1))
            elif k == "linear_rms":
                y = T.linear_rms(a[0], a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"), eps=s.attrs["eps"])
            elif k == "matmul":
                y = T.matmul(a[0], a[1])
            elif k == "softmax":
                y = T.softmax(a[0])
            elif k == "embedding":
                y = T.embedding(a[0], a[1])
            elif k == "rmsnorm":
                y = T.rmsnorm(a[0], a[1], s.attrs.get("eps", 1e-5))
            elif k == "rotary":
                y = T.rotary(a[0], a[1], a[2])
            elif k == "sdpa":
                y = T.sdpa(a[0], a[1], a[2], causal=s.attrs.get("causal", False), scale=s.attrs.get("scale"),
                           rope=(a[3], a[4]) if s.attrs.get("rope") else None)
            elif k == "layernorm":
                xx = a[0].contiguous()
                if xx.is_cuda and str(xx.dtype) == "torch.bfloat16":
                    y, _ = ops.layernorm(xx, a[1], a[2], s.attrs.get("eps", 1e-5))
                else:
                    import torch.nn.functional as F

                    y = F.layer_norm(xx, (xx.shape[-1],), a[1], a[2], s.attrs.get("eps", 1e-5))
            elif k == "relayout":
                y = _relayout(a[0], s.attrs["chain"], s.attrs["dtype"])
            elif k == "unary":
                y = T.unary(a[0], s.attrs["op"], torch_dtype(s.attrs["dtype"]))
            elif k == "patches":
                at = s.attrs
                y = T.patches(a[0], at["ph"], at["pw"], torch_dtype(at.get("dtype", "fp32")), at.get("hp"), at.get("wp"))
            elif k == "cat_buffer":  # its GEMM part was written in place; the constant parts at build
                y = self.aux[s.attrs["buf"]]
                if env.pop(s.inputs[0] + "::lnp", None) is not None:
                    # the GEMM wrote its rows' statistics into the buffer's stats, whose
                    # constant rows were filled at build: the whole buffer's, for its LN-GEMM
                    env[s.output + "::lnp"] = ops.RowStats(self.aux[s.attrs["stats"]], 128)
            else:
                y = _eager(k, a, s.attrs)
            env[s.output] = y
            for r in s.release:
                env.pop(r, None)
        return tuple(env[o] for o in self.outputs)


def _rows(x):
    """x as-is when its rows [..., K] view as a 2-D [M, K] with unit inner
    stride and 16-byte-aligned rows (what the GEMMs take), else contiguous."""
    if x.stride(-1) == 1 and x.element_size() * x.stride(-2 if x.dim() > 1 else -1) % 16 == 0 and x.data_ptr() % 16 == 0:
        try:
            x.view(-1, x.shape[-1])
            return x
        except RuntimeError:
            pass
    return x.contiguous()


def _relayout(x, chain, dtype: str):
    """Apply the reshape / permute chain as views; the first reshape that
    cannot be a view is the one copy, written straight in ``dtype``."""
    import torch

    td = torch_dtype(dtype)
    v, done = x, x.dtype == td
    for op, arg in chain:
        if op == "permute":
            v = v.permute(*arg)
            continue
        try:
            v = v.view(*arg)
        except RuntimeError:
            out = torch.empty(arg, dtype=td, device=v.device)
            out.view(v.shape).copy_(v)
            v, done = out, True
    return v if done else v.to(td)


# ---------------------------------------------------------------- building (numpy only)
def bf16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns (round to nearest even), as uint16."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u >> 16) & 1) + 0x7FFF
    return ((u + r) >> 16).astype(np.uint16)


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


class Builder:
    """Assemble a wire program with numpy only (the pod side never imports
    torch).  ``param`` appends a weight to the payload; op methods append
    nodes and return the output's name."""

    def __init__(self, name: str):
        self.name = name
        self.inputs: list[dict] = []
        self.params: list[dict] = []
        self.nodes: list[dict] = []
        self.chunks: list[bytes] = []
        self.offset = 0
        self._n = 0

    def input(self, name: str, shape, dtype: str = "fp32") -> str:
        self.inputs.append({"name": name, "shape": list(shape), "dtype": dtype})
        return name

    def param(self, name: str, array: np.ndarray, dtype: str = "fp32") -> str:
        a = np.ascontiguousarray(array, dtype=np.float32)
        raw = (a if dtype == "fp32" else bf16_bits(a)).tobytes()
        self.params.append({"name": name, "shape": list(a.shape), "dtype": dtype, "offset": self.offset,
                            "nbytes": len(raw)})
        self.chunks.append(raw)
        self.offset += len(raw)
        return name

    def op(self, op: str, *inputs: str, out: str | None = None, **attrs) -> str:
        self._n += 1
        out = out or f"%{self._n}"
        self.nodes.append({"op": op, "inputs": list(inputs), "output": out,
                           "attrs": {k: v for k, v in attrs.items() if v is not None}})
        return out

    def build(self, outputs: list[str]) -> tuple[dict, bytes]:
        return ({"format": FORMAT, "name": self.name, "inputs": self.inputs, "params": self.params,
                 "nodes": self.nodes, "outputs": list(outputs)}, b"".join(self.chunks))


def save_program(prefix: str, program: dict, weights: bytes) -> None:
    """A built program as ``<prefix>.json`` + ``<prefix>.bin`` (a tenant
    builds once -- e.g. with torch.fx -- and its pods ship the files)."""
    import json

    with open(prefix + ".json", "w") as f:
        json.dump(program, f)
    with open(prefix + ".bin", "wb") as f:
        f.write(weights)


def load_program(prefix: str) -> tuple[dict, bytes]:
    """:func:`save_program`'s files back (JSON + raw bytes: nothing executable)."""
    import json

    with open(prefix + ".json") as f:
        program = json.load(f)
    with open(prefix + ".bin", "rb") as f:
        return program, f.read()


def mlp_program(dim: int = 1024, layers: int = 4, batch: int = 256, dtype: str = "bf16", seed: int = 0,
                hidden: int | None = None) -> tuple[dict, bytes]:
    """The GEMM-MLP probe tenant (BASELINE config 4's workload): ``layers``
    pre-LN residual MLP blocks (LN -> fc1 + GELU -> fc2 + residual) on a
    ``batch x dim`` activation; every block lowers onto two GEMMs with fused
    LN prologue / GELU and residual epilogues."""
    rng = np.random.default_rng(seed)
    hid = hidden or 4 * dim
    b = Builder(f"mlp-{dim}x{layers}")
    x = b.input("x", [batch, dim], "fp32")
    h = b.op("cast", x, dtype=dtype) if dtype != "fp32" else x
    for i in range(layers):
        g = b.param(f"l{i}.ln_w", 1.0 + 0.1 * rng.standard_normal(dim), dtype)
        be = b.param(f"l{i}.ln_b", 0.1 * rng.standard_normal(dim), dtype)
        w1 = b.param(f"l{i}.fc1_w", rng.standard_normal((hid, dim)) / math.sqrt(dim), dtype)
        b1 = b.param(f"l{i}.fc1_b", 0.02 * rng.standard_normal(hid), dtype)
        w2 = b.param(f"l{i}.fc2_w", rng.standard_normal((dim, hid)) / math.sqrt(hid), dtype)
        b2 = b.param(f"l{i}.fc2_b", 0.02 * rng.standard_normal(dim), dtype)
        y = b.op("layernorm", h, g, be, eps=1e-5)
        y = b.op("gelu", b.op("linear", y, w1, b1))
        h = b.op("add", b.op("linear", y, w2, b2), h)
    return b.build([h])


__all__ = ["FORMAT", "Program", "CompiledProgram", "ProgramError", "Builder", "parse", "mlp_program", "bf16_bits",
           "save_program", "load_program",
           "bf16_to_f32", "OPS", "torch_dtype"]
