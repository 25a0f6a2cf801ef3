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

The compiled program is a callable ``(x) -> tuple(outputs)``, captured into a
HIP graph by the server exactly like a built-in model.  :meth:`Program.reference`
runs the unfused graph eagerly in fp32 (the numerics reference of tests).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

FORMAT = "nos-amd.program/v1"
WIRE_DTYPES = {"fp32": 4, "bf16": 2}
MAX_NODES = 8192
MAX_PARAMS = 8192
MAX_NUMEL = 1 << 31          # elements of one value
MAX_RANK = 8
UNARY = ("gelu", "relu", "sigmoid", "silu")
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
        _req(len(w.shape) == 2 and len(x.shape) >= 1 and x.shape[-1] == w.shape[1],
             f"{what}: x [..., K] and weight [N, K] required, got {x.shape} and {w.shape}")
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
        _req(ins[1].shape == (d,) and ins[2].shape == (d,), f"{what}: gamma/beta must be [{d}]")
        eps = a.get("eps", 1e-5)
        _req(isinstance(eps, (int, float)) and 0 < eps < 1, f"{what}: eps must be in (0, 1)")
        return ins[0].shape, dt
    if op == "attention":
        only("heads", "scale")
        arity(1, 1)
        x = ins[0]
        h = _int(a.get("heads"), f"{what}: heads", 1)
        _req(len(x.shape) == 3 and x.shape[2] % (3 * h) == 0,
             f"{what}: qkv must be [B, S, 3*heads*D], got {x.shape} with {h} heads")
        d = x.shape[2] // (3 * h)
        if "scale" in a:
            _req(isinstance(a["scale"], (int, float)) and a["scale"] > 0, f"{what}: scale must be > 0")
        if gpu:
            _req(d == 64, f"{what}: the attention kernels are built for head_dim 64, got {d}")
        return (x.shape[0], x.shape[1], h * d), x.dtype
    if op in ("add", "mul"):
        only()
        arity(2, 2)
        return _broadcast(ins[0].shape, ins[1].shape, what), same_dtype()
    if op in UNARY:
        only()
        arity(1, 1)
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
        _req(a.get("dtype") in WIRE_DTYPES, f"{what}: dtype must be one of {sorted(WIRE_DTYPES)}")
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
    raise ProgramError(f"{what}: op {op!r} is not one the pod server runs "
                       f"(whitelist: linear layernorm attention add mul {' '.join(UNARY)} cat slice reshape permute "
                       f"expand cast interpolate)")


OPS = ("linear", "layernorm", "attention", "add", "mul", *UNARY, "cat", "slice", "reshape", "permute", "expand",
       "cast", "interpolate")
NEVER_FOLD = ("attention",)
GEMM_OPS = ("linear",)


def _workspace(node: Node, ins: list[Value], out: Value, f32_math: str) -> int:
    """Transient device bytes one op allocates while it runs, beyond its
    inputs and output (an upper bound; :meth:`Program.bytes_estimate_for`)."""
    op = node.op
    if op == "linear" and ins[0].dtype == "fp32" and f32_math == "h3":
        m = ins[0].numel // ins[0].shape[-1]
        return ins[0].nbytes + 4 * m                       # A's fp16 planes + row scales
    if op == "attention":
        b, s, three_hd = ins[0].shape
        hd = three_hd // 3
        skvp = -(-s // 32) * 32
        return b * skvp * 6 * hd * 2 + 4 * b * s * (hd + 2 * node.attrs["heads"]) * 4 + ins[0].nbytes
    return 0


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
        x = torch.zeros(v.shape, dtype=torch_dtype(v.dtype)) if data is None else \
            torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32)).view(v.shape).to(torch_dtype(v.dtype))
        return x.to(device)

    # ------------------------------------------------------------ execution
    def compile(self, device, params: dict | None = None) -> "CompiledProgram":
        return CompiledProgram(self, device, params)

    def reference(self, x, params: dict | None = None) -> tuple:
        """Eager, unfused, fp32 evaluation of the graph on the CPU (the
        numerics reference: every op in plain PyTorch)."""
        import torch

        ps = params if params is not None else self.tensors("cpu")
        env = {k: t.float().cpu() for k, t in ps.items()}
        env[self.inputs[0].name] = x.float().cpu()
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

    return {"fp32": torch.float32, "bf16": torch.bfloat16}[dt]


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
        _req(dt in WIRE_DTYPES, f"param dtype must be one of {sorted(WIRE_DTYPES)}")
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
        return ops.attention_qkv(args[0].contiguous(), attrs["heads"], scale=attrs.get("scale"))
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
    raise ProgramError(f"op {op!r}")


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
        with torch.no_grad():
            steps = self._fold_constants(prog)
            steps = self._fold_layernorm(steps)
            steps = self._fuse_epilogues(steps)
            steps = self._fuse_qkv_attention(steps)
            steps = self._mark_plane_handoffs(steps)
            self.steps = self._plan_releases(steps)
            used = {i for s in self.steps for i in s.inputs} | set(self.outputs)
            for k in [k for k in self.consts if k not in used]:  # e.g. weights replaced by their LN-folded form
                del self.consts[k]
        self.stats["kernels"] = sum(1 for s in self.steps if s.kind in ("linear", "linear_ln", "ln_qkv_attention",
                                                                           "attention", "layernorm"))

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

    def _fuse_epilogues(self, steps: list[_Step]) -> list[_Step]:
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        rename: dict[str, str] = {}
        keep = []
        n_act = n_res = 0
        for s in steps:
            s.inputs = [rename.get(i, i) for i in s.inputs]
            src = by_out.get(s.inputs[0]) if s.inputs else None
            if (s.kind in ("gelu", "relu") and src is not None and src.kind in ("linear", "linear_ln")
                    and uses.get(src.output) == 1 and not src.attrs.get("act") and "residual" not in src.attrs):
                src.attrs["act"] = s.kind
                rename[s.output] = src.output
                n_act += 1
                continue
            if s.kind == "add":
                a, b = s.inputs
                for prod, other in ((a, b), (b, a)):
                    p = by_out.get(prod)
                    if (p is not None and p.kind == "linear" and uses.get(prod) == 1 and "residual" not in p.attrs
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
            s.kind = "ln_qkv_attention"
            s.attrs = {"heads": s.attrs["heads"], "eps": p.attrs["eps"]}
            s.inputs = list(p.inputs)
            drop.add(p.output)
            n += 1
        self.stats["qkv_attention_fused"] = n
        return [s for s in steps if s.output not in drop]

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
        v = self.program.values.get(name)
        return v.shape if v is not None else tuple(self.consts[name].shape)

    def _dtype(self, name: str):
        v = self.program.values.get(name)
        return v.dtype if v is not None else str(self.consts[name].dtype)

    # ------------------------------------------------------------ run
    def __call__(self, x) -> tuple:
        from .. import ops

        env = dict(self.consts)
        env[self.input_name] = x
        for s in self.steps:
            a = [env[i] for i in s.inputs]
            k = s.kind
            if k == "linear":
                res = a.pop() if s.attrs.get("residual") else None
                if isinstance(a[0], ops.H3Planes):
                    y = ops.linear_planes(a[0], a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                          residual=res)
                else:
                    y = ops.linear(a[0].contiguous(), a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                   residual=res)
            elif k == "linear_ln":
                xx = a[0].contiguous()
                if (s.attrs.get("planes_out") and xx.is_cuda and xx.dtype.itemsize == 4
                        and ops.h3_planes_active()):
                    y = ops.linear_ln_to_planes(xx, a[1], a[2], a[3], act=s.attrs.get("act"), eps=s.attrs["eps"])
                else:
                    y = ops.linear_ln(xx, a[1], a[2], a[3], act=s.attrs.get("act"), eps=s.attrs["eps"])
            elif k == "ln_qkv_attention":
                h = a[0].contiguous()
                if ops.ln_qkv_fusable(h):
                    y = ops.ln_qkv_attention(h, a[1], a[2], a[3], s.attrs["heads"], eps=s.attrs["eps"],
                                             planes_out=bool(s.attrs.get("planes_out"))
                                             and ops.h3_planes_active(attention=True))
                else:
                    qkv = ops.linear_ln(h, a[1], a[2], a[3], eps=s.attrs["eps"])
                    y = ops.attention_qkv(qkv, s.attrs["heads"])
            elif k == "attention":
                y = ops.attention_qkv(a[0].contiguous(), s.attrs["heads"], scale=s.attrs.get("scale"))
            elif k == "layernorm":
                xx = a[0].contiguous()
                if xx.is_cuda and str(xx.dtype) == "torch.bfloat16":
                    y, _ = ops.layernorm(xx, a[1], a[2], s.attrs.get("eps", 1e-5))
                else:
                    import torch.nn.functional as F

                    y = F.layer_norm(xx, (xx.shape[-1],), a[1], a[2], s.attrs.get("eps", 1e-5))
            else:
                y = _eager(k, a, s.attrs)
            env[s.output] = y
            for r in s.release:
                env.pop(r, None)
        return tuple(env[o] for o in self.outputs)


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
           "bf16_to_f32", "OPS", "torch_dtype"]
