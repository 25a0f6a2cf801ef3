"""Validation of a wire program: shape / dtype inference per op (with the
gfx950 kernels' constraints on a GPU), topological order and payload layout
-- everything is checked before a byte of device memory is allocated."""
from __future__ import annotations

import math

from .graph import Program
from .ir import (FLOAT_DTYPES, FORMAT, MAX_NUMEL, MAX_PARAMS, MAX_NODES, MAX_RANK, MAX_STATE, MAX_VARIANTS, OPS,
                 STATE_DTYPES, STATE_WRITERS, ACTS, BINARY,
                 INTERP_MODES, UNARY, WIRE_DTYPES, Node, ProgramError, Value, _broadcast, _eps, _int, _name,
                 _pair, _req, _shape)


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
    if op == "kv_write":
        # cache [B, L, Hkv, D] <- x [B, S, Hkv, D] at rows pos[b] .. pos[b] + S - 1 (rows past L are dropped)
        only()
        arity(3, 3)
        c, x, p = ins
        _req(len(c.shape) == 4 and c.dtype in FLOAT_DTYPES, f"{what}: the cache must be a float [B, L, Hkv, D] state")
        _req(len(x.shape) == 4 and x.shape[0] == c.shape[0] and x.shape[2:] == c.shape[2:] and x.dtype == c.dtype
             and x.shape[1] <= c.shape[1], f"{what}: x must be [{c.shape[0]}, S <= {c.shape[1]}, {c.shape[2]}, "
             f"{c.shape[3]}] {c.dtype}, got {x.shape} {x.dtype}")
        _pos_vector(p, c.shape[0], what)
        return c.shape, c.dtype
    if op == "sdpa_cache":
        # q [B, Sq, H, D] at positions pos[b] + i over the cached keys 0 .. pos[b] + i (causal)
        only("scale")
        arity(4, 4)
        q, kc, vc, p = ins
        _req(len(q.shape) == 4 and len(kc.shape) == 4 and kc.shape == vc.shape and kc.dtype == vc.dtype
             and q.shape[0] == kc.shape[0] and q.shape[3] == kc.shape[3] and q.shape[2] % kc.shape[2] == 0
             and q.shape[1] <= kc.shape[1] and q.dtype in FLOAT_DTYPES and kc.dtype in FLOAT_DTYPES,
             f"{what}: q [B, Sq, H, D], caches [B, L >= Sq, Hkv, D] with H % Hkv == 0 required, got {q.shape}, "
             f"{kc.shape}")
        _pos_vector(p, q.shape[0], what)
        if "scale" in a:
            _req(isinstance(a["scale"], (int, float)) and not isinstance(a["scale"], bool) and a["scale"] > 0,
                 f"{what}: scale must be > 0")
        if gpu:
            _req(q.shape[3] in (64, 128), f"{what}: the decode attention kernel takes head_dim 64 or 128")
            _req(q.shape[2] // kc.shape[2] <= 16, f"{what}: at most 16 query heads per K / V head")
        return q.shape, q.dtype
    if op == "rotary_at":
        only()
        arity(4, 4)
        x, c, sn, p = ins
        _req(len(x.shape) == 4 and x.shape[3] % 2 == 0 and x.dtype in FLOAT_DTYPES,
             f"{what}: x must be [B, S, H, D] with D even")
        _req(len(c.shape) == 2 and c.shape == sn.shape and c.shape[1] == x.shape[3] and c.dtype == sn.dtype == "fp32",
             f"{what}: cos / sin must be fp32 [positions, {x.shape[3]}]")
        _pos_vector(p, x.shape[0], what)
        return x.shape, x.dtype
    if op in ("pos_add", "pos_set"):
        only("n" if op == "pos_add" else "value")
        arity(1, 1)
        _req(ins[0].dtype == "i32" and len(ins[0].shape) == 1, f"{what}: takes an i32 [B] position state")
        v = a.get("n" if op == "pos_add" else "value")
        _req(isinstance(v, int) and not isinstance(v, bool) and 0 <= v <= 1 << 24,
             f"{what}: {'n' if op == 'pos_add' else 'value'} must be an int in [0, 2^24]")
        return ins[0].shape, "i32"
    if op == "argmax":
        only("dim")
        arity(1, 1)
        _req(a.get("dim", -1) in (-1, len(ins[0].shape) - 1) and len(ins[0].shape) >= 1,
             f"{what}: argmax runs over the last dim")
        _req(ins[0].dtype in FLOAT_DTYPES, f"{what}: takes a float tensor")
        return ins[0].shape[:-1], "i32"
    raise ProgramError(f"{what}: op {op!r} is not one the pod server runs (whitelist: {' '.join(OPS)})")


def _pos_vector(p: Value, b: int, what: str) -> None:
    _req(p.dtype == "i32" and p.shape == (b,), f"{what}: pos must be an i32 [{b}] (a position state), got {p.shape}")



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
        _req({k: (v.shape, v.dtype) for k, v in p.state.items()} == {k: (v.shape, v.dtype) for k, v in p0.state.items()},
             f"variant {p.name!r} declares other state than {p0.name!r}: variants share one state")
        _req(p.inputs[0].shape not in seen, f"two variants take the input shape {list(p.inputs[0].shape)}")
        seen.add(p.inputs[0].shape)
    return progs


def parse(obj: dict, payload: bytes | memoryview = b"", gpu: bool = False) -> Program:
    """Validate a wire program (see the module docstring) against its payload;
    ``gpu``: also check the native kernels' shape constraints."""
    _req(isinstance(obj, dict), "program must be a JSON object")
    _req(obj.get("format") == FORMAT, f"program format must be {FORMAT!r}")
    extra = set(obj) - {"format", "name", "inputs", "params", "state", "nodes", "outputs", "meta"}
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
    st = obj.get("state", [])
    _req(isinstance(st, list) and len(st) <= MAX_STATE, f"state must be a list of at most {MAX_STATE}")
    state: dict[str, Value] = {}
    for d in st:
        _req(isinstance(d, dict) and set(d) <= {"name", "shape", "dtype"}, "a state is {name, shape, dtype}")
        dt = d.get("dtype", "fp32")
        _req(dt in STATE_DTYPES, f"state dtype must be one of {STATE_DTYPES}")
        v = Value(_name(d.get("name"), "state name"), _shape(d.get("shape"), "state shape"), dt, "state")
        define(v)
        state[v.name] = v
    # state versions: root name -> its current version; an in-place writer's
    # output becomes the current version and the one it consumed is dead
    current = {k: k for k in state}
    root_of = {k: k for k in state}
    dead: set[str] = set()
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
            _req(r not in dead, f"node of op {op}: state version {r!r} was updated in place before this node "
                 f"(use {current.get(root_of.get(r, r), r)!r})")
        attrs = d.get("attrs") or {}
        _req(isinstance(attrs, dict), "attrs must be an object")
        n = Node(op, list(refs), _name(d.get("output"), "node output"), dict(attrs))
        shape, dt = _infer(n, [values[r] for r in refs], gpu)
        _req(math.prod(shape) <= MAX_NUMEL, f"node {n.output!r}: output too large")
        if op in STATE_WRITERS:
            tgt = refs[0]
            _req(tgt in root_of, f"node {n.output!r} ({op}): updates a state in place; {tgt!r} is not one")
            _req(refs.count(tgt) == 1, f"node {n.output!r} ({op}): the updated state cannot also be an operand")
            dead.add(tgt)
            root_of[n.output] = root_of[tgt]
            current[root_of[tgt]] = n.output
        define(Value(n.output, shape, dt, "node"))
        nodes.append(n)
    outs = obj.get("outputs")
    _req(isinstance(outs, list) and outs and all(isinstance(o, str) and o in values for o in outs),
         "outputs must name defined values")
    _req(not any(o in root_of for o in outs), "a state (or a version of one) cannot be an output: it is mutable")
    return Program(name, inputs, params, layout, nodes, list(outs), values, payload, state=state,
                   state_root={k: v for k, v in root_of.items() if k != v})

