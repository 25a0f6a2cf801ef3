"""The graph compiler: the passes that lower a validated :class:`Program`
onto the nos-amd ops (constant folding, norm folding, epilogue / attention
fusion, merges, plane and LayerNorm hand-offs, last-use release).  The
executor (execute.py) runs the resulting steps."""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

from .graph import Program
from .ir import BINARY, NATIVE_KINDS, NEVER_FOLD, STATE_WRITERS, UNARY, ProgramError, torch_dtype
from .reference import _eager


@dataclass
class _Step:
    kind: str                     # op name or a fused kind: linear_ln | ln_qkv_attention
    inputs: list[str]
    output: str
    attrs: dict
    release: list[str] = field(default_factory=list)   # values whose last use this is


class Lowered:
    """A parsed program lowered onto the nos-amd ops for one device: the
    passes below turn its nodes into ``self.steps`` (the package docstring
    lists them); :class:`execute.CompiledProgram` adds the executor."""

    def __init__(self, prog: Program, device, params: dict | None = None, state: dict | None = None,
                 derived: dict | None = None):
        import torch

        self.program = prog
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.consts: dict[str, object] = dict(params) if params is not None else prog.tensors(self.device)
        # the tenant's state buffers (shared by its variants; updated in place by every run)
        self.state: dict[str, object] = state if state is not None else prog.state_tensors(self.device)
        # derived constants (folded / merged weights) by recipe and source tensors, shared by
        # the variants compiled over the same params: one copy per tenant, not per shape
        self._derived: dict = derived if derived is not None else {}
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
            steps = self._lower_static_positions(steps)
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
            steps = self._fuse_rotary_at(steps)
            steps = self._merge_kv_writes(steps)
            if "kv_into_attention" not in skip:
                steps = self._fuse_kv_write_attention(steps)
            if os.environ.get("NOS_AMD_FOLD_DECODE_COMBINE", "0") == "1":   # opt-in (A/B: slower alone)
                self._fold_decode_combines(steps)
            steps = self._fuse_argmax_pos(steps)
            steps = self._fuse_gemv_glu(steps)
            if "combine_gemv" not in skip:
                steps = self._fold_combine_into_gemv(steps)
            if "cat_buffer" not in skip:
                steps = self._cat_into_buffer(steps)
            steps = self._mark_plane_handoffs(steps)
            steps = self._mark_ln_handoffs(steps)
            self._prep_conv_weights(steps)
            self.steps = self._plan_releases(steps)
            used = {i for s in self.steps for i in s.inputs} | set(self.outputs)
            for k in [k for k in self.consts if k not in used]:  # e.g. weights replaced by their LN-folded form
                del self.consts[k]
        # the memo holds its recipes' SOURCE tensors (raw weights a fold replaced): only the
        # build's variants share it -- a compiled program keeping it would keep them alive
        self._derived = None
        self.stats["kernels"] = sum(1 for s in self.steps if s.kind in NATIVE_KINDS)

    def _memo(self, tag: str, sources: list, extra, make):
        """``make()`` once per recipe: ``tag`` + the identities of the source
        tensors + ``extra`` (hashable).  The sources are held by the cache, so
        an id is never reused by another tensor while it lives."""
        import torch

        key = (tag, tuple(id(t) if torch.is_tensor(t) else t for t in sources), extra)
        hit = self._derived.get(key)
        if hit is None:
            hit = (make(), list(sources))
            self._derived[key] = hit
        return hit[0]

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
                srcs = [self.consts[i] for i in n.inputs]
                self.consts[n.output] = self._memo(
                    "fold:" + n.op, srcs, repr(sorted(n.attrs.items())),
                    lambda n=n, srcs=srcs: _eager(n.op, srcs, n.attrs).contiguous())
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

    def _lower_static_positions(self, steps: list[_Step]) -> list[_Step]:
        """Positions the program fixes itself (``pos_set`` and then ``pos_add``
        by constants) are known at build: a prefill program that starts a
        sequence (position 0) then needs no cache reads --
        ``rotary_at`` becomes ``rotary`` on constant table rows, and an
        ``sdpa_cache`` whose caches were just written from the same keys /
        values at position 0 (Sq = their S) is causal ``sdpa`` on those keys
        and values (the flash kernel; the writes stay, for the decode steps
        after it).  Dynamic positions keep the cache kernels."""
        by_out = {s.output: s for s in steps}
        known: dict[str, int] = {}
        n = 0
        for s in steps:
            if s.kind == "pos_set":
                known[s.output] = int(s.attrs["value"])
            elif s.kind == "pos_add" and s.inputs[0] in known:
                known[s.output] = known[s.inputs[0]] + int(s.attrs["n"])
            elif s.kind == "rotary_at" and s.inputs[3] in known and all(i in self.consts for i in s.inputs[1:3]):
                p0, S = known[s.inputs[3]], self._shape(s.inputs[0])[1]
                if p0 + S > self._shape(s.inputs[1])[0]:
                    continue
                tabs = []
                for t in s.inputs[1:3]:
                    name = f"{t}::rows{p0}:{p0 + S}"
                    if name not in self.consts:
                        self.consts[name] = self._memo("rows", [self.consts[t]], (p0, S),
                                                       lambda t=t: self.consts[t][p0:p0 + S].contiguous())
                    tabs.append(name)
                s.kind, s.inputs = "rotary", [s.inputs[0], *tabs]
                n += 1
            elif s.kind == "sdpa_cache" and known.get(s.inputs[3]) == 0:
                wk, wv = by_out.get(s.inputs[1]), by_out.get(s.inputs[2])
                sq = self._shape(s.inputs[0])[1]
                if (wk is None or wv is None or wk.kind != "kv_write" or wv.kind != "kv_write"
                        or wk.inputs[2] != s.inputs[3] or wv.inputs[2] != s.inputs[3]
                        or self._shape(wk.inputs[1])[1] != sq or self._shape(wv.inputs[1])[1] != sq):
                    continue
                s.kind, s.inputs = "sdpa", [s.inputs[0], wk.inputs[1], wv.inputs[1]]
                s.attrs = {"causal": True, **({"scale": s.attrs["scale"]} if "scale" in s.attrs else {})}
                n += 1
        self.stats["static_positions"] = n
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
        from ...ops.tenant import UNARY_CODES

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
        steps = [s for s in steps if id(s) not in drop]
        # gated units: mul(act(a), b) (SwiGLU's silu(gate) * up) -> ONE glu pass
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, g = set(), 0
        for s in steps:
            if s.kind != "mul":
                continue
            for ia, ib in ((0, 1), (1, 0)):
                p = by_out.get(s.inputs[ia])
                if (p is not None and p.kind in ("silu", "gelu", "relu", "sigmoid") and uses.get(p.output) == 1
                        and p.output not in self.outputs and id(p) not in drop
                        and tuple(self._shape(p.inputs[0])) == tuple(self._shape(s.inputs[ib])) == tuple(self._shape(s.output))
                        and self._dtype(p.inputs[0]) == self._dtype(s.inputs[ib]) in ("fp32", "bf16")):
                    drop.add(id(p))
                    s.kind, s.inputs, s.attrs = "glu", [p.inputs[0], s.inputs[ib]], {"op": p.kind}
                    g += 1
                    break
        self.stats["glu_fused"] = g
        steps = [s for s in steps if id(s) not in drop]
        # every other standalone activation on its native pass (no at::native kernel per replay)
        u = 0
        for s in steps:
            if s.kind in UNARY_CODES and self._dtype(s.inputs[0]) in ("fp32", "bf16"):
                s.attrs = {"op": s.kind, "dtype": self._dtype(s.output)}
                s.kind = "unary"
                u += 1
        self.stats["unary_native"] = u
        return steps

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
            eps = s.attrs.get("eps", 1e-5)
            srcs = [self.consts[i] for i in c.inputs[1:] + s.inputs[1:]]
            self.consts[base + ".w"], self.consts[base + ".b"] = self._memo(
                "bn", srcs, eps, lambda w=w, b=b, inv=inv, mu=mu, be=be: (
                    (w.float() * inv[:, None, None, None]).to(w.dtype).contiguous(),
                    ((b - mu) * inv + be).to(w.dtype).contiguous()))
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
            self.consts[name + ".w"] = self._memo("merge.w", ws, None, lambda ws=ws: torch.cat(ws, dim=0).contiguous())
            ins = [x, name + ".w"]
            if any(len(m.inputs) > 2 for m in g):
                bs = [self.consts[m.inputs[2]] if len(m.inputs) > 2 else None for m in g]
                self.consts[name + ".b"] = self._memo(
                    "merge.b", [*ws, *bs], None, lambda ws=ws, bs=bs: torch.cat(
                        [bb if bb is not None else torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
                         for bb, w in zip(bs, ws)]).contiguous())
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

                    def blockdiag(ws=ws):
                        nrow, ncol = sum(w.shape[0] for w in ws), sum(w.shape[1] for w in ws)
                        wbd = torch.zeros((nrow, ncol), dtype=ws[0].dtype, device=ws[0].device)
                        r = c = 0
                        for w in ws:
                            wbd[r:r + w.shape[0], c:c + w.shape[1]] = w
                            r, c = r + w.shape[0], c + w.shape[1]
                        return wbd

                    m0 = run[0][2]
                    name = f"{m0.output}::blockdiag"
                    self.consts[name + ".w"] = self._memo("blockdiag.w", ws, None, blockdiag)
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
                        bs = [self.consts[m.inputs[2]] if len(m.inputs) > 2 else None for _, _, m in run]
                        self.consts[name + ".b"] = self._memo(
                            "blockdiag.b", [*ws, *bs], None, lambda ws=ws, bs=bs: torch.cat(
                                [bb if bb is not None else torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
                                 for bb, w in zip(bs, ws)]).contiguous())
                        ins.append(name + ".b")
                    new_steps.append(_Step("linear", ins, name, {}))
                    self._new_shapes[name] = tuple(self._shape(x)[:-1]) + (sum(w.shape[0] for w in ws),)
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
        from ... import ops

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
            wg, c1, c2 = self._memo("ln", [w, b, g, be], None, lambda w=w, b=b, g=g, be=be: ops.fold_layernorm(w, b, g, be))
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
            self.consts[base + ".w"] = self._memo(
                "rms", [w, g], None, lambda w=w, g=g: (w.float() * g.float()[None, :]).to(w.dtype).contiguous())
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
        defined = set(self.consts) | {self.input_name} | set(self.state)
        # an in-place state update waits for every earlier reader of the version it overwrites
        readers_before = {}
        for k, s in enumerate(steps):
            if s.kind in STATE_WRITERS:
                readers_before[id(s)] = {id(r) for r in steps[:k] if s.inputs[0] in r.inputs}
        placed: set[int] = set()
        out, pending = [], list(steps)
        while pending:
            for i, s in enumerate(pending):
                if all(x in defined for x in s.inputs) and readers_before.get(id(s), set()) <= placed:
                    out.append(s)
                    defined.add(s.output)
                    placed.add(id(s))
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

    def _fuse_rotary_at(self, steps: list[_Step]) -> list[_Step]:
        """A decode step's rotary at the device-side position: the K rotation
        into its ``kv_write`` (rotated as it is written to the cache) and the Q
        rotation into ``sdpa_cache`` (rotated as the kernel loads it)."""
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind not in ("kv_write", "sdpa_cache") or s.attrs.get("rope"):
                continue
            slot, pos = (1, s.inputs[2]) if s.kind == "kv_write" else (0, s.inputs[3])
            r = by_out.get(s.inputs[slot])
            if (r is None or r.kind != "rotary_at" or uses.get(r.output) != 1 or r.inputs[3] != pos
                    or not all(i in self.consts for i in r.inputs[1:3])):
                continue
            s.inputs = s.inputs[:slot] + [r.inputs[0]] + s.inputs[slot + 1:] + r.inputs[1:3]
            s.attrs = {**s.attrs, "rope": True}
            drop.add(r.output)
            n += 1
        self.stats["rotary_at_fused"] = n
        return [s for s in steps if s.output not in drop]

    def _fuse_gemv_glu(self, steps: list[_Step]) -> list[_Step]:
        """Decode rows (at most 8, known statically): ``glu(silu)`` of the two
        column halves of a merged gate-up ``linear_rms`` becomes that GEMV's
        epilogue (each wave computes a gate and its up column), one launch
        instead of two."""
        from ...ops.tenant import GEMV_MAX_ROWS

        if not self.gpu:
            return steps
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "glu" or s.attrs.get("op") != "silu":
                continue
            a, b = by_out.get(s.inputs[0]), by_out.get(s.inputs[1])
            if a is None or b is None or a.kind != "slice" or b.kind != "slice" or a.inputs != b.inputs:
                continue
            lin = by_out.get(a.inputs[0])
            shp = tuple(self._shape(lin.output)) if lin is not None else ()
            if (lin is None or lin.kind != "linear_rms" or lin.attrs.get("act") or len(lin.inputs) > 2
                    or uses.get(lin.output) != 2 or uses.get(a.output) != 1 or uses.get(b.output) != 1
                    or math.prod(shp[:-1]) > GEMV_MAX_ROWS or shp[-1] % 2
                    or any(t.attrs.get("dim") not in (-1, len(shp) - 1) for t in (a, b))
                    or (a.attrs["start"], a.attrs["end"], b.attrs["start"], b.attrs["end"])
                    != (0, shp[-1] // 2, shp[-1] // 2, shp[-1])):
                continue
            lin.attrs = {**lin.attrs, "glu": True}
            self._new_shapes[lin.output] = shp[:-1] + (shp[-1] // 2,)
            drop |= {id(a), id(b), id(s)}
            rename = {s.output: lin.output}
            for t in steps:
                t.inputs = [rename.get(i, i) for i in t.inputs]
            self.outputs = [rename.get(o, o) for o in self.outputs]
            n += 1
        self.stats["gemv_glu_fused"] = n
        return [s for s in steps if id(s) not in drop]

    def _merge_kv_writes(self, steps: list[_Step]) -> list[_Step]:
        """A layer's K and V cache writes at the same position (the K one
        rotated, the V one plain) in ONE launch: the V write's step becomes
        the pair (it comes later, so both inputs exist) and names the K
        cache's new version too."""
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "sdpa_cache":
                continue
            wk, wv = by_out.get(s.inputs[1]), by_out.get(s.inputs[2])
            if (wk is None or wv is None or wk.kind != "kv_write" or wv.kind != "kv_write" or id(wk) in drop
                    or wv.attrs.get("rope") or wv.attrs.get("pair") or wk.inputs[2] != wv.inputs[2]
                    or tuple(self._shape(wk.inputs[1])) != tuple(self._shape(wv.inputs[1]))
                    or tuple(self._shape(wk.inputs[0])) != tuple(self._shape(wv.inputs[0]))
                    or self._dtype(wk.inputs[0]) != self._dtype(wv.inputs[0])
                    or steps.index(wk) > steps.index(wv)):
                continue
            wv.inputs = wk.inputs + [wv.inputs[0], wv.inputs[1]]   # K cache, K x, pos, [cos, sin], V cache, V x
            wv.attrs = {"pair": True, "rope": bool(wk.attrs.get("rope")), "k_out": wk.output}
            drop.add(id(wk))
            n += 1
        self.stats["kv_writes_paired"] = n
        return [s for s in steps if id(s) not in drop]

    def _fuse_kv_write_attention(self, steps: list[_Step]) -> list[_Step]:
        """GPU: a layer's paired K / V cache write whose new cache versions only
        its ``sdpa_cache`` reads, at the same positions and (K and q) with the
        same rotary tables, folds into that attention launch: the decode kernel
        writes the step's rows into the caches itself and attends them from
        registers (decode.hip ``Fresh``) -- one launch per layer fewer."""
        if not self.gpu:
            return steps
        uses = self._consumers(steps, self.outputs)
        by_out = {s.output: s for s in steps}
        drop, n = set(), 0
        for s in steps:
            if s.kind != "sdpa_cache" or s.attrs.get("fresh"):
                continue
            w = by_out.get(s.inputs[2])
            if w is None or w.kind != "kv_write" or not w.attrs.get("pair") or s.inputs[1] != w.attrs.get("k_out"):
                continue
            rope = bool(w.attrs.get("rope"))
            r = 5 if rope else 3                      # w: K cache, K x, pos, [cos, sin], V cache, V x
            if (rope != bool(s.attrs.get("rope")) or s.inputs[3] != w.inputs[2]
                    or (rope and list(w.inputs[3:5]) != list(s.inputs[4:6]))
                    or uses.get(w.output) != 1 or uses.get(w.attrs["k_out"]) != 1
                    or uses.get(w.inputs[0]) != 1 or uses.get(w.inputs[r]) != 1
                    or tuple(self._shape(w.inputs[1]))[1] != tuple(self._shape(s.inputs[0]))[1]):
                continue
            s.inputs = [s.inputs[0], w.inputs[0], w.inputs[r], s.inputs[3]] + (list(s.inputs[4:6]) if rope else []) \
                + [w.inputs[1], w.inputs[r + 1]]
            s.attrs = {**s.attrs, "fresh": True}
            drop.add(id(w))
            n += 1
        self.stats["kv_writes_into_attention"] = n
        return [s for s in steps if id(s) not in drop]

    def _fold_decode_combines(self, steps: list[_Step]) -> None:
        """GPU: every ``sdpa_cache`` gets its own zeroed counters (B x Hkv
        int32, kept with the program): the flash-decoding split combine then
        runs in the decode launch's last workgroup per K / V head
        (decode.hip ``decode_combine_last``) -- one launch per layer fewer.
        Opt-in (``NOS_AMD_FOLD_DECODE_COMBINE=1``): one decoder alone ran
        0.69-0.74 ms / token with it against 0.65 without (every workgroup's
        device-scope release writes its XCD's L2 back), 8 decoders 2.63 against
        2.70 ms (``profiles/r06_decode_combine_fold_ab.json``)."""
        import torch

        if not self.gpu:
            return
        n = 0
        for s in steps:
            if s.kind != "sdpa_cache":
                continue
            B, Hkv = tuple(self._shape(s.inputs[1]))[0], tuple(self._shape(s.inputs[1]))[2]
            name = s.output + "::sync"
            self.aux[name] = torch.zeros(B * Hkv, dtype=torch.int32, device=self.device)
            s.attrs = {**s.attrs, "sync": name}
            n += 1
        self.stats["decode_combines_folded"] = n

    def _fold_combine_into_gemv(self, steps: list[_Step]) -> list[_Step]:
        """GPU: a one-token fp32 ``sdpa_cache`` whose output only its layer's
        O-projection reads (through a reshape to [B, 1, H x D], B <= 8) leaves
        its split partials to that GEMV, which combines them while it stages
        x (``ops.tenant.gemv_partials``, decode.hip ``parts_x4``, the combine
        kernel's arithmetic) -- the combine launch of each layer folded away."""
        if not self.gpu:
            return steps
        uses = self._consumers(steps, self.outputs)
        by_input: dict[str, list[_Step]] = {}
        for t in steps:
            for i in t.inputs:
                by_input.setdefault(i, []).append(t)
        drop, n = set(), 0
        for s in steps:
            if s.kind != "sdpa_cache" or s.attrs.get("sync") or uses.get(s.output) != 1:
                continue
            shp = tuple(self._shape(s.output))
            if len(shp) != 4 or shp[1] != 1 or shp[0] > 8 or shp[3] not in (64, 128) or self._dtype(s.output) != "fp32":
                continue
            r = by_input.get(s.output, [None])[0]
            if r is None or r.kind != "reshape" or uses.get(r.output) != 1:
                continue
            rs = tuple(self._shape(r.output))
            if rs[0] != shp[0] or math.prod(rs[1:]) != shp[2] * shp[3] or rs[-1] != shp[2] * shp[3]:
                continue
            lin = by_input.get(r.output, [None])[0]
            if (lin is None or lin.kind != "linear" or lin.inputs[0] != r.output or lin.attrs.get("out_into")
                    or lin.attrs.get("row_stats") or lin.attrs.get("planes_out") or lin.attrs.get("act") == "glu"):
                continue
            s.attrs = {**s.attrs, "partials": True}
            lin.inputs = [s.output] + lin.inputs[1:]
            lin.attrs = {**lin.attrs, "x_partials": True}
            drop.add(id(r))
            n += 1
        self.stats["decode_combines_into_gemv"] = n
        return [t for t in steps if id(t) not in drop]

    def _fuse_argmax_pos(self, steps: list[_Step]) -> list[_Step]:
        """GPU: a step's closing ``pos_add`` folds into the ``argmax`` right
        before it when argmax has one row per counter and nothing between
        them reads the counter (the decode step's last two launches become
        one; argmax reads no position)."""
        if not self.gpu:
            return steps
        uses = self._consumers(steps, self.outputs)
        for k, p in enumerate(steps):
            if p.kind != "pos_add" or k == 0:
                continue
            a = steps[k - 1]
            shp = tuple(self._shape(a.inputs[0])) if a.kind == "argmax" else ()
            pshape = tuple(self._shape(p.inputs[0]))
            if (a.kind != "argmax" or a.attrs.get("pos_out") or len(pshape) != 1 or not shp
                    or math.prod(shp[:-1]) != pshape[0] or uses.get(p.output, 0) != 0
                    or self._dtype(p.inputs[0]) != "i32"):
                continue
            a.inputs = a.inputs + [p.inputs[0]]
            a.attrs = {**a.attrs, "pos_out": p.output, "pos_n": int(p.attrs["n"])}
            self.stats["pos_add_into_argmax"] = 1
            return steps[:k] + steps[k + 1:]
        self.stats["pos_add_into_argmax"] = 0
        return steps

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
            kp = -(-k // 32) * 32
            name = s.inputs[1] + "::mat"

            def mat(w=w, k=k, kp=kp):
                w2 = w.float().reshape(w.shape[0], k)
                return (F.pad(w2, (0, kp - k)) if kp != k else w2).contiguous()

            self.aux[name] = self._memo("conv.mat", [w], None, mat)
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
        cats of fp32 rows whose width is whole statistics parts (``ops.stats_pw()``) only."""
        import torch

        p = by_out.get(c.inputs[0])
        buf = self.aux[c.attrs["buf"]]
        shape = tuple(buf.shape)
        into = p.attrs.get("out_into") if p is not None else None
        from ... import ops

        pw = ops.stats_pw() if self.gpu else 128   # the producer GEMM's statistics part width (its tile width)
        if (p is None or p.kind != "linear" or into is None or buf.dtype != torch.float32 or len(shape) < 2
                or into[1] % len(shape) != len(shape) - 2 or shape[-1] % pw or math.prod(shape[:-2]) != 1):
            return False
        rows = buf.reshape(-1, shape[-1]).double().view(shape[-2], shape[-1] // pw, pw)
        mean = rows.mean(-1)
        st = torch.stack([mean, ((rows - mean[..., None]) ** 2).sum(-1)], dim=-1).float().contiguous()
        name = c.attrs["buf"] + "::stats"
        self.aux[name] = st
        c.attrs["stats"] = name
        c.attrs["stats_pw"] = pw
        p.attrs["row_stats"] = True
        p.attrs["stats_into"] = name
        return True

    def _plan_releases(self, steps: list[_Step]) -> list[_Step]:
        last: dict[str, int] = {}
        for k, s in enumerate(steps):
            for i in s.inputs:
                last[i] = k
        keep = set(self.outputs) | set(self.consts) | {self.input_name} | set(self.state)
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

