"""The executor of a compiled program: ``CompiledProgram(x)`` runs its
steps on the gfx950 kernels (stream-ordered only, so the server captures it
into a HIP graph)."""
from __future__ import annotations

from .compile import Lowered
from .ir import torch_dtype
from .reference import _eager, _pair2


class CompiledProgram(Lowered):
    """A parsed program lowered onto the nos-amd ops for one device (see the
    package docstring for the passes).  ``__call__(x)`` returns the outputs as
    a tuple; it launches only stream-ordered work, so it can be captured into
    a HIP graph."""

    # ------------------------------------------------------------ run
    def __call__(self, x) -> tuple:
        from ... import ops
        from ...ops import tenant as T

        env = dict(self.consts)
        env.update(self.state)
        env[self.input_name] = x
        for s in self.steps:
            a = [env[i] for i in s.inputs]
            k = s.kind
            if k == "linear" and s.attrs.get("x_partials"):   # x = the decode attention's split partials
                res = a.pop() if s.attrs.get("residual") else None
                y = T.gemv_partials(a[0], a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"),
                                    residual=res).reshape(self._shape(s.output))
            elif k == "linear":
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
                y = T.linear_rms(a[0], a[1], a[2] if len(a) > 2 else None, act=s.attrs.get("act"), eps=s.attrs["eps"],
                                 glu=bool(s.attrs.get("glu")))
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
                D = xx.shape[-1]
                if xx.is_cuda and str(xx.dtype) == "torch.bfloat16" and D % 8 == 0 and D <= 4096:   # 16-B rows
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
            elif k == "glu":
                y = T.glu(a[0], a[1], s.attrs["op"])
            elif k == "kv_write" and s.attrs.get("pair"):   # K (maybe rotated) and V of one layer, one launch
                r = 5 if s.attrs.get("rope") else 3
                env[s.attrs["k_out"]] = T.kv_write(a[0], a[1], a[2], rope=(a[3], a[4]) if s.attrs.get("rope") else None,
                                                   second=(a[r], a[r + 1]))
                y = a[r]
            elif k == "kv_write":
                y = T.kv_write(a[0], a[1], a[2], rope=(a[3], a[4]) if s.attrs.get("rope") else None)
            elif k == "sdpa_cache":
                y = T.sdpa_cache(a[0], a[1], a[2], a[3], scale=s.attrs.get("scale"),
                                 rope=(a[4], a[5]) if s.attrs.get("rope") else None,
                                 fresh=(a[-2], a[-1]) if s.attrs.get("fresh") else None,
                                 sync=self.aux.get(s.attrs.get("sync")), partials=bool(s.attrs.get("partials")))
            elif k == "rotary_at":
                y = T.rotary_at(a[0], a[1], a[2], a[3])
            elif k in ("pos_add", "pos_set"):
                y = T.pos_update(a[0], add=k == "pos_add", n=int(s.attrs["n" if k == "pos_add" else "value"]))
            elif k == "argmax" and s.attrs.get("pos_out"):   # the step's pos_add folded in
                y = T.argmax(a[0], pos=a[1], pos_n=int(s.attrs["pos_n"]))
                env[s.attrs["pos_out"]] = a[1]
            elif k == "argmax":
                y = T.argmax(a[0])
            elif k == "cat_buffer":  # its GEMM part was written in place; the constant parts at build
                y = self.aux[s.attrs["buf"]]
                if env.pop(s.inputs[0] + "::lnp", None) is not None:
                    # the GEMM wrote its rows' statistics into the buffer's stats, whose
                    # constant rows were filled at build: the whole buffer's, for its LN-GEMM
                    env[s.output + "::lnp"] = ops.RowStats(self.aux[s.attrs["stats"]], s.attrs.get("stats_pw", 128))
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

