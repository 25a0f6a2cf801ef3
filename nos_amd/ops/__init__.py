"""Hot ops of the nos-amd tenant workloads and probes.

Every op has two implementations:

* the gfx950 HIP kernel in ``libnos_hip.so`` (used for every CUDA/ROCm
  tensor -- there is no silent fallback on a GPU: a missing library raises);
* a plain PyTorch fp32 reference (used for CPU tensors and by the numerics
  tests, which compare the HIP kernel against it).
"""
from __future__ import annotations

import math
from typing import NamedTuple

import torch
import torch.nn.functional as F

from . import _lib

EPI_BIAS, EPI_GELU, EPI_RESID, EPI_RELU = 1, 2, 4, 8


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


# ----------------------------------------------------------------- references
def linear_ref(x, weight, bias=None, act=None, residual=None):
    y = x.float() @ weight.float().t()
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y)
    elif act == "relu":
        y = F.relu(y)
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype)


def layernorm_ref(x, gamma, beta, eps=1e-12, residual=None):
    s = x.float() if residual is None else (x.float() + residual.float())
    if residual is not None:
        s = s.to(x.dtype).float()
    y = F.layer_norm(s, (s.shape[-1],), gamma.float(), beta.float(), eps)
    return y.to(x.dtype), (s.to(x.dtype) if residual is not None else None)


def attention_ref(q, k, v, scale=None):
    """q,k,v: [B, S, H, D] -> [B, S, H, D] (fp32 math)."""
    d = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    p = torch.softmax((qf @ kf.transpose(-1, -2)) * scale, dim=-1)
    return (p @ vf).transpose(1, 2).to(q.dtype)


# ---------------------------------------------------------------- dispatchers
def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           act: str | None = None, residual: torch.Tensor | None = None,
           out: torch.Tensor | None = None, max_wg: int = 0, row_stats: bool = False):
    """y = act(x @ weight^T + bias) + residual; x [..., K], weight [N, K].
    ``row_stats`` (fp32 under h3 math): also return y's row statistics for
    the next LN-GEMM, ``(y, RowStats)`` (:func:`linear_planes`)."""
    if row_stats:
        if not (x.is_cuda and x.dtype == torch.float32 and _F32_MATH == "h3"):
            raise ValueError("row_stats needs an fp32 CUDA input under h3 math")
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if x2.stride(-1) != 1 or K % 32:
            raise ValueError("row_stats needs unit inner stride and K % 32 == 0")
        ap, rinv = _split_rows_h3(x2, ln=False)
        return linear_planes(H3Planes(ap, rinv, 0.0, tuple(x.shape)), weight, bias, act, residual, row_stats=True)
    if not x.is_cuda:
        return linear_ref(x, weight, bias, act, residual)
    K = x.shape[-1]
    N = weight.shape[0]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if M <= _GEMV_ROWS and weight.dim() == 2 and weight.shape[1] == K:
        from . import tenant as T

        if T.gemv_ok(x2, weight) and (bias is None or bias.is_contiguous()):
            # a decode step's skinny GEMM: weight-streaming, exact fp32 math
            o2, r2 = _gemm_io(x, weight, out, residual, M, N, K)
            T.gemv(x2, weight, bias, act, r2, out=o2)
            return o2.view(*x.shape[:-1], N)
    if x.dtype == torch.float32:
        return _linear_f32(x, x2, weight, bias, act, residual, out, M, N, K)
    if x2.stride(-1) != 1 or weight.stride(-1) != 1 or K % 64 or x.dtype != torch.bfloat16:
        raise ValueError("native linear needs bf16, unit inner stride and K % 64 == 0")
    o2, r2 = _gemm_io(x, weight, out, residual, M, N, K)
    epi = _epi(bias, act, residual)
    rc = _lib.lib().nos_gemm_bf16(x2.data_ptr(), x2.stride(0), weight.data_ptr(), weight.stride(0),
                                  _ptr(bias), _ptr(r2), r2.stride(0) if r2 is not None else 0,
                                  o2.data_ptr(), o2.stride(0), M, N, K, epi, max_wg, _stream())
    _lib.check(rc, "nos_gemm_bf16")
    return o2.view(*x.shape[:-1], N)


def _epi(bias, act, residual) -> int:
    e = EPI_BIAS if bias is not None else 0
    e |= EPI_GELU if act == "gelu" else (EPI_RELU if act == "relu" else 0)
    return e | (EPI_RESID if residual is not None else 0)


def _check_f32(**ts) -> None:
    for name, t in ts.items():
        if t is not None and (t.dtype != torch.float32 or t.stride(-1) != 1):
            raise ValueError(f"native fp32 GEMM: {name} must be fp32 with unit inner stride")


def _gemm_io(x: torch.Tensor, weight: torch.Tensor, out: torch.Tensor | None, residual: torch.Tensor | None,
             M: int, N: int, K: int) -> tuple[torch.Tensor, torch.Tensor | None]:
    """Shape/dtype checks every native GEMM does before launching: the kernels
    write M x N elements of x's dtype through raw pointers, so a short, mistyped
    or non-viewable ``out`` would corrupt GPU memory or silently lose the result.
    Returns (out as a [M, N] view, residual as [M, N] or None)."""
    if weight.dim() != 2 or weight.shape[1] != K:
        raise ValueError(f"weight must be [N, {K}], got {tuple(weight.shape)}")
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if out.dtype != x.dtype or out.device != x.device:
        raise ValueError(f"out must be {x.dtype} on {x.device}, got {out.dtype} on {out.device}")
    if out.shape[-1] != N or out.numel() != M * N:
        raise ValueError(f"out must hold [{M}, {N}], got {tuple(out.shape)}")
    try:
        o2 = out.view(-1, N)
    except RuntimeError as e:  # a reshape copy would be written and dropped
        raise ValueError("out must be viewable as [M, N] (no copy)") from e
    if o2.stride(-1) != 1:
        raise ValueError("out must have unit inner stride")
    r2 = None
    if residual is not None:
        if residual.shape[-1] != N or residual.numel() != M * N or residual.dtype != x.dtype:
            raise ValueError(f"residual must be [{M}, {N}] of {x.dtype}, got {tuple(residual.shape)} {residual.dtype}")
        r2 = residual.reshape(-1, N)
    return o2, r2


def _linear_f32(x, x2, weight, bias, act, residual, out, M, N, K):
    """fp32 GEMM with fused bias/act/residual: the exact-f32 MFMA kernel
    (csrc/hip/gemm_f32.hip) or, under ``set_f32_math("x6")``, the bf16x6 split
    kernel (gemm_f32x.hip) on the weight's cached bf16 planes."""
    _check_f32(x=x2, weight=weight, bias=bias)
    if K % 32:
        raise ValueError("native fp32 linear needs K % 32 == 0")
    if bias is not None and not bias.is_contiguous():
        raise ValueError("bias must be contiguous")
    o2, r2 = _gemm_io(x, weight, out, residual, M, N, K)
    _check_f32(residual=r2)
    ldr = r2.stride(0) if r2 is not None else 0
    if _F32_MATH == "h3" and M > H3_MIN_ROWS:
        ap, rinv = _split_rows_h3(x2, ln=False)
        _gemm_h3(ap, rinv, weight, bias, r2, o2, _epi(bias, act, residual))
    elif _F32_MATH == "x6":
        wp = split_f32_weight(weight)
        rc = _lib.lib().nos_gemm_f32x6(x2.data_ptr(), x2.stride(0), wp.data_ptr(), wp.stride(1), wp.stride(0),
                                       _ptr(bias), _ptr(r2), ldr, o2.data_ptr(), o2.stride(0), M, N, K,
                                       _epi(bias, act, residual), _stream())
        _lib.check(rc, "nos_gemm_f32x6")
    else:
        rc = _lib.lib().nos_gemm_f32(x2.data_ptr(), x2.stride(0), weight.data_ptr(), weight.stride(0), _ptr(bias),
                                     _ptr(r2), ldr, o2.data_ptr(), o2.stride(0), M, N, K, _epi(bias, act, residual),
                                     _stream())
        _lib.check(rc, "nos_gemm_f32")
    return o2.view(*x.shape[:-1], N)


_F32_MATH = "exact"
_GEMV_ROWS = 8   # tenant.GEMV_MAX_ROWS: GEMMs of at most this many rows run on the GEMV kernel
# h3 math: a GEMM of at most this many rows (YOLOS's detection-head layers on
# their 100 tokens) runs on the exact-f32 MFMA kernel -- one launch, no split
# pass, the f32 pipe's rate is ample for ~30 MFLOP -- instead of split + h3 GEMM
H3_MIN_ROWS = int(__import__("os").environ.get("NOS_AMD_H3_MIN_ROWS", "128"))
_SPLIT_CACHE: dict[int, tuple] = {}
_SPLIT_H3_CACHE: dict[int, tuple] = {}


def _pow2_exp(mx: torch.Tensor) -> torch.Tensor:
    """Exponents e with mx * 2^e < 2^14 (0 where mx == 0), clamped to +-126."""
    e = 14 - torch.frexp(mx).exponent.to(torch.int64)
    return torch.where(mx > 0, e, torch.zeros_like(e)).clamp(-126, 126)


@torch.no_grad()
def split_f32_weight_h3(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """The fp16x3 form of an fp32 weight [N, K]: every row on its own
    power-of-two scale (max |w| just under 2^14) as hi / lo fp16 planes
    [2, N, K], and the inverse scales [N] -- cached per tensor and version
    like :func:`split_f32_weight`."""
    key = id(w)
    hit = _SPLIT_H3_CACHE.get(key)
    if hit is not None:
        ref, ver, ptr, out = hit
        if ref() is w and ver == w._version and ptr == w.data_ptr():
            return out
    import weakref

    wf = w.float()
    e = _pow2_exp(wf.abs().amax(dim=1))
    ws = torch.ldexp(wf, e[:, None].to(wf.device))
    hi = ws.half()
    lo = (ws - hi.float()).half()
    out = (torch.stack([hi, lo]).contiguous(),
           torch.ldexp(torch.ones_like(e, dtype=torch.float32), -e).to(w.device).contiguous())
    _SPLIT_H3_CACHE[key] = (weakref.ref(w, lambda _r, k=key: _SPLIT_H3_CACHE.pop(k, None)), w._version,
                            w.data_ptr(), out)
    return out


def _split_rows_h3(x2: torch.Tensor, ln: bool, eps: float = 0.0) -> tuple[torch.Tensor, torch.Tensor]:
    """Rows of fp32 x2 [M, K] -> (hi / lo fp16 planes [2, M, K], 1 / row
    scale [M]) by ``nos_split_rows_h3``; ``ln``: the rows LayerNorm-normalised
    first, on the sqrt(K) bound's scale."""
    M, K = x2.shape
    planes = torch.empty((2, M, K), dtype=torch.float16, device=x2.device)
    rinv = torch.empty((M,), dtype=torch.float32, device=x2.device)
    eln = 14 - math.frexp(math.sqrt(K))[1]
    rc = _lib.lib().nos_split_rows_h3(x2.data_ptr(), x2.stride(0), planes.data_ptr(), K, M * K, rinv.data_ptr(), M,
                                      K, int(ln), float(eps), eln, _stream())
    _lib.check(rc, "nos_split_rows_h3")
    return planes, rinv


def _gemm_h3(ap, rinv, weight, bias, r2, o2, epi, kv=None, rconst: float = 0.0, planes_out=None) -> None:
    """One h3 GEMM on A planes ap [2, M, K] (row scales rinv, or rconst for
    every row) into o2 [M, N] -- or, with ``planes_out`` = (planes [2, M, N],
    scale), into the next GEMM's A planes."""
    M, K = ap.shape[1], ap.shape[2]
    N = weight.shape[0]
    wp, csc = split_f32_weight_h3(weight)
    kvs, S, skvp, kvsc = kv if kv is not None else (None, 0, 0, None)
    pp, psc = planes_out if planes_out is not None else (None, 1.0)
    rc = _lib.lib().nos_gemm_f32h3(ap.data_ptr(), K, M * K, _ptr(rinv), float(rconst), wp.data_ptr(), K, N * K,
                                   csc.data_ptr(), _ptr(bias), _ptr(r2), r2.stride(0) if r2 is not None else 0,
                                   _ptr(o2), o2.stride(0) if o2 is not None else N, M, N, K, epi, _ptr(kvs), S, skvp,
                                   _ptr(kvsc), _ptr(pp), N, M * N, float(psc), _stream())
    _lib.check(rc, "nos_gemm_f32h3")


class H3Planes(NamedTuple):
    """An activation handed between two h3 kernels as the consumer GEMM's A
    operand: hi / lo fp16 planes [2, M, K] on per-row scales (``rinv``) or one
    static scale (``rconst`` = its inverse), with the logical shape [..., K]."""
    planes: torch.Tensor
    rinv: torch.Tensor | None
    rconst: float
    shape: tuple


def _pow2_scale_under(bound: float) -> float:
    """The power of two s with bound * s < 2^14 (fp16's headroom for h3)."""
    if not bound > 0:
        return 1.0
    e = max(-126, min(126, 14 - math.frexp(bound)[1]))
    return math.ldexp(1.0, e)


_H3_OUT_SCALE: dict[tuple, tuple] = {}


@torch.no_grad()
def _h3_out_scale(wg: torch.Tensor, c2: torch.Tensor, act: str | None) -> float:
    """Static scale for the output of the LN-folded GEMM (wg, c2) as planes:
    |y_j| <= sqrt(K) ||wg_j||_2 + |c2_j| for every LayerNorm-normalised row,
    and GELU / ReLU never exceed that (or 0.17 below zero)."""
    key = (id(wg), act)
    hit = _H3_OUT_SCALE.get(key)
    if hit is not None and hit[0]() is wg and hit[1] == wg._version:
        return hit[2]
    import weakref

    b = float((math.sqrt(wg.shape[1]) * wg.double().norm(dim=1) + c2.double().abs()).max())
    if act in ("gelu", "relu"):
        b = max(b, 0.2)
    sc = _pow2_scale_under(b)
    _H3_OUT_SCALE[key] = (weakref.ref(wg, lambda _r, k=key: _H3_OUT_SCALE.pop(k, None)), wg._version, sc)
    return sc


class RowStats(NamedTuple):
    """LayerNorm statistics of an fp32 activation [M, K] handed from its
    producer GEMM to the LN-GEMM after it: ``stats`` [M, nparts, 2] = (mean,
    sum of squared deviations) over parts of ``pw`` columns."""
    stats: torch.Tensor
    pw: int


def linear_planes(a: H3Planes, weight: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
                  residual: torch.Tensor | None = None, row_stats: bool = False, out: torch.Tensor | None = None,
                  stats_out: torch.Tensor | None = None):
    """act(A @ weight^T + bias) + residual for an A handed over as h3 planes
    (see :class:`H3Planes`): no split pre-pass, no fp32 round trip of A.
    ``row_stats``: also return the output's row statistics for the next
    LN-GEMM (``nos_gemm_f32h3_stats``) -- ``(out, RowStats)``, written into
    ``stats_out`` (fp32 [M, ceil(N / stats_pw()), 2], contiguous) when given.
    ``out``: an [M, N]-viewable fp32 destination (e.g. a slab of a cat's
    buffer)."""
    M, K = a.planes.shape[1], a.planes.shape[2]
    N = weight.shape[0]
    if weight.dim() != 2 or weight.shape[1] != K or weight.dtype != torch.float32 or weight.stride(-1) != 1:
        raise ValueError(f"weight must be fp32 [N, {K}] with unit inner stride")
    _check_f32(bias=bias)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.planes.device)
    else:
        if out.dtype != torch.float32 or out.numel() != M * N:
            raise ValueError(f"out must hold fp32 [{M}, {N}]")
        out = out.view(M, N)
    r2 = None
    if residual is not None:
        if residual.numel() != M * N or residual.dtype != torch.float32:
            raise ValueError(f"residual must be fp32 [{M}, {N}]")
        r2 = residual.reshape(M, N)
        _check_f32(residual=r2)
    if row_stats:
        wp, csc = split_f32_weight_h3(weight)
        pw = stats_pw()
        shape = (M, (N + pw - 1) // pw, 2)
        if stats_out is None:
            st = torch.empty(shape, dtype=torch.float32, device=out.device)
        else:
            if tuple(stats_out.shape) != shape or stats_out.dtype != torch.float32 or not stats_out.is_contiguous():
                raise ValueError(f"stats_out must be a contiguous fp32 {list(shape)}")
            st = stats_out
        rc = _lib.lib().nos_gemm_f32h3_stats(a.planes.data_ptr(), K, M * K, _ptr(a.rinv), float(a.rconst),
                                             wp.data_ptr(), K, N * K, csc.data_ptr(), _ptr(bias), _ptr(r2),
                                             r2.stride(0) if r2 is not None else 0, out.data_ptr(), N, M, N, K,
                                             _epi(bias, act, residual), st.data_ptr(), _stream())
        _lib.check(rc, "nos_gemm_f32h3_stats")
        return out.view(*a.shape[:-1], N), RowStats(st, pw)
    _gemm_h3(a.planes, a.rinv, weight, bias, r2, out, _epi(bias, act, residual), rconst=a.rconst)
    return out.view(*a.shape[:-1], N)


def _row_stats(x2: torch.Tensor) -> RowStats:
    """(mean, M2) of every row of fp32 x2 [M, K] in one part (``nos_row_stats``):
    the LN-GEMM's statistics when no h3 GEMM produced x2."""
    M, K = x2.shape
    st = torch.empty((M, 1, 2), dtype=torch.float32, device=x2.device)
    _lib.check(_lib.lib().nos_row_stats(x2.data_ptr(), x2.stride(0), st.data_ptr(), M, K, _stream()), "nos_row_stats")
    return RowStats(st, K)


def _lna_ok(x2: torch.Tensor) -> bool:
    return x2.stride(1) == 1 and x2.stride(0) % 4 == 0 and x2.data_ptr() % 16 == 0


def _gemm_ln_h3(x2: torch.Tensor, pre, eps: float, wg: torch.Tensor, c2: torch.Tensor, o2, epi: int, kv=None,
                planes_out=None) -> None:
    """act(LayerNorm(x2) @ wg^T + c2) under h3 math (LN's gamma / beta folded
    into wg / c2).  With the LN hand-off on (:func:`set_ln_handoff`) the GEMM
    normalises and splits x2 itself, K-slice by K-slice
    (``nos_gemm_f32h3_lna``), from the row statistics its producer wrote
    (``pre``: :class:`RowStats`) or ``nos_row_stats``; otherwise the split
    pre-pass writes x2's normalised planes first (``nos_split_rows_h3``)."""
    M, K = x2.shape
    N = wg.shape[0]
    if _LN_HANDOFF and _lna_ok(x2):
        st = pre if isinstance(pre, RowStats) else _row_stats(x2)
        wp, csc = split_f32_weight_h3(wg)
        kvs, S, skvp, kvsc = kv if kv is not None else (None, 0, 0, None)
        pp, psc = planes_out if planes_out is not None else (None, 1.0)
        eln = 14 - math.frexp(math.sqrt(K))[1]
        rc = _lib.lib().nos_gemm_f32h3_lna(x2.data_ptr(), x2.stride(0), st.stats.data_ptr(), st.stats.shape[1], st.pw,
                                           float(eps), eln, wp.data_ptr(), K, N * K, csc.data_ptr(), c2.data_ptr(),
                                           None, 0, _ptr(o2), o2.stride(0) if o2 is not None else N, M, N, K, epi,
                                           _ptr(kvs), S, skvp, _ptr(kvsc), _ptr(pp), N, M * N, float(psc), _stream())
        _lib.check(rc, "nos_gemm_f32h3_lna")
        return
    ap, rinv = (pre.planes, pre.rinv) if isinstance(pre, H3Planes) else _split_rows_h3(x2, ln=True, eps=eps)
    _gemm_h3(ap, rinv, wg, c2, None, o2, epi, kv=kv, planes_out=planes_out)


_LN_HANDOFF = False


def set_ln_handoff(on: bool) -> None:
    """LayerNorm hand-off under h3 math: the LN-GEMMs normalise and split
    their fp32 input inside the GEMM (no ``nos_split_rows_h3`` pass), from
    row statistics the pre-LN residual GEMM wrote in its epilogue."""
    global _LN_HANDOFF
    _LN_HANDOFF = bool(on)


def ln_handoff_active() -> bool:
    return _LN_HANDOFF and _F32_MATH == "h3"


def linear_ln_to_planes(x: torch.Tensor, wg: torch.Tensor, c1: torch.Tensor, c2: torch.Tensor,
                        act: str | None = None, eps: float = 1e-12, pre=None) -> H3Planes:
    """:func:`linear_ln` under h3 math whose output goes straight to the next
    GEMM's A planes on the static scale of :func:`_h3_out_scale` (fc1 -> fc2)."""
    if _F32_MATH != "h3" or not x.is_cuda or x.dtype != torch.float32:
        raise ValueError("linear_ln_to_planes needs h3 math and an fp32 CUDA input")
    K = x.shape[-1]
    N = wg.shape[0]
    x2 = x.reshape(-1, K)
    _check_f32(x=x2, weight=wg, c1=c1, c2=c2)
    if K % 32:
        raise ValueError("linear_ln_to_planes needs K % 32 == 0")
    M = x2.shape[0]
    sc = _h3_out_scale(wg, c2, act)
    planes = torch.empty((2, M, N), dtype=torch.float16, device=x.device)
    _gemm_ln_h3(x2, pre, eps, wg, c2, None, EPI_BIAS | _epi(None, act, None), planes_out=(planes, sc))
    return H3Planes(planes, None, 1.0 / sc, (*x.shape[:-1], N))


def h3_planes_active(attention: bool = False) -> bool:
    """Whether producers hand activations over as h3 planes (h3 math, and for
    the attention an h3 variant)."""
    return _F32_MATH == "h3" and (not attention or _ATTN_F32_VARIANT.startswith("h3"))


def set_f32_math(mode: str) -> None:
    """How fp32 GEMMs use the matrix pipes: ``"exact"`` -- the f32-input MFMA
    (v_mfma_f32_32x32x2_f32, an fmaf chain, 1/16 of the bf16 rate) -- or
    ``"x6"`` -- every operand split into three bf16 pieces (exact: 3 x 8
    mantissa bits) and the six piece products of order >= 2^-16 summed by
    bf16 MFMAs in fp32 (csrc/hip/split_bf16.h): the same accuracy against fp64
    (tests/test_kernels_gpu.py) at 6/16 of the matrix-pipe time -- or
    ``"h3"`` -- every operand as two fp16 pieces on a power-of-two scale
    per row (csrc/hip/split_f16.h, gemm_f32h.hip: the activation rows split
    by a pre-pass, LayerNorm applied in it, the weight once), three fp16
    MFMAs per product: half of x6's matrix-pipe work, within the exact
    kernel's error against fp64 (tests/test_gemm_h3_gpu.py).  The fp32
    attention has its own switch (``set_attention_f32_variant("x6")``)."""
    global _F32_MATH
    if mode not in ("exact", "x6", "h3"):
        raise ValueError(f"f32 math must be 'exact', 'x6' or 'h3', got {mode!r}")
    _F32_MATH = mode


def f32_math() -> str:
    return _F32_MATH


def set_gemm_f32x6_tile(tile: str) -> None:
    """x6 GEMM tile: ``"policy"`` (the fp32 GEMM policy's tile), ``"128x64"`` or
    ``"128x128"`` (4 x 1 waves: each wave splits one A block for all of its W
    blocks -- 8 fractional pods 425 (64x64) -> 448 (128x64) -> 466 (128x128)
    inf/s, profiles/r03_f32x6_fleet_ab.json), ``"wide"`` (128x128 where
    N >= 1024, else 128x64)."""
    names = {"policy": -1, "128x64": 3, "128x128": 5, "wide": 6, "256x128": 7}  # wide: 128x128 if N >= 1024, else 128x64
    code = names[tile] if tile in names else int(tile)  # numeric codes: gemm_f32x.hip g_tile (A/B)
    _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(code), "nos_gemm_f32x6_set_tile")


def set_gemm_f32h3_lds_epilogue(on: bool) -> None:
    """Plain fp32-C h3 GEMMs store C through LDS (float4 row stores and
    residual loads, the LN hand-off producer's epilogue) instead of one dword
    per element in the MFMA layout."""
    _lib.check(_lib.lib().nos_gemm_f32h3_set_lds_epilogue(int(bool(on))), "nos_gemm_f32h3_set_lds_epilogue")


def set_gemm_f32h3_hot_ring(stages: int) -> None:
    """LDS ring depth of the row-statistics / LDS-epilogue h3 GEMMs (the
    residual GEMMs of a transformer): 2 (64 KiB, two workgroups per CU) or 3
    (96 KiB, one workgroup per CU; a stage two ahead in flight)."""
    _lib.check(_lib.lib().nos_gemm_f32h3_set_hot_ring(int(stages)), "nos_gemm_f32h3_set_hot_ring")


def set_gemm_f32h3_hot_bn(bn: int) -> None:
    """Tile width of the row-statistics producers and LDS-epilogue GEMMs
    (a transformer's residual GEMMs): 64 (48 KiB ring, three workgroups per
    CU) or 128.  The row statistics come in parts of this many columns
    (:func:`stats_pw`); the LN-in-A-load consumers stay 128 x 128."""
    _lib.check(_lib.lib().nos_gemm_f32h3_set_hot_bn(int(bn)), "nos_gemm_f32h3_set_hot_bn")


def set_gemm_f32h3_lna_wide(on: bool) -> None:
    """LN-in-A-load GEMMs writing the next GEMM's planes (fc1 -> fc2) on
    128 x 256 tiles with 8 waves (half the A normalise-and-split work per
    MFMA) instead of 128 x 128 -- A/B; the results are bit-identical."""
    _lib.check(_lib.lib().nos_gemm_f32h3_set_lna_wide(int(bool(on))), "nos_gemm_f32h3_set_lna_wide")


def stats_pw() -> int:
    """Column width of a row-statistics part (the producer GEMM's tile width)."""
    return int(_lib.lib().nos_gemm_f32h3_hot_bn())


def set_gemm_f32h3_layout(layout: str) -> None:
    """h3 GEMM tiles / waves: ``"2x2"`` (default: 128x128, 64x64 per wave),
    ``"4x1"`` (128x128, 32-row strips, each wave reads the whole W tile),
    ``"256x128"`` (8 waves of 64x64, one workgroup per CU), ``"4x1r3"``
    (3-deep ring of BK-32 stages), ``"4x1k16"`` / ``"2x2k16"`` (4-deep ring
    of BK-16 stages), ``"2x2r3"`` (2x2, 3-deep BK-32 ring), ``"2x2n64"``
    (128 x 64 tiles, 48 KiB: three workgroups per CU) -- A/B; the
    results are bit-identical."""
    _lib.check(_lib.lib().nos_gemm_f32h3_set_layout({"4x1": 0, "2x2": 1, "256x128": 2, "4x1r3": 3, "4x1k16": 4,
                                                     "2x2k16": 5, "2x2r3": 6, "2x2n64": 7}[layout]),
               "nos_gemm_f32h3_set_layout")


def set_attention_f32h3_waves(waves: int) -> None:
    """h3 attention workgroups of 8 waves (default: 256 query rows, 2 per CU,
    each key tile loaded once for twice the queries; fleet 756 vs 743 inf/s)
    or 4 (128 rows, 4 per CU); bit-identical results."""
    _lib.check(_lib.lib().nos_attn_f32h3_set_waves(int(waves)), "nos_attn_f32h3_set_waves")


def set_gemm_f32x6_pipeline(on: bool) -> None:
    """x6 GEMM K loop: software-pipelined (default: the next MFMA step's
    fragments are read and split under the current step's MFMAs) or the
    plain loop (A/B; bit-identical results)."""
    _lib.check(_lib.lib().nos_gemm_f32x6_set_pipeline(int(bool(on))), "nos_gemm_f32x6_set_pipeline")


def split_bf16x3(t: torch.Tensor) -> torch.Tensor:
    """fp32 tensor -> [3, *t.shape] bf16 pieces with t == p0 + p1 + p2 exactly."""
    t = t.float()
    p0 = t.to(torch.bfloat16)
    r = t - p0.float()
    p1 = r.to(torch.bfloat16)
    p2 = (r - p1.float()).to(torch.bfloat16)
    return torch.stack([p0, p1, p2]).contiguous()


@torch.no_grad()
def split_f32_weight(w: torch.Tensor) -> torch.Tensor:
    """The bf16x3 planes [3, N, K] of an fp32 weight, cached per tensor and
    version (a weight is split once; the first forward, before any graph
    capture, fills the cache)."""
    key = id(w)
    hit = _SPLIT_CACHE.get(key)
    if hit is not None:
        ref, ver, ptr, planes = hit
        if ref() is w and ver == w._version and ptr == w.data_ptr():
            return planes
    import weakref

    planes = split_bf16x3(w)
    _SPLIT_CACHE[key] = (weakref.ref(w, lambda _r, k=key: _SPLIT_CACHE.pop(k, None)), w._version, w.data_ptr(),
                         planes)
    return planes


def set_gemm_policy(policy: str) -> None:
    """bf16 GEMM tile choice (``csrc/hip/gemm.hip:pick_tile``):
    ``"throughput"`` (default: least padded work over 128x128 / 256x192 /
    256x256 tiles, best when pods share a GPU) or ``"latency"`` (fewest rounds
    of tiles over the CUs, 128x64 included, best for a single tenant);
    ``"narrow"`` / ``"big"`` / ``"wide"`` force 128x64 / 256x256 / 256x192
    (A/B measurements)."""
    code = {"throughput": 0, "latency": 1, "narrow": 2, "big": 3, "wide": 4}[policy]
    _lib.check(_lib.lib().nos_gemm_set_policy(code), "nos_gemm_set_policy")


def set_gemm_persistent(wgs_per_cu: int) -> None:
    """bf16 GEMM grid: 0 = one workgroup per tile; n > 0 = at most n
    workgroups per CU, each walking several tiles of its XCD's chunk and
    loading the next tile while it runs the current epilogue."""
    _lib.check(_lib.lib().nos_gemm_set_persistent(int(wgs_per_cu)), "nos_gemm_set_persistent")


def set_cu_budget(cus: int) -> None:
    """CUs this process may use (a CU-mask slice: the popcount of its
    ``ROC_GLOBAL_CU_MASK``; 0 = no limit).  The fp32 GEMM / attention and the
    bf16 GEMM then launch slice-sized persistent grids (resident workgroups x
    budgeted CUs) instead of one workgroup per tile: every dispatch completes at
    launch, so a pod never holds a command-processor pipe that another pod's
    queue shares (profiles/r03_hol_*.json: 8 masked pods on 4 pipes per XCD)."""
    _lib.check(_lib.lib().nos_set_cu_budget(int(cus)), "nos_set_cu_budget")


def cu_budget() -> int:
    return int(_lib.lib().nos_get_cu_budget())


def set_gemm_f32_policy(policy: str) -> None:
    """fp32 GEMM tiles: ``"latency"`` (default; fewest rounds of tiles over
    the CUs) or ``"throughput"`` (most MFMA-efficient tile; other co-running
    pods fill the CUs a small grid leaves idle) or ``"small"`` (always 64x64:
    the least LDS and registers per workgroup)."""
    _lib.check(_lib.lib().nos_gemm_f32_set_policy({"throughput": 0, "latency": 1, "small": 2}[policy]),
               "nos_gemm_f32_set_policy")


def set_attention_f32_variant(variant: str) -> None:
    """fp32 attention tiling: ``"auto"`` (default), ``"w4k64"`` (4 waves x 64-key
    LDS tiles) or ``"w4k64g2"`` (two such wave groups per workgroup on
    interleaved key tiles, merged at the end: 2 waves per SIMD from one
    workgroup); A/B tilings: ``"w4k32"`` (32-key tiles, half the LDS),
    ``"w2k64"`` (64-query blocks), ``"w8k64"`` (256-query blocks), ``"w4k32o4"`` (32-key tiles in 127
    VGPRs: 4 waves per SIMD), ``"w4k32g2"`` (two groups on 32-key tiles); ``"x6"``: the bf16x6 split
    kernel (attention_f32x.hip: fp32 operands as three bf16 pieces, six
    exact piece products per product on the bf16 matrix pipes; the keys are
    split 1-4 ways when the grid would leave CU slots empty), ``"x6k<n>"``
    with n key splits forced, ``"x6n"`` = ``"x6k1"`` (never split);
    ``"h3"`` / ``"h3n"`` / ``"h3k<n>"``: the fp16x3 kernel (two fp16 pieces
    per operand on power-of-two scales, three MFMAs per product: the x6
    kernel's per-product error bound at half its matrix-pipe work) wherever
    the attention follows a fused-LN QKV projection
    (:func:`ln_qkv_attention`), whose weights bound every key and value; a
    bare :func:`attention_qkv` runs the x6 kernel."""
    global _ATTN_F32_VARIANT
    x6 = {"x6": 0, "x6n": 1, "x6k1": 1, "x6k2": 2, "x6k3": 3, "x6k4": 4,
          "h3": 0, "h3n": 1, "h3k1": 1, "h3k2": 2, "h3k3": 3, "h3k4": 4}
    code = {"auto": 0, "w4k64": 1, "w4k64g2": 2, "w4k32": 3, "w2k64": 4, "w8k64": 5, "w4k32o4": 6,
            "w4k32g2": 7}.get(variant, 0)
    if variant not in x6 and code == 0 and variant != "auto":
        raise KeyError(variant)
    _lib.check(_lib.lib().nos_attn_f32_set_variant(code), "nos_attn_f32_set_variant")
    if variant in x6:  # x6k<n>: n key splits (x6: auto)
        _lib.check(_lib.lib().nos_attn_f32x6_set_kvsplit(x6[variant]), "nos_attn_f32x6_set_kvsplit")
    _ATTN_F32_VARIANT = variant


_ATTN_F32_VARIANT = "auto"


def attention_f32_variant() -> str:
    return _ATTN_F32_VARIANT


@torch.no_grad()
def fold_layernorm(weight: torch.Tensor, bias: torch.Tensor | None, gamma: torch.Tensor, beta: torch.Tensor
                   ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Fold LayerNorm(gamma, beta) into the following linear layer.

    LN(x) @ W^T + b = rstd * (x @ (W*gamma)^T - mu * c1) + c2 with
    c1 = rowsum(W*gamma) (from the bf16-rounded folded weight, so the identity
    holds for the values the kernel multiplies) and c2 = W @ beta + b.
    Returns (W*gamma in W's dtype, c1 fp32, c2 fp32)."""
    wg = (weight.float() * gamma.float()[None, :]).to(weight.dtype).contiguous()
    c1 = wg.float().sum(dim=1).contiguous()
    # elementwise, not a GEMV: a BLAS call here would make the pod server's first
    # tenant pay hipBLASLt's ~128 MB per-stream workspace in its measured footprint
    c2 = (weight.float() * beta.float()[None, :]).sum(dim=1)
    if bias is not None:
        c2 = c2 + bias.float()
    return wg, c1, c2.contiguous()


def linear_ln_ref(x, wg, c1, c2, act=None, eps=1e-12):
    xf = x.float()
    mu = xf.mean(-1, keepdim=True)
    var = xf.var(-1, unbiased=False, keepdim=True)
    y = ((xf @ wg.float().t()) - mu * c1) * torch.rsqrt(var + eps) + c2
    if act == "gelu":
        y = F.gelu(y)
    elif act == "relu":
        y = F.relu(y)
    return y.to(x.dtype)


def linear_ln(x: torch.Tensor, wg: torch.Tensor, c1: torch.Tensor, c2: torch.Tensor, act: str | None = None,
              eps: float = 1e-12, out: torch.Tensor | None = None, max_wg: int = 0,
              pre=None) -> torch.Tensor:
    """act(LayerNorm(x) @ W^T + b) with LN folded by :func:`fold_layernorm`
    (``pre``: x's row statistics, :class:`RowStats`, from its producer)."""
    if not x.is_cuda:
        return linear_ln_ref(x, wg, c1, c2, act, eps)
    K = x.shape[-1]
    N = wg.shape[0]
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if x.dtype == torch.float32:
        _check_f32(x=x2, weight=wg, c1=c1, c2=c2)
        if K % 32:
            raise ValueError("native fp32 linear_ln needs K % 32 == 0")
        o2, _ = _gemm_io(x, wg, out, None, M, N, K)
        if _F32_MATH == "h3":
            _gemm_ln_h3(x2, pre, eps, wg, c2, o2, EPI_BIAS | _epi(None, act, None))
        elif _F32_MATH == "x6":
            wp = split_f32_weight(wg)
            rc = _lib.lib().nos_gemm_ln_f32x6(x2.data_ptr(), x2.stride(0), wp.data_ptr(), wp.stride(1), wp.stride(0),
                                              c1.data_ptr(), c2.data_ptr(), o2.data_ptr(), o2.stride(0), M, N, K,
                                              _epi(None, act, None), float(eps), _stream())
            _lib.check(rc, "nos_gemm_ln_f32x6")
        else:
            rc = _lib.lib().nos_gemm_ln_f32(x2.data_ptr(), x2.stride(0), wg.data_ptr(), wg.stride(0), c1.data_ptr(),
                                            c2.data_ptr(), o2.data_ptr(), o2.stride(0), M, N, K,
                                            _epi(None, act, None), float(eps), _stream())
            _lib.check(rc, "nos_gemm_ln_f32")
        return o2.view(*x.shape[:-1], N)
    if x2.stride(-1) != 1 or K % 64 or x.dtype != torch.bfloat16:
        raise ValueError("native linear_ln needs bf16, unit inner stride and K % 64 == 0")
    o2, _ = _gemm_io(x, wg, out, None, M, N, K)
    epi = EPI_GELU if act == "gelu" else (EPI_RELU if act == "relu" else 0)
    rc = _lib.lib().nos_gemm_ln_bf16(x2.data_ptr(), x2.stride(0), wg.data_ptr(), wg.stride(0), c1.data_ptr(),
                                     c2.data_ptr(), o2.data_ptr(), o2.stride(0), M, N, K, epi, float(eps), max_wg,
                                     _stream())
    _lib.check(rc, "nos_gemm_ln_bf16")
    return o2.view(*x.shape[:-1], N)


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12,
              residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
              sum_out: torch.Tensor | None = None):
    """LayerNorm(x + residual). Returns (y, sum) where sum = x + residual (or None)."""
    if not x.is_cuda:
        return layernorm_ref(x, gamma, beta, eps, residual)
    D = x.shape[-1]
    for name, t in (("x", x), ("gamma", gamma), ("beta", beta), ("residual", residual), ("out", out),
                    ("sum_out", sum_out)):
        if t is not None and t.dtype != torch.bfloat16:
            raise ValueError(f"native layernorm takes bf16 tensors ({name} is {t.dtype})")
    if gamma.numel() != D or beta.numel() != D or not (gamma.is_contiguous() and beta.is_contiguous()):
        raise ValueError("gamma/beta must be contiguous [D]")

    def rows2d(name, t):
        t2 = t.reshape(-1, D)  # a view when the rows are evenly strided, else a copy (never written back)
        if t2.stride(-1) != 1 or t2.shape[0] != x2.shape[0]:
            raise ValueError(f"{name} must have unit inner stride and x's rows")
        return t2

    x2 = x.reshape(-1, D)
    if x2.stride(-1) != 1:
        raise ValueError("x must have unit inner stride")
    rows = x2.shape[0]
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    if residual is not None and sum_out is None:
        sum_out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    o2 = out.view(-1, D)
    r2 = rows2d("residual", residual) if residual is not None else None
    s2 = sum_out.view(-1, D) if sum_out is not None else None
    rc = _lib.lib().nos_layernorm_bf16(x2.data_ptr(), _ptr(r2), o2.data_ptr(), _ptr(s2), gamma.data_ptr(),
                                       beta.data_ptr(), rows, D, x2.stride(0), o2.stride(0),
                                       r2.stride(0) if r2 is not None else D, s2.stride(0) if s2 is not None else D,
                                       float(eps), _stream())
    _lib.check(rc, "nos_layernorm_bf16")
    return out, sum_out


def attention_qkv(qkv: torch.Tensor, num_heads: int, out: torch.Tensor | None = None,
                  scale: float | None = None) -> torch.Tensor:
    """Self-attention on a fused projection qkv [B, S, 3*H*64] -> [B, S, H*64]."""
    B, S, three_hd = qkv.shape
    D = three_hd // (3 * num_heads)
    if not qkv.is_cuda:
        q, k, v = qkv.view(B, S, 3, num_heads, D).unbind(2)
        return attention_ref(q, k, v, scale).reshape(B, S, num_heads * D)
    if D != 64:
        raise ValueError("native attention supports head_dim 64")
    if qkv.stride(-1) != 1:
        raise ValueError("qkv must have unit inner stride")
    if qkv.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("native attention takes bf16 or fp32")
    if out is None:
        out = torch.empty((B, S, num_heads * D), dtype=qkv.dtype, device=qkv.device)
    if out.dtype != qkv.dtype or out.stride(-1) != 1 or out.shape != (B, S, num_heads * D):
        raise ValueError("out must be [B, S, H*64] of qkv's dtype with unit inner stride")
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    hd = num_heads * D
    base = qkv.data_ptr()
    es = qkv.element_size()
    L = _lib.lib()
    args = (base, base + hd * es, base + 2 * hd * es, out.data_ptr(), B, num_heads, S, S, qkv.stride(1),
            qkv.stride(0), out.stride(1), out.stride(0), float(scale))
    if qkv.dtype == torch.float32 and _ATTN_F32_VARIANT[:2] in ("x6", "h3"):
        # the split K/V planes: a stream-ordered allocation (graph-capture safe)
        nbytes = int(L.nos_attn_f32x6_workspace(B, num_heads, S, S))
        ws = torch.empty(nbytes // 2, dtype=torch.int16, device=qkv.device)
        _lib.check(L.nos_attn_fwd_f32x6_d64(*args, ws.data_ptr(), nbytes, _stream()), "nos_attn_fwd_f32x6_d64")
        return out
    fn, name = ((L.nos_attn_fwd_f32_d64, "nos_attn_fwd_f32_d64") if qkv.dtype == torch.float32
                else (L.nos_attn_fwd_d64, "nos_attn_fwd_d64"))
    _lib.check(fn(*args, _stream()), name)
    return out


def linear_ln_qkv_x6(x: torch.Tensor, wg: torch.Tensor, c1: torch.Tensor, c2: torch.Tensor, num_heads: int,
                     eps: float = 1e-12) -> tuple[torch.Tensor, torch.Tensor]:
    """The fused-LayerNorm QKV projection of an fp32 pod under x6 math, with
    its K / V columns written straight into the bf16x6 attention's plane
    workspace (``nos_gemm_ln_f32x6_qkv``): returns (qkv [B, S, 3*H*64] whose
    Q columns are valid, workspace) for :func:`attention_presplit`.  The
    planes are exactly the split the attention's own streaming kernel makes:
    the result equals ``attention_qkv(linear_ln(...))`` bit for bit."""
    B, S, K = x.shape
    N = wg.shape[0]
    D = 64
    if N != 3 * num_heads * D or x.dtype != torch.float32 or not x.is_cuda:
        raise ValueError("linear_ln_qkv_x6: fp32 CUDA input and a [3*H*64, K] projection")
    _check_f32(x=x, weight=wg, c1=c1, c2=c2)
    if K % 32:
        raise ValueError("linear_ln_qkv_x6 needs K % 32 == 0")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    out = torch.empty((B, S, N), dtype=torch.float32, device=x.device)
    L = _lib.lib()
    nbytes = int(L.nos_attn_f32x6_workspace(B, num_heads, S, S))
    ws = torch.empty(nbytes // 2, dtype=torch.int16, device=x.device)
    skvp = (S + 31) // 32 * 32
    wp = split_f32_weight(wg)
    rc = L.nos_gemm_ln_f32x6_qkv(x2.data_ptr(), x2.stride(0), wp.data_ptr(), wp.stride(1), wp.stride(0),
                                 c1.data_ptr(), c2.data_ptr(), out.data_ptr(), N, M, N, K, 0, float(eps),
                                 ws.data_ptr(), S, skvp, _stream())
    _lib.check(rc, "nos_gemm_ln_f32x6_qkv")
    return out, ws


def attention_presplit(qkv: torch.Tensor, ws: torch.Tensor, num_heads: int, scale: float | None = None,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16x6 attention from the planes :func:`linear_ln_qkv_x6` wrote (the Q
    columns of ``qkv`` are read)."""
    B, S, three_hd = qkv.shape
    hd = three_hd // 3
    if out is None:
        out = torch.empty((B, S, hd), dtype=torch.float32, device=qkv.device)
    if out.dtype != torch.float32 or out.stride(-1) != 1 or out.shape != (B, S, hd):
        raise ValueError("out must be [B, S, H*64] fp32 with unit inner stride")
    scale = scale if scale is not None else 1.0 / math.sqrt(64)
    rc = _lib.lib().nos_attn_fwd_f32x6_presplit_d64(qkv.data_ptr(), out.data_ptr(), B, num_heads, S, S,
                                                    qkv.stride(1), qkv.stride(0), out.stride(1), out.stride(0),
                                                    float(scale), ws.data_ptr(), ws.numel() * ws.element_size(),
                                                    _stream())
    _lib.check(rc, "nos_attn_fwd_f32x6_presplit_d64")
    return out


_H3_SCALES: dict[int, tuple] = {}


@torch.no_grad()
def h3_head_scales(wg: torch.Tensor, c2: torch.Tensor, num_heads: int) -> torch.Tensor:
    """Per-head power-of-two scales [2, H] (K, V) for the fp16x3 attention's
    planes, from the folded LN-QKV weights alone: the LayerNorm output x^ of
    a row has ||x^||_2 <= sqrt(K), so every output column j obeys
    |y_j| <= sqrt(K) ||wg_j||_2 + |c2_j|; each head's K and V get the scale
    that puts that bound just under 2^14 (fp16 holds 65504).  Cached per
    weight tensor and version, like :func:`split_f32_weight`."""
    key = id(wg)
    hit = _H3_SCALES.get(key)
    if hit is not None:
        ref, ver, ptr, sc = hit
        if ref() is wg and ver == wg._version and ptr == wg.data_ptr():
            return sc
    import weakref

    K = wg.shape[1]
    hd = num_heads * 64
    bound = math.sqrt(K) * wg.double().norm(dim=1) + c2.double().abs()
    b = bound[hd:].view(2, num_heads, 64).amax(dim=2).cpu()           # [K|V, head]
    e = 14 - torch.frexp(b).exponent.to(torch.int64)                  # b < 2^exponent
    e = torch.where(b > 0, e, torch.zeros_like(e)).clamp(-126, 126)
    sc_host = torch.ldexp(torch.ones_like(b), e).float().contiguous()
    sc = sc_host.to(wg.device)
    def drop(_r, k=key):
        _H3_SCALES.pop(k, None)
        _H3_SCALES_HOST.pop(k, None)

    _H3_SCALES[key] = (weakref.ref(wg, drop), wg._version, wg.data_ptr(), sc)
    _H3_SCALES_HOST[key] = sc_host
    return sc


_H3_SCALES_HOST: dict[int, torch.Tensor] = {}


def linear_ln_qkv_h3(x: torch.Tensor, wg: torch.Tensor, c1: torch.Tensor, c2: torch.Tensor, num_heads: int,
                     eps: float = 1e-12, pre=None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """:func:`linear_ln_qkv_x6` writing the fp16x3 attention's planes (K and V
    as fp16 hi / lo pieces on the per-head scales of :func:`h3_head_scales`):
    returns (qkv with valid Q columns, workspace, scales) for
    :func:`attention_presplit_h3`."""
    B, S, K = x.shape
    N = wg.shape[0]
    if N != 3 * num_heads * 64 or x.dtype != torch.float32 or not x.is_cuda:
        raise ValueError("linear_ln_qkv_h3: fp32 CUDA input and a [3*H*64, K] projection")
    _check_f32(x=x, weight=wg, c1=c1, c2=c2)
    if K % 32:
        raise ValueError("linear_ln_qkv_h3 needs K % 32 == 0")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    out = torch.empty((B, S, N), dtype=torch.float32, device=x.device)
    L = _lib.lib()
    nbytes = int(L.nos_attn_f32x6_workspace(B, num_heads, S, S))
    ws = torch.empty(nbytes // 2, dtype=torch.int16, device=x.device)
    skvp = (S + 31) // 32 * 32
    sc = h3_head_scales(wg, c2, num_heads)
    if _F32_MATH == "h3":
        _gemm_ln_h3(x2, pre, eps, wg, c2, out.view(M, N), EPI_BIAS, kv=(ws, S, skvp, sc))
        return out, ws, sc
    wp = split_f32_weight(wg)
    rc = L.nos_gemm_ln_f32x6_qkv_h3(x2.data_ptr(), x2.stride(0), wp.data_ptr(), wp.stride(1), wp.stride(0),
                                    c1.data_ptr(), c2.data_ptr(), out.data_ptr(), N, M, N, K, 0, float(eps),
                                    ws.data_ptr(), S, skvp, sc.data_ptr(), _stream())
    _lib.check(rc, "nos_gemm_ln_f32x6_qkv_h3")
    return out, ws, sc


def attention_presplit_h3(qkv: torch.Tensor, ws: torch.Tensor, scales: torch.Tensor, num_heads: int,
                          scale: float | None = None, out: torch.Tensor | None = None,
                          planes_out: float | None = None, q_range: tuple[int, int] | None = None):
    """fp16x3 attention from the planes :func:`linear_ln_qkv_h3` wrote.
    ``planes_out`` = a static scale s with |O| * s < 2^14 (every O row is a
    convex combination of V rows: the smallest V head scale works): the
    output goes to the proj GEMM's A planes instead, as :class:`H3Planes`.
    ``q_range`` = (q0, q1): only those query rows (every key): O [B, q1 - q0, hd]."""
    B, Skv, three_hd = qkv.shape
    hd = three_hd // 3
    q0, q1 = q_range if q_range is not None else (0, Skv)
    if not 0 <= q0 < q1 <= Skv:
        raise ValueError(f"q_range {q_range} outside 0..{Skv}")
    S = q1 - q0
    planes = None
    if planes_out is not None:  # planes [2, B*S, hd] with o's strides; o itself is never written
        planes = torch.empty((2, B * S, hd), dtype=torch.float16, device=qkv.device)
        o_ptr, ld_out, bs_out = planes.data_ptr(), hd, S * hd
    else:
        if out is None:
            out = torch.empty((B, S, hd), dtype=torch.float32, device=qkv.device)
        if out.dtype != torch.float32 or out.stride(-1) != 1 or out.shape != (B, S, hd):
            raise ValueError("out must be [B, S, H*64] fp32 with unit inner stride")
        o_ptr, ld_out, bs_out = out.data_ptr(), out.stride(1), out.stride(0)
    if scales.shape != (2, num_heads) or scales.dtype != torch.float32 or not scales.is_contiguous():
        raise ValueError("scales must be the [2, H] fp32 tensor of linear_ln_qkv_h3")
    scale = scale if scale is not None else 1.0 / math.sqrt(64)
    q_ptr = qkv.data_ptr() + q0 * qkv.stride(1) * qkv.element_size()
    rc = _lib.lib().nos_attn_fwd_f32h3_presplit_d64(q_ptr, o_ptr, B, num_heads, S, Skv,
                                                    qkv.stride(1), qkv.stride(0), ld_out, bs_out,
                                                    float(scale), scales.data_ptr(), ws.data_ptr(),
                                                    ws.numel() * ws.element_size(), _ptr(planes), B * S * hd,
                                                    float(planes_out or 1.0), _stream())
    _lib.check(rc, "nos_attn_fwd_f32h3_presplit_d64")
    if planes is not None:
        return H3Planes(planes, None, 1.0 / planes_out, (B, S, hd))
    return out


def ln_qkv_fusable(x: torch.Tensor) -> bool:
    """Whether :func:`ln_qkv_attention` runs fused for this input: an fp32 pod
    on the GPU under x6 math and an x6 / h3 attention variant."""
    return (x.is_cuda and x.dtype == torch.float32 and _F32_MATH in ("x6", "h3")
            and _ATTN_F32_VARIANT[:2] in ("x6", "h3"))


def ln_qkv_attention(x: torch.Tensor, wg: torch.Tensor, c1: torch.Tensor, c2: torch.Tensor, num_heads: int,
                     eps: float = 1e-12, planes_out: bool = False, pre=None,
                     q_range: tuple[int, int] | None = None):
    """attention(LayerNorm(x) @ W_qkv^T + b) for an fp32 pod (see
    :func:`ln_qkv_fusable`): the QKV projection writes the attention's K / V
    planes straight from its epilogue -- fp16x3 planes under an ``h3``
    variant, bf16x6 planes otherwise.  ``planes_out`` (h3 variant only):
    the output as the proj GEMM's :class:`H3Planes`."""
    if _ATTN_F32_VARIANT.startswith("h3"):
        qkv, ws, sc = linear_ln_qkv_h3(x, wg, c1, c2, num_heads, eps=eps, pre=pre)
        osc = float(_H3_SCALES_HOST[id(wg)][1].min()) if planes_out else None
        return attention_presplit_h3(qkv, ws, sc, num_heads, planes_out=osc, q_range=q_range)
    if _F32_MATH == "h3":  # x6 attention after an h3 projection: the unfused pair
        y = attention_qkv(linear_ln(x, wg, c1, c2, eps=eps), num_heads)
    else:
        qkv, ws = linear_ln_qkv_x6(x, wg, c1, c2, num_heads, eps=eps)
        y = attention_presplit(qkv, ws, num_heads)
    return y[:, q_range[0]:q_range[1]] if q_range is not None else y


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """q,k,v [B, S, H, 64] (rows contiguous per token) -> [B, Sq, H, 64]."""
    if not q.is_cuda:
        return attention_ref(q, k, v, scale)
    B, Sq, H, D = q.shape
    Skv = k.shape[1]
    if D != 64:
        raise ValueError("native attention supports head_dim 64")
    for t in (q, k, v):
        if t.stride(-1) != 1 or t.stride(-2) != D:
            raise ValueError("q/k/v need contiguous heads")
    if not (q.stride(1) == k.stride(1) == v.stride(1) and q.stride(0) == k.stride(0) == v.stride(0)):
        raise ValueError("q/k/v must share row and batch strides")
    if out is None:
        out = torch.empty((B, Sq, H, D), dtype=q.dtype, device=q.device)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rc = _lib.lib().nos_attn_fwd_d64(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B, H,
                                     Sq, Skv, q.stride(1), q.stride(0), out.stride(1), out.stride(0),
                                     float(scale), _stream())
    _lib.check(rc, "nos_attn_fwd_d64")
    return out


__all__ = ["set_ln_handoff", "ln_handoff_active", "set_f32_math", "f32_math", "h3_head_scales", "linear_ln_qkv_h3", "split_f32_weight_h3", "set_gemm_f32h3_layout", "set_gemm_f32h3_hot_ring", "set_gemm_f32h3_hot_bn", "set_gemm_f32h3_lna_wide", "stats_pw", "H3Planes", "set_attention_f32h3_waves", "linear_planes", "linear_ln_to_planes", "h3_planes_active", "attention_presplit_h3", "ln_qkv_fusable", "ln_qkv_attention", "set_gemm_f32x6_tile", "set_gemm_f32x6_pipeline", "linear_ln_qkv_x6", "attention_presplit", "split_f32_weight", "split_bf16x3", "set_cu_budget", "cu_budget", "set_gemm_policy", "set_gemm_persistent", "linear", "linear_ln", "fold_layernorm", "layernorm", "attention", "attention_qkv", "linear_ref",
           "linear_ln_ref", "layernorm_ref", "attention_ref"]
