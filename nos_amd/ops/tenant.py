"""Ops of general pod-server tenant programs (decoder LLMs, conv nets).

The YOLOS-class encoder ops live in :mod:`nos_amd.ops`; this module adds
what conv nets and decoder LLMs need, each lowered onto gfx950 kernels of
``libnos_hip.so`` for CUDA tensors and onto a plain PyTorch fp32 reference
for CPU tensors (the numerics tests compare the two):

* :func:`conv2d` -- implicit-GEMM convolution on the fp16x3 (h3) matrix
  pipes: ``nos_im2col_h3`` writes an image's patches straight as the GEMM's
  split planes (per-patch power-of-two scales), and ONE batched
  ``nos_gemm_f32h3_batched`` launch computes ``W . patches^T`` for every
  image, NCHW out, bias per output channel, ReLU / GELU and a residual in
  the epilogue (BatchNorm is folded into the weights by the compiler);
* :func:`matmul` -- batched activation x activation GEMM on the same kernel
  (both sides split at run time, a broadcast side has stride 0);
* :func:`sdpa` -- attention with causal masking, head_dim 64 / 128,
  grouped-query K/V heads and fused rotary embeddings (``nos_attn_h3g``);
* :func:`linear_rms` -- RMSNorm folded into the following GEMM (the row
  statistics in the split pre-pass, gamma in the weight);
* :func:`embedding`, :func:`rmsnorm`, :func:`softmax`, :func:`rotary` --
  row / gather kernels (``tenant_ops.hip``), fp32 and bf16.

bf16 tensors run the fp32-only GEMM / attention kernels on an fp32 copy
(more precision than the tenant asked for, never less).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import EPI_BIAS, EPI_GELU, EPI_RELU, EPI_RESID, _lib, _split_rows_h3, _stream, split_f32_weight_h3

EPI_BIAS_ROW, EPI_RESID_PRE = 16, 32  # gemm_f32h.hip: bias per row; residual added before the activation


def _ptr(t):
    return None if t is None else t.data_ptr()


def _act_epi(act: str | None) -> int:
    return EPI_GELU if act == "gelu" else (EPI_RELU if act == "relu" else 0)


def _act(y: torch.Tensor, act: str | None) -> torch.Tensor:
    return F.gelu(y) if act == "gelu" else (F.relu(y) if act == "relu" else y)


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t if t.dtype == torch.float32 else t.float()


def _pad_k(t: torch.Tensor, mult: int = 32) -> torch.Tensor:
    k = t.shape[-1]
    kp = -(-k // mult) * mult
    return t if kp == k else F.pad(t, (0, kp - k))


def _bf(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise ValueError(f"tenant ops take fp32 or bf16 tensors, got {t.dtype}")


# ------------------------------------------------------------------ references
def conv2d_ref(x, w, bias=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1), act=None, residual=None,
               residual_first: bool = False, groups: int = 1):
    y = F.conv2d(x.float(), w.float(), None if bias is None else bias.float(), stride, padding, dilation, groups)
    if residual is not None and residual_first:
        y = y + residual.float()
    y = _act(y, act)
    if residual is not None and not residual_first:
        y = y + residual.float()
    return y.to(x.dtype)


def rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos0: int = 0) -> torch.Tensor:
    """rotate_half rotary on x [B, S, H, D] with tables [>= pos0 + S, D]."""
    S, D = x.shape[1], x.shape[-1]
    c = cos[pos0:pos0 + S].float()[None, :, None, :]
    s = sin[pos0:pos0 + S].float()[None, :, None, :]
    xf = x.float()
    rot = torch.cat([-xf[..., D // 2:], xf[..., :D // 2]], dim=-1)
    return (xf * c + rot * s).to(x.dtype)


def sdpa_ref(q, k, v, causal: bool = False, scale: float | None = None, rope=None) -> torch.Tensor:
    """q [B, Sq, H, D], k / v [B, Skv, Hkv, D] -> [B, Sq, H, D] in fp32 math."""
    B, Sq, H, D = q.shape
    Skv, Hkv = k.shape[1], k.shape[2]
    qf, kf, vf = q.float(), k.float(), v.float()
    if rope is not None:
        cos, sin = rope[0], rope[1]
        qf = rope_ref(qf, cos, sin, Skv - Sq)
        kf = rope_ref(kf, cos, sin, 0)
    if Hkv != H:
        kf = kf.repeat_interleave(H // Hkv, dim=2)
        vf = vf.repeat_interleave(H // Hkv, dim=2)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * scale
    if causal:
        i = torch.arange(Sq, device=q.device)[:, None] + (Skv - Sq)
        j = torch.arange(Skv, device=q.device)[None, :]
        s = s.masked_fill(j > i, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, vf).to(q.dtype)


def rmsnorm_ref(x, weight, eps=1e-6):
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (weight.float() * y.to(x.dtype).float()).to(x.dtype)


def linear_rms_ref(x, wg, bias=None, act=None, eps=1e-6):
    xf = x.float()
    y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)) @ wg.float().t()
    if bias is not None:
        y = y + bias.float()
    return _act(y, act).to(x.dtype)


# ------------------------------------------------------------------ gather / row kernels
def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    """table[ids] for int ids of any shape; out [*ids.shape, D]."""
    if not table.is_cuda:
        return F.embedding(ids.long(), table)
    V, D = table.shape
    ids32 = ids.to(torch.int32).contiguous()
    out = torch.empty((*ids.shape, D), dtype=table.dtype, device=table.device)
    row_bytes = D * table.element_size()
    if row_bytes % 16 or not table.is_contiguous():
        raise ValueError("native embedding needs a contiguous table with 16-byte rows")
    _lib.check(_lib.lib().nos_embedding(ids32.data_ptr(), table.data_ptr(), out.data_ptr(), ids32.numel(), V,
                                        row_bytes, _stream()), "nos_embedding")
    return out


def rmsnorm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    if not x.is_cuda:
        return rmsnorm_ref(x, weight, eps)
    D = x.shape[-1]
    x2 = x.reshape(-1, D)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    w = weight.to(x.dtype).contiguous()
    out = torch.empty(x2.shape, dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib().nos_rmsnorm(x2.data_ptr(), w.data_ptr(), out.data_ptr(), x2.shape[0], D, x2.stride(0), D,
                                      float(eps), _bf(x), _stream()), "nos_rmsnorm")
    return out.view(x.shape)


UNARY_CODES = {"relu": 1, "sigmoid": 2, "silu": 3, "gelu": 4, "tanh": 5, "exp": 6, "neg": 7}


def unary(x: torch.Tensor, op: str, dtype: torch.dtype) -> torch.Tensor:
    """``op`` (a :data:`UNARY_CODES` activation) of fp32 / bf16 x into a
    ``dtype`` tensor: evaluated in fp32 and rounded once, in one pass on the
    GPU (a cast beside an activation costs no launch of its own)."""
    if not x.is_cuda:
        xf = x.float()
        y = {"relu": F.relu, "sigmoid": torch.sigmoid, "silu": F.silu, "gelu": F.gelu, "tanh": torch.tanh,
             "exp": torch.exp, "neg": torch.neg}[op](xf)
        return y.to(dtype)
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    if not out.numel():
        return out
    N = x.shape[-1] if x.dim() else 1
    try:   # rows at a uniform stride (e.g. a column slice of a merged GEMM's output): read in place
        x2 = x.view(-1, N) if x.dim() > 1 else None
    except RuntimeError:
        x2 = None
    if x2 is not None and not x.is_contiguous() and x2.stride(-1) == 1:
        _lib.check(_lib.lib().nos_unary_rows(x2.data_ptr(), x2.stride(0), _bf(x2), out.data_ptr(),
                                             int(dtype == torch.bfloat16), x2.shape[0], N, UNARY_CODES[op], _stream()),
                   "nos_unary_rows")
        return out
    xc = x.contiguous()
    _lib.check(_lib.lib().nos_unary(xc.data_ptr(), _bf(xc), out.data_ptr(), int(dtype == torch.bfloat16),
                                    xc.numel(), UNARY_CODES[op], _stream()), "nos_unary")
    return out


def glu(a: torch.Tensor, b: torch.Tensor, op: str = "silu") -> torch.Tensor:
    """f(a) * b in one pass (SwiGLU: silu(gate) * up), a and b of one shape
    and dtype; rows of a and b may be strided (column slices of one GEMM)."""
    f = {"relu": F.relu, "sigmoid": torch.sigmoid, "silu": F.silu, "gelu": F.gelu}[op]
    if not a.is_cuda or a.shape != b.shape or a.dtype != b.dtype or a.dtype not in (torch.float32, torch.bfloat16):
        return (f(a.float()) * b.float()).to(a.dtype)
    N = a.shape[-1]

    def rows(t):
        t2 = t.reshape(-1, N) if t.is_contiguous() else None
        if t2 is None:
            try:
                t2 = t.view(-1, N)
            except RuntimeError:
                t2 = t.contiguous().view(-1, N)
        return t2 if t2.stride(-1) == 1 else t2.contiguous()

    a2, b2 = rows(a), rows(b)
    out = torch.empty(a.shape, dtype=a.dtype, device=a.device)
    if out.numel():
        _lib.check(_lib.lib().nos_glu(a2.data_ptr(), a2.stride(0), b2.data_ptr(), b2.stride(0), out.data_ptr(),
                                      a2.shape[0], N, UNARY_CODES[op], _bf(a), _stream()), "nos_glu")
    return out


def softmax(x: torch.Tensor) -> torch.Tensor:
    """softmax over the last dim."""
    if not x.is_cuda:
        return torch.softmax(x.float(), dim=-1).to(x.dtype)
    L = x.shape[-1]
    x2 = x.reshape(-1, L)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    out = torch.empty(x2.shape, dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib().nos_softmax(x2.data_ptr(), out.data_ptr(), x2.shape[0], L, x2.stride(0), L, _bf(x),
                                      _stream()), "nos_softmax")
    return out.view(x.shape)


def _rows_view(x: torch.Tensor) -> tuple[int, int]:
    """(token row stride, batch stride) of x [B, S, H, D] whose heads are
    contiguous per token (e.g. a slice of a fused projection)."""
    B, S, H, D = x.shape
    if x.stride(-1) != 1 or x.stride(-2) != D:
        raise ValueError("x needs contiguous heads per token")
    return x.stride(1), x.stride(0)


def rotary(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """rotate_half rotary embedding of x [B, S, H, D] with fp32 tables [S, D]."""
    if not x.is_cuda:
        return rope_ref(x, cos, sin)
    B, S, H, D = x.shape
    if x.stride(-1) != 1 or x.stride(-2) != D:
        x = x.contiguous()
    ld, bs = _rows_view(x)
    c, s = cos.float().contiguous(), sin.float().contiguous()
    if c.shape[0] < S or c.shape[1] != D:
        raise ValueError(f"rotary tables must be [>= {S}, {D}]")
    out = torch.empty((B, S, H, D), dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib().nos_rotary(x.data_ptr(), c.data_ptr(), s.data_ptr(), out.data_ptr(), B, S, H, D, ld, bs,
                                     _bf(x), _stream()), "nos_rotary")
    return out


# ------------------------------------------------------------------ GEMM-class ops (h3)
def _gemm_batched(ap, rinv, sa, srinv, wp, csc, sw, scsc, out, M, N, K, nb, epi, bias=None, residual=None,
                  ldc=None, sc=None, ldr=None, sr=None, sbias=0, c_off=0, w_off=0, wr_off=0) -> None:
    """``c_off`` / ``w_off`` / ``wr_off``: element offsets of batch element
    0's C, W-operand planes and W-operand row scales (a grouped conv's image
    n; the planes keep the whole tensor's plane stride)."""
    L = _lib.lib()
    ldc = N if ldc is None else ldc
    rc = L.nos_gemm_f32h3_batched(ap.data_ptr(), K, ap[0].numel(), sa,
                                  rinv.data_ptr(), srinv, 0.0, wp.data_ptr() + 2 * w_off, K, wp[0].numel(), sw,
                                  csc.data_ptr() + 4 * wr_off, scsc, _ptr(bias), sbias, _ptr(residual), ldr or ldc,
                                  sr or 0, out.data_ptr() + 4 * c_off, ldc, M * ldc if sc is None else sc, M, N, K, nb,
                                  epi, _stream())
    _lib.check(rc, "nos_gemm_f32h3_batched")


def conv2d(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, stride=(1, 1), padding=(0, 0),
           dilation=(1, 1), act: str | None = None, residual: torch.Tensor | None = None,
           w2: torch.Tensor | None = None, residual_first: bool = False, groups: int = 1) -> torch.Tensor:
    """act(conv2d(x, w) + bias) + residual, NCHW
    (``residual_first``: act(conv2d(x, w) + bias + residual), a ResNet block's
    tail).  ``w2``: the weight as a [OC, Kp] fp32 matrix (K = C/groups*KH*KW
    zero-padded to 32), which the compiler keeps as a constant so its split
    planes are cached.  ``groups``: the image seen as N*groups images of
    C/groups channels (each group's channels are contiguous in NCHW), one
    batched GEMM per image over the groups (depthwise: groups = C)."""
    if not x.is_cuda:
        return conv2d_ref(x, w, bias, stride, padding, dilation, act, residual, residual_first, groups)
    dt = x.dtype
    xf = _f32(x).contiguous()
    N, C, H, W = xf.shape
    OC, Cg, KH, KW = w.shape
    G = groups
    if C != Cg * G or OC % G:
        raise ValueError(f"conv2d groups={G}: input channels {C} / weight {tuple(w.shape)} do not match")
    OCg = OC // G
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    OH = (H + 2 * ph - dh * (KH - 1) - 1) // sh + 1
    OW = (W + 2 * pw - dw * (KW - 1) - 1) // sw + 1
    K = Cg * KH * KW
    Kp = -(-K // 32) * 32
    if w2 is None:
        w2 = _pad_k(_f32(w).reshape(OC, K)).contiguous()
    if w2.shape != (OC, Kp) or w2.dtype != torch.float32:
        raise ValueError(f"conv weight matrix must be fp32 [{OC}, {Kp}]")
    P = OH * OW
    NG = N * G
    planes = torch.empty((2, NG * P, Kp), dtype=torch.float16, device=x.device)
    prinv = torch.empty((NG * P,), dtype=torch.float32, device=x.device)
    L = _lib.lib()
    _lib.check(L.nos_im2col_h3(xf.data_ptr(), planes.data_ptr(), NG * P * Kp, prinv.data_ptr(), NG, Cg, H, W, KH, KW,
                               sh, sw, ph, pw, dh, dw, Kp, _stream()), "nos_im2col_h3")
    wp, wsc = split_f32_weight_h3(w2)
    out = torch.empty((N, OC, OH, OW), dtype=torch.float32, device=x.device)
    epi = _act_epi(act) | (EPI_BIAS_ROW if bias is not None else 0)
    if residual is not None:
        epi |= EPI_RESID_PRE if residual_first else EPI_RESID
    b = _f32(bias).contiguous() if bias is not None else None
    r = _f32(residual).contiguous() if residual is not None else None
    if r is not None and r.shape != out.shape:
        raise ValueError(f"residual must be {tuple(out.shape)}")
    if G == 1:
        # out[n] = W [OC, Kp] . patches[n]^T: A = the weight (shared, stride 0), W-operand = image n's patches
        _gemm_batched(wp, wsc, 0, 0, planes, prinv, P * Kp, P, out, OC, P, Kp, N, epi, bias=b, residual=r,
                      ldc=P, sc=OC * P, ldr=P, sr=OC * P)
    else:
        # per image: batch = the groups -- A = group g's weight rows, W-operand
        # = group g's patches (image n*G + g of the im2col), C = its OCg channels
        for n in range(N):
            _gemm_batched(wp, wsc, OCg * Kp, OCg, planes, prinv, P * Kp, P, out, OCg, P, Kp, G, epi,
                          bias=b, residual=r[n:] if r is not None else None, ldc=P, sc=OCg * P, ldr=P,
                          sr=OCg * P, sbias=OCg, c_off=n * OC * P, w_off=n * G * P * Kp, wr_off=n * G * P)
    return out if dt == torch.float32 else out.to(dt)


def patches(x: torch.Tensor, ph: int, pw: int, dtype: torch.dtype = torch.float32, hp: int | None = None,
            wp: int | None = None):
    """A ViT's patch rows of an fp32 NCHW image: [N, (H/ph)(W/pw), C ph pw]
    with columns (c, dy, dx), in ``dtype``.  On the GPU one im2col pass over
    the image (stride = kernel, no padding; a cropped view is read through
    its strides, no contiguous copy): fp32 under h3 math as the GEMM's A
    planes (:class:`ops.H3Planes`), bf16 as the GEMM's bf16 operand (the cast
    folded in); otherwise the PyTorch views + copy.  ``hp`` x ``wp`` patches
    from the image's top-left corner (default: as many as fit)."""
    from .. import ops

    N, C, H, W = x.shape
    hp = H // ph if hp is None else hp
    wp = W // pw if wp is None else wp
    if not (0 < hp * ph <= H and 0 < wp * pw <= W):
        raise ValueError(f"patches: {hp}x{wp} patches of {ph}x{pw} exceed the {H}x{W} image")
    K = C * ph * pw
    P = hp * wp
    bf = dtype == torch.bfloat16
    gpu = x.is_cuda and x.dtype == torch.float32 and (bf or (dtype == torch.float32 and ops.h3_planes_active()
                                                                and K % 32 == 0))
    if not gpu:
        x = x[:, :, :hp * ph, :wp * pw]
        y = x.reshape(N, C, hp, ph, wp, pw).permute(0, 2, 4, 1, 3, 5).reshape(N, P, K)
        return y.to(dtype)
    if x.stride(3) != 1:
        x = x.contiguous()
    sN, sC, sH = x.stride(0), x.stride(1), x.stride(2)
    if bf:
        out = torch.empty((N, P, K), dtype=torch.bfloat16, device=x.device)
        _lib.check(_lib.lib().nos_im2col(x.data_ptr(), sN, sC, sH, out.data_ptr(), 0, None, N, C, hp * ph, wp * pw, ph,
                                         pw, ph, pw, 0, 0, 1, 1, K, 1, _stream()), "nos_im2col")
        return out
    planes = torch.empty((2, N * P, K), dtype=torch.float16, device=x.device)
    prinv = torch.empty((N * P,), dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().nos_im2col(x.data_ptr(), sN, sC, sH, planes.data_ptr(), N * P * K, prinv.data_ptr(), N, C,
                                     hp * ph, wp * pw, ph, pw, ph, pw, 0, 0, 1, 1, K, 0, _stream()), "nos_im2col")
    return ops.H3Planes(planes, prinv, 0.0, (N, P, K))


COLS_NCH = 32   # gemm_f32h.hip: row chunks of the column maxima (nos_split_cols_h3's work buffer)


def _split_cols_h3(x3: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """The columns of fp32 x3 [nb, R, C] as h3 plane rows (``nos_split_cols_h3``):
    planes [2, nb * C, ceil32(R)] (zero-padded), 1 / row scale [nb * C] -- the
    split of x3's transpose without a transposed copy."""
    nb, R, C = x3.shape
    if x3.stride(-1) != 1 or (nb > 1 and x3.stride(0) < (R - 1) * x3.stride(1) + C):
        x3 = x3.contiguous()
    Rp = _pad_k_len(R)
    planes = torch.empty((2, nb * C, Rp), dtype=torch.float16, device=x3.device)
    rinv = torch.empty((nb * C,), dtype=torch.float32, device=x3.device)
    work = torch.empty((COLS_NCH * nb * C,), dtype=torch.float32, device=x3.device)
    _lib.check(_lib.lib().nos_split_cols_h3(x3.data_ptr(), x3.stride(1), x3.stride(0) if nb > 1 else 0, R, C, nb,
                                            planes.data_ptr(), Rp, planes[0].numel(), rinv.data_ptr(),
                                            work.data_ptr(), _stream()), "nos_split_cols_h3")
    return planes, rinv


def _rows_h3(x3: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """The rows of fp32 x3 [nb, R, C] as h3 plane rows [2, nb * R, ceil32(C)]."""
    R, C = x3.shape[1:]
    x2 = _pad_k(x3).reshape(-1, _pad_k_len(C))
    return _split_rows_h3(x2 if x2.stride(-1) == 1 and x2.is_contiguous() else x2.contiguous(), ln=False)


def mm(a: torch.Tensor, b: torch.Tensor, a_t: bool = False, b_t: bool = False) -> torch.Tensor:
    """op(a) @ op(b) on the h3 batched GEMM, op(x) = x^T (last two dims) when
    the flag is set; batch dims equal, or one side 2-D.  A transposed A or a
    plain B operand is split by columns (``nos_split_cols_h3``), so no
    operand is ever copied into its transpose (training's dX = dY W and
    dW = dY^T X, attention's P V and P^T dO)."""
    if not a.is_cuda:
        A = a.transpose(-1, -2) if a_t else a
        B = b.transpose(-1, -2) if b_t else b
        return (A.float() @ B.float()).to(a.dtype)
    dt = a.dtype
    M, K = (a.shape[-1], a.shape[-2]) if a_t else (a.shape[-2], a.shape[-1])
    N, Kb = (b.shape[-2], b.shape[-1]) if b_t else (b.shape[-1], b.shape[-2])
    ba, bb = a.shape[:-2], b.shape[:-2]
    if Kb != K or (ba and bb and ba != bb):
        raise ValueError(f"mm shapes: {tuple(a.shape)}{'^T' if a_t else ''} @ {tuple(b.shape)}{'^T' if b_t else ''}")
    bshape = ba or bb
    nb = math.prod(bshape) if bshape else 1
    a3, b3 = _f32(a).reshape(-1, *a.shape[-2:]), _f32(b).reshape(-1, *b.shape[-2:])
    ap, arinv = _split_cols_h3(a3) if a_t else _rows_h3(a3)      # A rows: op(a)'s M rows of K
    bp, brinv = _rows_h3(b3) if b_t else _split_cols_h3(b3)      # W rows: op(b)'s N columns of K
    Kp = ap.shape[2]
    out = torch.empty((nb, M, N), dtype=torch.float32, device=a.device)
    _gemm_batched(ap, arinv, M * Kp if ba else 0, M if ba else 0, bp, brinv, N * Kp if bb else 0, N if bb else 0,
                  out, M, N, Kp, nb, 0)
    out = out.view(*bshape, M, N)
    return out if dt == torch.float32 else out.to(dt)


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [..., M, K] @ b [..., K, N]; batch dims equal, or one side 2-D."""
    return mm(a, b)


def _pad_k_len(k: int) -> int:
    return -(-k // 32) * 32


def linear_rms(x: torch.Tensor, wg: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
               eps: float = 1e-6, glu: bool = False) -> torch.Tensor:
    """act(RMSNorm(x) @ (W * gamma)^T + b): the row statistics in the h3 split
    pre-pass (``nos_split_rows_h3`` mode 2), gamma folded into ``wg``.
    ``glu``: ``wg`` is a merged [gate; up] weight and the result is
    silu(gate) * up (the GEMV's epilogue for decode rows)."""
    if glu:
        x2g = _f32(x).reshape(-1, x.shape[-1])
        if not (x.is_cuda and x2g.shape[0] <= GEMV_MAX_ROWS and gemv_ok(x2g.contiguous(), wg)):
            y = linear_rms(x, wg, bias, act, eps)
            h = y.shape[-1] // 2
            return (F.silu(y[..., :h].float()) * y[..., h:].float()).to(y.dtype)
    if not x.is_cuda:
        return linear_rms_ref(x, wg, bias, act, eps)
    dt = x.dtype
    K = x.shape[-1]
    N = wg.shape[0]
    if K % 32:
        raise ValueError("native linear_rms needs K % 32 == 0")
    x2 = _f32(x).reshape(-1, K)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    M = x2.shape[0]
    if glu and not gemv_ok(x2, wg):
        x2 = x2.clone()   # an aligned copy: the GLU form exists only on the GEMV
    if M <= GEMV_MAX_ROWS and gemv_ok(x2, wg):   # a decode step: the RMS statistics in the GEMV's prologue
        out = gemv(x2, wg, bias, act, rms_eps=float(eps) or 1e-30, glu=glu)
        out = out.view(*x.shape[:-1], N // 2 if glu else N)
        return out if dt == torch.float32 else out.to(dt)
    planes = torch.empty((2, M, K), dtype=torch.float16, device=x.device)
    rinv = torch.empty((M,), dtype=torch.float32, device=x.device)
    eln = 14 - math.frexp(math.sqrt(K))[1]
    _lib.check(_lib.lib().nos_split_rows_h3(x2.data_ptr(), x2.stride(0), planes.data_ptr(), K, M * K, rinv.data_ptr(),
                                            M, K, 2, float(eps), eln, _stream()), "nos_split_rows_h3")
    wp, csc = split_f32_weight_h3(wg)
    out = torch.empty((M, N), dtype=torch.float32, device=x.device)
    b = _f32(bias).contiguous() if bias is not None else None
    epi = _act_epi(act) | (EPI_BIAS if b is not None else 0)
    _gemm_batched(planes, rinv, 0, 0, wp, csc, 0, 0, out, M, N, K, 1, epi, bias=b)
    out = out.view(*x.shape[:-1], N)
    return out if dt == torch.float32 else out.to(dt)


_ROPE_BOUND: dict[int, tuple] = {}


def _rope_bound(cos: torch.Tensor, sin: torch.Tensor) -> float:
    key = id(cos)
    hit = _ROPE_BOUND.get(key)
    if hit is not None and hit[0] is sin and hit[1] == cos._version:
        return hit[2]
    b = float(cos.abs().max() + sin.abs().max())
    _ROPE_BOUND[key] = (sin, cos._version, b)
    return b


def sdpa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False, scale: float | None = None,
         rope: tuple | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """softmax(scale q k^T [causal]) v: q [B, Sq, H, D], k / v [B, Skv, Hkv, D]
    (heads contiguous per token; any token / batch strides, e.g. slices of a
    fused QKV projection), D = 64 or 128, H % Hkv == 0.  ``rope`` = (cos, sin)
    fp32 tables [Skv, D]: q and k are rotated first (inside the kernels)."""
    if not q.is_cuda:
        return sdpa_ref(q, k, v, causal, scale, rope)
    dt = q.dtype
    B, Sq, H, D = q.shape
    Skv, Hkv = k.shape[1], k.shape[2]
    if D not in (64, 128) or H % Hkv or v.shape != k.shape or k.shape[0] != B or k.shape[3] != D:
        raise ValueError(f"native sdpa: head_dim 64/128, H % Hkv == 0; got q {tuple(q.shape)}, k {tuple(k.shape)}")
    qf, kf, vf = (_f32(t) for t in (q, k, v))
    try:
        (ldq, bsq), (ldk, bsk), (ldv, bsv) = _rows_view(qf), _rows_view(kf), _rows_view(vf)
    except ValueError:
        qf, kf, vf = qf.contiguous(), kf.contiguous(), vf.contiguous()
        (ldq, bsq), (ldk, bsk), (ldv, bsv) = _rows_view(qf), _rows_view(kf), _rows_view(vf)
    if any(s % 4 for s in (ldq, bsq, ldk, bsk, ldv, bsv)) or any(t.data_ptr() % 16 for t in (qf, kf, vf)):
        qf, kf, vf = qf.contiguous(), kf.contiguous(), vf.contiguous()
        (ldq, bsq), (ldk, bsk), (ldv, bsv) = _rows_view(qf), _rows_view(kf), _rows_view(vf)
    if out is None or out.dtype != torch.float32:
        o = torch.empty((B, Sq, H, D), dtype=torch.float32, device=q.device)
    else:
        o = out
    L = _lib.lib()
    nbytes = int(L.nos_attn_h3g_workspace(B, H, Hkv, Sq, Skv, D))
    ws = torch.empty((nbytes + 256,), dtype=torch.uint8, device=q.device)
    wptr = (ws.data_ptr() + 255) // 256 * 256
    rc_, rs_, rb = None, None, 0.0
    if rope is not None:
        rc_, rs_ = rope[0], rope[1]
        if rc_.dtype != torch.float32 or not rc_.is_contiguous() or rc_.shape != (Skv, D) or rs_.shape != (Skv, D):
            raise ValueError(f"rope tables must be contiguous fp32 [{Skv}, {D}]")
        rb = _rope_bound(rc_, rs_)
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    rc = L.nos_attn_h3g(qf.data_ptr(), ldq, bsq, kf.data_ptr(), ldk, bsk, vf.data_ptr(), ldv, bsv, o.data_ptr(),
                        o.stride(1), o.stride(0), B, H, Hkv, Sq, Skv, D, int(bool(causal)), float(sc), _ptr(rc_),
                        _ptr(rs_), float(rb), wptr, nbytes, _stream())
    _lib.check(rc, "nos_attn_h3g")
    if out is not None and out is not o:
        out.copy_(o)
        return out
    return o if dt == torch.float32 else o.to(dt)


# ------------------------------------------------------------------ stateful decoding (decode.hip)
def _i32_pos(pos: torch.Tensor, B: int) -> torch.Tensor:
    if pos.dtype != torch.int32 or pos.shape != (B,) or not pos.is_contiguous():
        raise ValueError(f"positions must be a contiguous i32 [{B}] tensor, got {pos.dtype} {tuple(pos.shape)}")
    return pos


def kv_write(cache: torch.Tensor, x: torch.Tensor, pos: torch.Tensor, rope: tuple | None = None,
             second: tuple | None = None) -> torch.Tensor:
    """cache[b, pos[b] + s] = x[b, s] in place (rows past the cache dropped);
    ``rope`` = (cos, sin) fp32 tables: x rotated at those positions first.
    ``second`` = (cache2, x2): a second, unrotated write of the same shape in
    the same launch (a layer's V beside its K).  Returns ``cache``."""
    from ..podserver.program.reference import kv_write_ref, rotary_at_ref

    if not cache.is_cuda:
        if second is not None:
            kv_write_ref(second[0], second[1], pos)
        return kv_write_ref(cache, rotary_at_ref(x, rope[0], rope[1], pos) if rope else x, pos)
    B, L, H, D = cache.shape
    S = x.shape[1]
    if x.shape[0] != B or x.shape[2:] != cache.shape[2:] or not cache.is_contiguous():
        raise ValueError(f"kv_write: x {tuple(x.shape)} does not fit the cache {tuple(cache.shape)}")
    try:
        ldx, bsx = _rows_view(x)
    except ValueError:
        x = x.contiguous()
        ldx, bsx = _rows_view(x)
    c = s_ = None
    R = 0
    if rope is not None:
        c, s_ = rope[0].float().contiguous(), rope[1].float().contiguous()
        R = c.shape[0]
    x2p, ld2, bs2, c2p = None, 0, 0, None
    if second is not None:
        c2, x2 = second
        if c2.shape != cache.shape or c2.dtype != cache.dtype or x2.shape != x.shape or x2.dtype != x.dtype \
                or not c2.is_contiguous():
            raise ValueError("kv_write: the second write must match the first's shapes and dtypes")
        try:
            ld2, bs2 = _rows_view(x2)
        except ValueError:
            x2 = x2.contiguous()
            ld2, bs2 = _rows_view(x2)
        x2p, c2p = x2.data_ptr(), c2.data_ptr()
    _lib.check(_lib.lib().nos_kv_write(x.data_ptr(), _bf(x), ldx, bsx, cache.data_ptr(), _bf(cache),
                                       _i32_pos(pos, B).data_ptr(), _ptr(c), _ptr(s_), R, B, S, H, D, L, x2p, ld2, bs2,
                                       c2p, _stream()), "nos_kv_write")
    return cache


def rotary_at(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """rotate_half rotary of x [B, S, H, D] at positions pos[b] + s (table rows clamped)."""
    from ..podserver.program.reference import rotary_at_ref

    if not x.is_cuda:
        return rotary_at_ref(x, cos, sin, pos)
    B, S, H, D = x.shape
    try:
        ldx, bsx = _rows_view(x)
    except ValueError:
        x = x.contiguous()
        ldx, bsx = _rows_view(x)
    c, s_ = cos.float().contiguous(), sin.float().contiguous()
    if c.shape[1] != D or s_.shape != c.shape:
        raise ValueError(f"rotary tables must be [positions, {D}]")
    out = torch.empty((B, S, H, D), dtype=x.dtype, device=x.device)
    _lib.check(_lib.lib().nos_rotary_pos(x.data_ptr(), ldx, bsx, out.data_ptr(), _i32_pos(pos, B).data_ptr(),
                                         c.data_ptr(), s_.data_ptr(), c.shape[0], B, S, H, D, _bf(x), _stream()),
               "nos_rotary_pos")
    return out


class DecodePartials:
    """The decode attention's split partials (``sdpa_cache(partials=True)``):
    ws [B x Hkv, NS, G, D + 2] fp32 -- consumed by :func:`gemv_partials`,
    which combines them in its x staging (the combine launch folded into the
    O-projection).  ``shape``: the attention output's [B, 1, H, D]."""

    def __init__(self, ws, NS, G, Hkv, D, shape, dtype):
        self.ws, self.NS, self.G, self.Hkv, self.D, self.shape, self.dtype = ws, NS, G, Hkv, D, tuple(shape), dtype


def sdpa_cache(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, pos: torch.Tensor, scale: float | None = None,
               rope: tuple | None = None, fresh: tuple | None = None, sync: torch.Tensor | None = None,
               partials: bool = False):
    """Query i of sequence b, at position pos[b] + i, attends the cached keys
    0 .. pos[b] + i: q [B, Sq, H, D], caches [B, L, Hkv, D] (fp32 / bf16).
    ``rope`` = (cos, sin): q rotated at its positions inside the kernel.
    ``fresh`` = (k, v) [B, Sq, Hkv, D]: the step's own K / V rows, written
    into the caches at the positions (K rotated by ``rope``) by the same
    launch -- a ``kv_write`` pair folded in.  ``sync``: a zeroed int32
    device buffer of >= B x Hkv counters owned by the call site (the kernel
    leaves it zero): the split combine runs in the decode launch's last
    workgroup per K / V head instead of a launch of its own.  ``partials``
    (CUDA, fp32 q, one query token): no combine -- returns the splits'
    :class:`DecodePartials` for :func:`gemv_partials`.  The
    flash-decoding kernel (decode.hip) for CUDA tensors, fp32 math."""
    from ..podserver.program.reference import kv_write_ref, rotary_at_ref, sdpa_cache_ref

    if not q.is_cuda:
        if fresh is not None:
            kv_write_ref(kc, rotary_at_ref(fresh[0], rope[0], rope[1], pos) if rope else fresh[0], pos)
            kv_write_ref(vc, fresh[1], pos)
        return sdpa_cache_ref(rotary_at_ref(q, rope[0], rope[1], pos) if rope else q, kc, vc, pos, scale)
    B, Sq, H, D = q.shape
    L, Hkv = kc.shape[1], kc.shape[2]
    if (kc.shape != vc.shape or kc.dtype != vc.dtype or kc.shape[0] != B or kc.shape[3] != D or H % Hkv
            or D not in (64, 128) or not kc.is_contiguous() or not vc.is_contiguous()):
        raise ValueError(f"sdpa_cache: q {tuple(q.shape)} vs caches {tuple(kc.shape)}")
    try:
        ldq, bsq = _rows_view(q)
    except ValueError:
        q = q.contiguous()
        ldq, bsq = _rows_view(q)
    c = s_ = None
    R = 0
    if rope is not None:
        c, s_ = rope[0].float().contiguous(), rope[1].float().contiguous()
        R = c.shape[0]
    L_ = _lib.lib()
    nb = int(L_.nos_attn_decode_workspace(B, H, Hkv, Sq, L, D))
    ws = torch.empty((max(nb, 4) // 4,), dtype=torch.float32, device=q.device)
    out = torch.empty((B, Sq, H, D), dtype=q.dtype, device=q.device)
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    kn = vn = None
    ldk = ldv = bsk = bsv = nbf = 0
    if fresh is not None:
        kn, vn = fresh
        if kn.shape != (B, Sq, Hkv, D) or vn.shape != kn.shape or kn.dtype != vn.dtype:
            raise ValueError(f"sdpa_cache: fresh K / V {tuple(kn.shape)} for q {tuple(q.shape)}")
        try:
            ldk, bsk = _rows_view(kn)
        except ValueError:
            kn = kn.contiguous()
            ldk, bsk = _rows_view(kn)
        try:
            ldv, bsv = _rows_view(vn)
        except ValueError:
            vn = vn.contiguous()
            ldv, bsv = _rows_view(vn)
        nbf = _bf(kn)
    if sync is not None and (not sync.is_cuda or sync.dtype != torch.int32 or not sync.is_contiguous()
                             or sync.numel() < B * Hkv):
        raise ValueError(f"sdpa_cache: sync needs >= {B * Hkv} contiguous int32 device counters")
    if partials and (Sq != 1 or sync is not None or q.dtype != torch.float32):
        raise ValueError("sdpa_cache: partials need one fp32 query token and no sync")
    _lib.check(L_.nos_attn_decode(q.data_ptr(), _bf(q), ldq, bsq, kc.data_ptr(), vc.data_ptr(), _bf(kc),
                                  _i32_pos(pos, B).data_ptr(), _ptr(c), _ptr(s_), R, out.data_ptr(), _bf(out), B, H,
                                  Hkv, Sq, L, D, float(sc), ws.data_ptr(), ws.numel() * 4, _ptr(kn), _ptr(vn), nbf,
                                  ldk, bsk, ldv, bsv, Sq if fresh is not None else 0, _ptr(sync),
                                  sync.numel() if sync is not None else 0, int(bool(partials)), _stream()),
               "nos_attn_decode")
    if partials:
        return DecodePartials(ws, (L + 127) // 128, H // Hkv, Hkv, D, (B, Sq, H, D), q.dtype)
    return out


def pos_update(pos: torch.Tensor, add: bool, n: int) -> torch.Tensor:
    """pos += n (``add``) or pos = n, in place; returns ``pos``."""
    if not pos.is_cuda:
        return pos.add_(n) if add else pos.fill_(n)
    _lib.check(_lib.lib().nos_pos_update(_i32_pos(pos, pos.shape[0]).data_ptr(), pos.shape[0], int(bool(add)), int(n),
                                         _stream()), "nos_pos_update")
    return pos


def argmax(x: torch.Tensor, pos: torch.Tensor | None = None, pos_n: int = 0) -> torch.Tensor:
    """Index of the maximum over the last dim (first on ties), i32.
    ``pos`` (i32, one counter per row of x): advanced by ``pos_n`` in the same
    launch (a decode step's closing ``pos_add`` folded in)."""
    if not x.is_cuda:
        if pos is not None:
            pos.add_(pos_n)
        return x.float().argmax(dim=-1).to(torch.int32)
    L = x.shape[-1]
    x2 = x.reshape(-1, L)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    if pos is not None and (pos.numel() != x2.shape[0] or pos.dtype != torch.int32 or not pos.is_contiguous()):
        raise ValueError(f"argmax: pos needs one i32 counter per row ({x2.shape[0]})")
    out = torch.empty(x.shape[:-1], dtype=torch.int32, device=x.device)
    _lib.check(_lib.lib().nos_argmax(x2.data_ptr(), _bf(x2), x2.shape[0], L, x2.stride(0), out.data_ptr(), _ptr(pos),
                                     int(pos_n), _stream()), "nos_argmax")
    return out


GEMV_MAX_ROWS = 8
EPI_SILU = 64  # decode.hip's GEMV: SiLU epilogue
EPI_GLU = 256  # decode.hip's GEMV: W = [gate; up], y = silu(gate) * up


def gemv_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    """Whether the skinny-GEMM kernel takes this [M, K] x [N, K] product."""
    M, K = x2.shape
    return (x2.is_cuda and 0 < M <= GEMV_MAX_ROWS and K % 4 == 0 and M * K * 4 <= 65536 and x2.stride(-1) == 1
            and w.stride(-1) == 1 and x2.stride(0) % 4 == 0 and w.stride(0) % 4 == 0
            and x2.dtype in (torch.float32, torch.bfloat16) and w.dtype in (torch.float32, torch.bfloat16)
            and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def gemv(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
         residual: torch.Tensor | None = None, out: torch.Tensor | None = None, rms_eps: float = 0.0,
         glu: bool = False) -> torch.Tensor:
    """y [M, N] = act(rms(x) [M, K] W^T + b) + R for M <= 8 (:func:`gemv_ok`):
    the weight-streaming kernel of a decode step, exact fp32 math; y, R in
    x's dtype, bias in W's.  ``rms_eps`` > 0: x rows RMS-normalised first
    (RMSNorm folded into the GEMM, gamma in W)."""
    M, K = x2.shape
    N = w.shape[0]
    y = out if out is not None else torch.empty((M, N // 2 if glu else N), dtype=x2.dtype, device=x2.device)
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_RESID if residual is not None else 0) | (EPI_GLU if glu else 0)
    epi |= {"gelu": EPI_GELU, "relu": EPI_RELU, "silu": EPI_SILU}.get(act or "", 0)
    b = None if bias is None else bias.to(w.dtype).contiguous()
    r = None if residual is None else residual.reshape(M, N).to(x2.dtype)
    if r is not None and r.stride(-1) != 1:
        r = r.contiguous()
    if y.dtype != x2.dtype or y.stride(-1) != 1:
        raise ValueError("gemv: out must be x's dtype with unit inner stride")
    _lib.check(_lib.lib().nos_gemv(x2.data_ptr(), _bf(x2), x2.stride(0), w.data_ptr(), _bf(w), w.stride(0), _ptr(b),
                                   _ptr(r), r.stride(0) if r is not None else 0, y.data_ptr(), y.stride(0), M, N, K,
                                   epi, float(rms_eps), _stream()), "nos_gemv")
    return y


def gemv_partials(p: DecodePartials, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
                  residual: torch.Tensor | None = None) -> torch.Tensor:
    """:func:`gemv` whose x [B, H x D] is the decode attention's output,
    combined from its split partials in the kernel's x staging
    (decode.hip ``parts_x4``, the combine kernel's arithmetic): y [B, N] fp32."""
    B, _, H, D = p.shape
    K = H * D
    N = w.shape[0]
    if w.shape[1] != K or w.stride(-1) != 1 or w.stride(0) % 4 or w.data_ptr() % 16 or B > GEMV_MAX_ROWS:
        raise ValueError(f"gemv_partials: W {tuple(w.shape)} for x [{B}, {K}]")
    y = torch.empty((B, N), dtype=torch.float32, device=w.device)
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_RESID if residual is not None else 0)
    epi |= {"gelu": EPI_GELU, "relu": EPI_RELU, "silu": EPI_SILU}.get(act or "", 0)
    b = None if bias is None else bias.to(w.dtype).contiguous()
    r = None if residual is None else residual.reshape(B, N).float()
    if r is not None and r.stride(-1) != 1:
        r = r.contiguous()
    _lib.check(_lib.lib().nos_gemv_partials(p.ws.data_ptr(), p.ws.numel(), p.NS, p.G, p.G, p.Hkv, D, 0, w.data_ptr(),
                                            _bf(w), w.stride(0), _ptr(b), _ptr(r), r.stride(0) if r is not None else 0,
                                            y.data_ptr(), y.stride(0), B, N, K, epi, _stream()), "nos_gemv_partials")
    return y


def set_attention_h3g_kvsplit(n: int) -> None:
    """Key splits of :func:`sdpa` (0 = auto: fill the CU slots)."""
    _lib.check(_lib.lib().nos_attn_h3g_set_kvsplit(int(n)), "nos_attn_h3g_set_kvsplit")


__all__ = ["glu", "kv_write", "rotary_at", "sdpa_cache", "pos_update", "argmax", "gemv", "gemv_ok", "gemv_partials",
           "DecodePartials", "conv2d", "matmul", "sdpa", "linear_rms", "embedding", "rmsnorm", "softmax", "rotary", "conv2d_ref",
           "sdpa_ref", "rope_ref", "rmsnorm_ref", "linear_rms_ref", "set_attention_h3g_kvsplit", "EPI_BIAS_ROW"]
