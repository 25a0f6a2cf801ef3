"""Differentiable ops of training tenants on the gfx950 kernels (training.py).

A training tenant's forward + backward + optimizer step is captured into one
HIP graph; round 5 ran its GEMMs on hipBLASLt and its attention as the
materialised ``softmax(QK^T)V`` (a B x H x S x S score tensor kept for
backward).  Here both run on ``libnos_hip.so``:

* :class:`H3Linear` -- ``y = x W^T + b``: the forward and BOTH backward GEMMs
  (``dX = dY W``, ``dW = dY^T X``) on the fp16x3 ("h3") batched GEMM
  (``ops.tenant.matmul``: every operand split into hi / lo planes per row by
  ``nos_split_rows_h3`` at run time -- the weights change every step, so no
  split is cached across replays);
* :class:`ChunkedAttention` -- attention with causal masking and grouped-query
  heads, forward and backward over query CHUNKS: per chunk of ``C`` query rows
  the scores ``Q_c K^T`` (h3 GEMM), the row log-sum-exp, ``P V``; backward
  recomputes ``P`` from the saved log-sum-exp (no S x S tensor is ever kept:
  the live scores are ``B x H x C x S``), then ``dV += P^T dO_c``,
  ``dP = dO_c V^T``, ``dS = P (dP - rowsum(dO_c O_c))``, ``dQ_c = dS K``,
  ``dK += dS^T Q_c`` -- the four products per chunk on the h3 GEMM;
* :class:`CrossEntropy` -- the classification loss from the rows'
  log-sum-exp (no softmax kernel; the round-5 step ran ``F.cross_entropy``).

The math is the textbook flash-attention backward (recompute from the
log-sum-exp), organised for the h3 GEMM's batched form.  CPU tensors take the
same code path on PyTorch matmuls (the numerics tests compare it with torch
autograd).
"""
from __future__ import annotations

import math

import torch

CHUNK = 512   # query rows per attention chunk (live scores: B x H x CHUNK x S fp32)


def _mm(a: torch.Tensor, b: torch.Tensor, a_t: bool = False, b_t: bool = False) -> torch.Tensor:
    """op(a) @ op(b) (op = transpose of the last two dims when flagged) on the
    h3 GEMM for CUDA tensors -- transposed operands split by columns, never
    copied (``ops.tenant.mm``); batch dims equal or one side 2-D."""
    if a.is_cuda:
        from ..ops import tenant as T

        return T.mm(a, b, a_t, b_t)
    return (a.transpose(-1, -2) if a_t else a) @ (b.transpose(-1, -2) if b_t else b)


class H3Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        y = _mm(x2, w, b_t=True)
        if b is not None:
            y = y + b
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        dx = _mm(dy2, w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = _mm(dy2, x2, a_t=True) if ctx.needs_input_grad[1] else None     # dY^T X, no transposed copies
        db = dy2.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear(x, w, b=None):
    return H3Linear.apply(x, w, b)


def _heads(t: torch.Tensor) -> torch.Tensor:
    """[B, S, H, D] -> [B, H, S, D] contiguous (the batched GEMM's operand)."""
    return t.permute(0, 2, 1, 3).contiguous()


class ChunkedAttention(torch.autograd.Function):
    """softmax(scale q k^T [causal]) v with q [B, Sq, H, D], k / v [B, Skv,
    Hkv, D] (H % Hkv == 0); the causal mask aligns the last query with the
    last key (Sq <= Skv), as the inference kernels do.  Grouped-query heads
    are GEMM rows: the g query heads of a KV head stack into one [g * C, D]
    operand per chunk against that head's K / V (no repeated K / V copies;
    dK / dV sum over the group inside the P^T dO / dS^T Q products)."""

    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float):
        B, Sq, H, D = q.shape
        Skv, Hkv = k.shape[1], k.shape[2]
        g = H // Hkv
        ct = torch.float64 if q.dtype == torch.float64 else torch.float32   # fp32 math (fp64 kept for tests)
        qh, kh, vh = _heads(q.to(ct)), _heads(k.to(ct)), _heads(v.to(ct))  # [B, heads, S, D]
        o = torch.empty_like(qh)
        lse = torch.empty(B, H, Sq, device=q.device, dtype=ct)
        k3, v3 = kh.reshape(B * Hkv, Skv, D), vh.reshape(B * Hkv, Skv, D)
        q5, o5 = qh.view(B, Hkv, g, Sq, D), o.view(B, Hkv, g, Sq, D)
        for c0 in range(0, Sq, CHUNK):
            c1 = min(Sq, c0 + CHUNK)
            C = c1 - c0
            s = _mm(q5[:, :, :, c0:c1].reshape(B * Hkv, g * C, D), k3, b_t=True).view(B, H, C, Skv)
            s = s * scale
            if causal:
                s = s.masked_fill(_mask(c0, c1, Sq, Skv, q.device), float("-inf"))
            m = s.amax(-1, keepdim=True)
            p = torch.exp(s - m)
            l_ = p.sum(-1, keepdim=True)
            lse[:, :, c0:c1] = (m + torch.log(l_)).squeeze(-1)
            o5[:, :, :, c0:c1] = _mm((p / l_).reshape(B * Hkv, g * C, Skv), v3).view(B, Hkv, g, C, D)
        ctx.save_for_backward(qh, kh, vh, o, lse)
        ctx.causal, ctx.scale, ctx.g, ctx.dt = causal, scale, g, q.dtype
        return o.permute(0, 2, 1, 3).to(q.dtype)

    @staticmethod
    def backward(ctx, do):
        qh, kh, vh, o, lse = ctx.saved_tensors
        B, H, Sq, D = qh.shape
        Hkv, Skv = kh.shape[1], kh.shape[2]
        g = ctx.g
        doh = _heads(do.to(qh.dtype))
        dq = torch.empty_like(qh)
        dk = torch.zeros_like(kh)
        dv = torch.zeros_like(vh)
        k3, v3 = kh.reshape(B * Hkv, Skv, D), vh.reshape(B * Hkv, Skv, D)
        dk3, dv3 = dk.view(B * Hkv, Skv, D), dv.view(B * Hkv, Skv, D)
        q5, do5, dq5 = qh.view(B, Hkv, g, Sq, D), doh.view(B, Hkv, g, Sq, D), dq.view(B, Hkv, g, Sq, D)
        delta = (doh * o).sum(-1)                                   # rowsum(dO . O)
        for c0 in range(0, Sq, CHUNK):
            c1 = min(Sq, c0 + CHUNK)
            C = c1 - c0
            qc = q5[:, :, :, c0:c1].reshape(B * Hkv, g * C, D)
            doc = do5[:, :, :, c0:c1].reshape(B * Hkv, g * C, D)
            s = _mm(qc, k3, b_t=True).view(B, H, C, Skv) * ctx.scale
            if ctx.causal:
                s = s.masked_fill(_mask(c0, c1, Sq, Skv, qh.device), float("-inf"))
            p = torch.exp(s - lse[:, :, c0:c1, None])               # recomputed from the log-sum-exp
            pf = p.reshape(B * Hkv, g * C, Skv)
            dv3 += _mm(pf, doc, a_t=True)                                      # P^T dO (the group summed)
            dp = _mm(doc, v3, b_t=True).view(B, H, C, Skv)                    # dO V^T
            ds = (p * (dp - delta[:, :, c0:c1, None]) * ctx.scale).reshape(B * Hkv, g * C, Skv)
            dq5[:, :, :, c0:c1] = _mm(ds, k3).view(B, Hkv, g, C, D)           # dS K
            dk3 += _mm(ds, qc, a_t=True)                                       # dS^T Q (the group summed)
        back = lambda t: t.permute(0, 2, 1, 3).to(ctx.dt)   # noqa: E731
        return back(dq), back(dk), back(dv), None, None


def _mask(c0: int, c1: int, sq: int, skv: int, device) -> torch.Tensor:
    """True where query row i (of c0..c1-1) must not see key j: j > i + skv - sq."""
    i = torch.arange(c0, c1, device=device)[:, None] + (skv - sq)
    j = torch.arange(skv, device=device)[None, :]
    return j > i


def attention(q, k, v, causal: bool = False, scale: float | None = None):
    sc = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    return ChunkedAttention.apply(q, k, v, bool(causal), sc)


class CrossEntropy(torch.autograd.Function):
    """Mean cross-entropy of logits x [N, C] against class ids t [N]
    (``ignore_index`` -100, as ``F.cross_entropy``): the loss from the rows'
    log-sum-exp, the gradient ``(exp(x - lse) - onehot(t)) / n_valid`` in one
    elementwise pass and a scatter -- no softmax kernel, no [N, C]
    probability tensor kept between forward and backward."""

    @staticmethod
    def forward(ctx, x, t):
        valid = t != -100
        tc = torch.where(valid, t, torch.zeros_like(t)).long()
        lse = torch.logsumexp(x, -1)
        nll = (lse - x.gather(1, tc[:, None]).squeeze(1)) * valid
        n = valid.sum()
        ctx.save_for_backward(x, tc, lse, valid, n)
        return nll.sum() / n

    @staticmethod
    def backward(ctx, g):
        x, tc, lse, valid, n = ctx.saved_tensors
        d = torch.exp(x - lse[:, None])
        d.scatter_add_(1, tc[:, None], -torch.ones_like(lse)[:, None])
        return d * (valid.to(d.dtype) * (g / n))[:, None], None


def cross_entropy(x, t):
    return CrossEntropy.apply(x, t)


def scores_bytes(b: int, h: int, sq: int, skv: int) -> int:
    """Live score bytes of :class:`ChunkedAttention` (a chunk's s, p, dp, ds)."""
    return 4 * b * h * min(sq, CHUNK) * skv * 4


__all__ = ["H3Linear", "ChunkedAttention", "CrossEntropy", "linear", "attention", "cross_entropy", "scores_bytes",
           "CHUNK"]
