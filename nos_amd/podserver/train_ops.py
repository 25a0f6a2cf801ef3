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


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b on the h3 GEMM for CUDA tensors (batch dims equal or one side 2-D)."""
    if a.is_cuda:
        from ..ops import tenant as T

        return T.matmul(a, b)
    return a @ b


class H3Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        y = _mm(x2, w.t())
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
        dw = _mm(dy2.t(), x2) if ctx.needs_input_grad[1] else None
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
    last key (Sq <= Skv), as the inference kernels do."""

    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float):
        B, Sq, H, D = q.shape
        Skv, Hkv = k.shape[1], k.shape[2]
        g = H // Hkv
        ct = torch.float64 if q.dtype == torch.float64 else torch.float32   # fp32 math (fp64 kept for tests)
        qh = _heads(q.to(ct))
        kh = _heads(k.to(ct)).repeat_interleave(g, dim=1) if g > 1 else _heads(k.to(ct))
        vh = _heads(v.to(ct)).repeat_interleave(g, dim=1) if g > 1 else _heads(v.to(ct))
        o = torch.empty_like(qh)
        lse = torch.empty(B, H, Sq, device=q.device, dtype=ct)
        kt = kh.transpose(-1, -2)
        for c0 in range(0, Sq, CHUNK):
            c1 = min(Sq, c0 + CHUNK)
            s = _mm(qh[:, :, c0:c1].reshape(B * H, c1 - c0, D), kt.reshape(B * H, D, Skv)).view(B, H, c1 - c0, Skv)
            s = s * scale
            if causal:
                s = s.masked_fill(_mask(c0, c1, Sq, Skv, q.device), float("-inf"))
            m = s.amax(-1, keepdim=True)
            p = torch.exp(s - m)
            l_ = p.sum(-1, keepdim=True)
            lse[:, :, c0:c1] = (m + torch.log(l_)).squeeze(-1)
            o[:, :, c0:c1] = _mm((p / l_).reshape(B * H, c1 - c0, Skv), vh.reshape(B * H, Skv, D)).view(
                B, H, c1 - c0, D)
        ctx.save_for_backward(qh, kh, vh, o, lse)
        ctx.causal, ctx.scale, ctx.g, ctx.dt = causal, scale, g, q.dtype
        return o.permute(0, 2, 1, 3).to(q.dtype)

    @staticmethod
    def backward(ctx, do):
        qh, kh, vh, o, lse = ctx.saved_tensors
        B, H, Sq, D = qh.shape
        Skv = kh.shape[2]
        doh = _heads(do.to(qh.dtype))
        dq = torch.empty_like(qh)
        dk = torch.zeros_like(kh)
        dv = torch.zeros_like(vh)
        kt = kh.transpose(-1, -2).reshape(B * H, D, Skv)
        vt = vh.transpose(-1, -2).reshape(B * H, D, Skv)
        delta = (doh * o).sum(-1)                                   # rowsum(dO . O)
        for c0 in range(0, Sq, CHUNK):
            c1 = min(Sq, c0 + CHUNK)
            C = c1 - c0
            qc = qh[:, :, c0:c1].reshape(B * H, C, D)
            doc = doh[:, :, c0:c1].reshape(B * H, C, D)
            s = _mm(qc, kt).view(B, H, C, Skv) * ctx.scale
            if ctx.causal:
                s = s.masked_fill(_mask(c0, c1, Sq, Skv, qh.device), float("-inf"))
            p = torch.exp(s - lse[:, :, c0:c1, None])               # recomputed from the log-sum-exp
            pf = p.reshape(B * H, C, Skv)
            dv += _mm(pf.transpose(-1, -2), doc).view(B, H, Skv, D)
            dp = _mm(doc, vt).view(B, H, C, Skv)
            ds = (p * (dp - delta[:, :, c0:c1, None]) * ctx.scale).reshape(B * H, C, Skv)
            dq[:, :, c0:c1] = _mm(ds, kh.reshape(B * H, Skv, D)).view(B, H, C, D)
            dk += _mm(ds.transpose(-1, -2), qc).view(B, H, Skv, D)
        g = ctx.g
        if g > 1:   # grouped-query: the K / V gradients of a group's heads add up
            dk = dk.view(B, H // g, g, Skv, D).sum(2)
            dv = dv.view(B, H // g, g, Skv, D).sum(2)
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
