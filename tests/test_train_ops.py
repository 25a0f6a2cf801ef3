"""Training tenants' differentiable ops (podserver/train_ops.py) against torch
autograd: the h3-GEMM linear (forward + both backward products) and the
chunked attention (causal, grouped-query, several query chunks, a log-sum-exp
recompute instead of kept S x S scores).  CPU here (the same code on torch
matmuls); the GPU twin runs them on the gfx950 kernels."""
from __future__ import annotations

import pytest
import torch

from nos_amd.podserver import train_ops


def _ref64(q, k, v, causal):
    """softmax(q k^T / sqrt(D)) v in fp64 autograd (grouped-query heads repeated)."""
    g = q.shape[2] // k.shape[2]
    k, v = k.repeat_interleave(g, 2), v.repeat_interleave(g, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / q.shape[-1] ** 0.5
    if causal:
        i = torch.arange(q.shape[1])[:, None] + (k.shape[1] - q.shape[1])
        s = s.masked_fill(torch.arange(k.shape[1])[None, :] > i, float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v)


def _grads(fn, *xs):
    xs = [x.detach().clone().requires_grad_(True) for x in xs]
    y = fn(*xs)
    g = torch.randn_like(y, generator=torch.Generator().manual_seed(7))
    y.backward(g)
    return y.detach(), [x.grad for x in xs]


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("g, sq, skv", [(1, 37, 37), (4, 70, 70), (2, 9, 40)])
def test_chunked_attention_matches_autograd(monkeypatch, causal, g, sq, skv):
    monkeypatch.setattr(train_ops, "CHUNK", 16)   # several chunks, a ragged last one
    torch.manual_seed(0)
    B, hkv, D = 2, 2, 16
    q = torch.randn(B, sq, hkv * g, D, dtype=torch.float64)
    k = torch.randn(B, skv, hkv, D, dtype=torch.float64)
    v = torch.randn(B, skv, hkv, D, dtype=torch.float64)
    y, gs = _grads(lambda a, b, c: train_ops.attention(a, b, c, causal), q, k, v)
    y0, g0 = _grads(lambda a, b, c: _ref64(a, b, c, causal), q, k, v)
    torch.testing.assert_close(y, y0, rtol=1e-10, atol=1e-10)
    for a, b in zip(gs, g0):
        torch.testing.assert_close(a, b, rtol=1e-9, atol=1e-9)


def test_h3_linear_matches_autograd():
    torch.manual_seed(1)
    x = torch.randn(3, 5, 48, dtype=torch.float64)
    w = torch.randn(20, 48, dtype=torch.float64)
    b = torch.randn(20, dtype=torch.float64)
    y, gs = _grads(train_ops.linear, x, w, b)
    y0, g0 = _grads(torch.nn.functional.linear, x, w, b)
    torch.testing.assert_close(y, y0)
    for a, c in zip(gs, g0):
        torch.testing.assert_close(a, c)


def test_the_estimate_keeps_no_full_score_tensor():
    """A seq-4096 decoder's training estimate grows with S (chunked scores),
    not S^2 per layer."""
    from nos_amd.models.llama_program import llama_config, llama_model, llama_program
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.training import parse_train_spec, train_bytes_estimate

    m = llama_model(llama_config(False), 0)
    est = {}
    for s in (1024, 4096):
        p = PG.parse(*llama_program(m, s))
        est[s] = train_bytes_estimate(p, parse_train_spec({"loss": "cross_entropy", "optimizer": "adamw"}, p))
    assert est[4096] < 8 * est[1024]     # the S x S form would be ~16x


def test_cross_entropy_matches_torch_with_ignored_rows():
    import torch.nn.functional as F

    from nos_amd.podserver.train_ops import cross_entropy

    torch.manual_seed(0)
    x = (torch.randn(37, 101, dtype=torch.float64) * 4).requires_grad_()
    t = torch.randint(0, 101, (37,))
    t[[3, 9]] = -100
    x2 = x.detach().clone().requires_grad_()
    loss, ref = cross_entropy(x, t), F.cross_entropy(x2, t)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-12, atol=1e-12)
