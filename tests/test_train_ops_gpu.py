"""Training tenants on the gfx950 kernels (podserver/train_ops.py): the h3
linear and the chunked attention's forward and backward against fp64 torch
autograd on the GPU, and a seq-2048 decoder fine-tune that fits a 10 GB
slice (no S x S score tensor is kept)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from nos_amd.podserver import train_ops  # noqa: E402


def _grads(fn, *xs):
    xs = [x.detach().clone().requires_grad_(True) for x in xs]
    y = fn(*xs)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(7)).to(y.device, y.dtype)
    y.backward(g)
    return y.detach(), [x.grad for x in xs]


def _rel(a, b) -> float:
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


def _ref(q, k, v, causal):
    g = q.shape[2] // k.shape[2]
    k, v = k.repeat_interleave(g, 2), v.repeat_interleave(g, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / q.shape[-1] ** 0.5
    if causal:
        i = torch.arange(q.shape[1], device=q.device)[:, None] + (k.shape[1] - q.shape[1])
        s = s.masked_fill(torch.arange(k.shape[1], device=q.device)[None, :] > i, float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("g, s", [(1, 300), (4, 1100)])
def test_chunked_attention_on_gpu_matches_fp64(causal, g, s):
    torch.manual_seed(0)
    q = torch.randn(1, s, 2 * g, 128, device="cuda")
    k = torch.randn(1, s, 2, 128, device="cuda")
    v = torch.randn(1, s, 2, 128, device="cuda")
    y, gs = _grads(lambda a, b, c: train_ops.attention(a, b, c, causal), q, k, v)
    y64, g64 = _grads(lambda a, b, c: _ref(a, b, c, causal), q.double(), k.double(), v.double())
    y32, g32 = _grads(lambda a, b, c: _ref(a, b, c, causal), q, k, v)
    assert _rel(y, y64) <= max(4 * _rel(y32, y64), 1e-5)
    for a, b, c in zip(gs, g64, g32):
        assert _rel(a, b) <= max(4 * _rel(c, b), 1e-5), (_rel(a, b), _rel(c, b))


def test_h3_linear_on_gpu_matches_fp64():
    torch.manual_seed(1)
    x = torch.randn(4, 333, 1024, device="cuda")
    w = torch.randn(2816, 1024, device="cuda") / 32
    b = torch.randn(2816, device="cuda")
    y, gs = _grads(train_ops.linear, x, w, b)
    y64, g64 = _grads(torch.nn.functional.linear, x.double(), w.double(), b.double())
    y32, g32 = _grads(torch.nn.functional.linear, x, w, b)
    assert _rel(y, y64) <= max(4 * _rel(y32, y64), 1e-5)
    for a, r, c in zip(gs, g64, g32):
        assert _rel(a, r) <= max(4 * _rel(c, r), 1e-5)


def test_seq2048_decoder_fine_tune_fits_a_10gb_slice(tmp_path):
    """The small Llama (1024 hidden, 8 layers, 32000 vocab) fine-tuned at
    sequence 2048 in a 10 GB slice: the static estimate admits it, the
    captured step runs and the loss moves."""
    from nos_amd.models.llama_program import llama_config, llama_model, llama_program
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    prog, w = llama_program(llama_model(llama_config(True), 0), 2048)
    srv = PodServer(tmp_path / "t.sock", device="cuda", lanes=2, memory_gb=64).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=60)
        rep = c.register("ft", prog, w, memory_limit_gb=10,
                         train={"loss": "cross_entropy", "optimizer": "adamw", "lr": 1e-4})
        assert rep["footprint_gb"] < 10
        ids = np.random.default_rng(0).integers(0, 32000, (1, 2049)).astype(np.int32)
        losses = [c.train_step(ids[:, :-1], ids[:, 1:])["loss"] for _ in range(3)]
        assert all(np.isfinite(losses)) and losses[-1] < losses[0]
        c.close()
    finally:
        srv.stop()


@pytest.mark.parametrize("shape", [(1, 37, 45, 29), (6, 128, 100, 64), (3, 513, 64, 200)])
@pytest.mark.parametrize("a_t, b_t", [(False, False), (True, False), (False, True), (True, True)])
def test_mm_transposed_operands_match_fp64(shape, a_t, b_t):
    """ops.tenant.mm: a transposed A or a plain B is split by columns
    (nos_split_cols_h3, zero-padded reduction dim) -- against fp64, within the
    h3 GEMM's fp32-class error; 2-D and batched."""
    from nos_amd.ops import tenant as T

    nb, M, K, N = shape
    g = torch.Generator(device="cuda").manual_seed(M + K + N)
    a = torch.randn(nb, K, M, device="cuda", generator=g) if a_t else torch.randn(nb, M, K, device="cuda", generator=g)
    b = torch.randn(nb, N, K, device="cuda", generator=g) if b_t else torch.randn(nb, K, N, device="cuda", generator=g)
    a[..., 3] *= 1e3                       # per-row / per-column scales matter
    for x, y in ((a, b), (a[0], b[0])):
        got = T.mm(x, y, a_t, b_t)
        A = x.double().transpose(-1, -2) if a_t else x.double()
        B = y.double().transpose(-1, -2) if b_t else y.double()
        ref = A @ B
        err = (got.double() - ref).abs().max() / ref.abs().max()
        assert got.shape == ref.shape and float(err) < 2e-6, (shape, a_t, b_t, float(err))
