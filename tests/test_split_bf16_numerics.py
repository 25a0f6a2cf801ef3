"""The numerical argument behind the bf16x6 fp32 kernels (csrc/hip/split_bf16.h),
checked on the CPU:

* the three-piece split x = x0 + x1 + x2 (bf16 each) is exact for fp32 values
  in the normal range (property test);
* a product summed from the six piece products of order >= 2^-16, each exact
  in fp32 and accumulated in fp32 per 16-deep step (what
  v_mfma_f32_32x32x16_bf16 does), is as accurate against fp64 as the exact-f32
  MFMA's one-rounding-per-product fmaf chain; dropping to three products (a
  "bf16x3" shortcut) is an order of magnitude worse and is NOT what the
  kernels do.
The GPU tests (tests/test_kernels_gpu.py) check the kernels themselves."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from nos_amd import ops

X6 = [(0, 0), (0, 1), (1, 0), (0, 2), (1, 1), (2, 0)]
X3 = [(0, 0), (0, 1), (1, 0)]


@settings(max_examples=200, deadline=None)
@given(st.lists(st.floats(min_value=float(np.float32(-3.3e38)), max_value=float(np.float32(3.3e38)),
                          allow_nan=False, width=32), min_size=1, max_size=64))
def test_three_bf16_pieces_reconstruct_every_normal_fp32_exactly(xs):
    x = torch.tensor(xs, dtype=torch.float32)
    # normal range with room for the pieces (the third is ~2^-16 of x) and
    # below bf16's rounding-to-infinity threshold
    x = torch.where(x.abs() < 1e-30, torch.ones_like(x), x)
    p = ops.split_bf16x3(x)
    assert p.dtype == torch.bfloat16 and p.shape == (3, *x.shape)
    # summed in fp64 the pieces give x exactly, and in fp32 too (each partial sum is exact)
    assert torch.equal(p.double().sum(0), x.double())
    assert torch.equal(p[0].float() + p[1].float() + p[2].float(), x)


def _mfma_emulated(a: torch.Tensor, b: torch.Tensor, terms) -> torch.Tensor:
    """a [M,K] @ b [K,N] as the kernels compute it: exact piece products, one
    fp32 rounding per 16-deep MFMA step and term."""
    A, B = ops.split_bf16x3(a), ops.split_bf16x3(b)
    acc = torch.zeros(a.shape[0], b.shape[1], dtype=torch.float32)
    for k0 in range(0, a.shape[1], 16):
        for i, j in terms:
            p = A[i][:, k0:k0 + 16].double() @ B[j][k0:k0 + 16].double()
            acc = (acc.double() + p).float()
    return acc


def _fmaf_chain(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """The exact-f32 MFMA's numerics: one fp32 rounding per product."""
    acc = torch.zeros(a.shape[0], b.shape[1], dtype=torch.float32)
    for k in range(a.shape[1]):
        acc = (acc.double() + a[:, k:k + 1].double() * b[k:k + 1].double()).float()
    return acc


@pytest.mark.parametrize("K", [64, 384])
def test_six_piece_products_are_as_accurate_as_the_exact_f32_mfma(K):
    g = torch.Generator().manual_seed(K)
    a = torch.randn(48, K, generator=g)
    b = torch.randn(K, 40, generator=g)
    ref = a.double() @ b.double()
    scale = a.abs().double() @ b.abs().double()

    def rel(y):
        e = (y.double() - ref).abs() / scale
        return e.max().item(), e.mean().item()

    x6, exact, x3 = rel(_mfma_emulated(a, b, X6)), rel(_fmaf_chain(a, b)), rel(_mfma_emulated(a, b, X3))
    assert x6[0] <= 1.25 * exact[0] and x6[1] <= 1.25 * exact[1], (x6, exact)
    assert x3[1] > 5 * exact[1], (x3, exact)  # the reduced-precision shortcut the kernels avoid
    assert np.isfinite(x6[0])
