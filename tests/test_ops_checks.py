"""Host-side argument checks of the native GEMM dispatchers: the
kernels write M x N elements through raw pointers, so a wrong ``out`` must be
refused before launch.  Pure tensor-metadata checks: they run on the CPU."""
from __future__ import annotations

import pytest
import torch

from nos_amd.ops import _gemm_io


def _x(M=6, K=32, dt=torch.float32):
    return torch.zeros(M, K, dtype=dt)


def test_gemm_io_accepts_and_views():
    x, w = _x(), torch.zeros(8, 32)
    o2, r2 = _gemm_io(x, w, None, torch.zeros(6, 8), 6, 8, 32)
    assert o2.shape == (6, 8) and r2.shape == (6, 8)
    out = torch.empty(2, 3, 8)
    o2, _ = _gemm_io(x, w, out, None, 6, 8, 32)
    assert o2.data_ptr() == out.data_ptr()


@pytest.mark.parametrize("bad, match", [
    (lambda: dict(out=torch.empty(6, 8, dtype=torch.bfloat16)), "out must be"),
    (lambda: dict(out=torch.empty(5, 8)), "must hold"),
    (lambda: dict(out=torch.empty(8, 6).t()), "viewable|unit inner"),
    (lambda: dict(weight=torch.zeros(8, 64)), "weight must be"),
    (lambda: dict(residual=torch.zeros(6, 4)), "residual must be"),
    (lambda: dict(residual=torch.zeros(6, 8, dtype=torch.float64)), "residual must be"),
])
def test_gemm_io_refuses(bad, match):
    kw = dict(weight=torch.zeros(8, 32), out=None, residual=None)
    kw.update(bad())
    with pytest.raises(ValueError, match=match):
        _gemm_io(_x(), kw["weight"], kw["out"], kw["residual"], 6, 8, 32)
