"""The numerical argument behind the fp16x3 ("h3") fp32 attention
(csrc/hip/split_f16.h), checked on the CPU:

* on a power-of-two scale putting |x| just under 2^14, two round-to-nearest
  fp16 pieces h + l hold an fp32 x to 22 significant bits (<= 2^-22
  relative in the worst case, ~2^-24 on average: fp32 holds 24), and the
  three piece products ah.bh + ah.bl + al.bh, each exact in fp32, summed in
  fp32 per 16-deep step, are as accurate against fp64 as an fp32 fmaf chain
  -- the chain's own rounding of the running sum dominates both;
* :func:`nos_amd.ops.h3_head_scales` -- the per-head scales the QKV
  projection writes K / V on -- bounds every key and value the LN-folded
  projection can produce, including the input that attains the bound,
  under fp16's 65504."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from nos_amd import ops


def _split_h3(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """The kernels' split of rows of x: scale 2^e per row (max just under
    2^14), hi = f16(x'), lo = f16(x' - hi).  Returns (hi, lo, 2^-e)."""
    mx = x.abs().amax(dim=-1, keepdim=True)
    e = 14 - torch.frexp(mx).exponent
    e = torch.where(mx > 0, e, torch.zeros_like(e)).clamp(-126, 126)
    xs = torch.ldexp(x, e)
    hi = xs.half()
    lo = (xs - hi.float()).half()
    return hi, lo, torch.ldexp(torch.ones_like(mx), -e)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.floats(min_value=float(np.float32(-1e30)), max_value=float(np.float32(1e30)), allow_nan=False, width=32), min_size=2, max_size=64),
       st.integers(min_value=-60, max_value=60))
def test_two_fp16_pieces_hold_an_fp32_row_to_one_rounding(xs, shift):
    x = torch.tensor(xs, dtype=torch.float32) * float(2.0 ** shift)
    x = x[torch.isfinite(x)]
    if x.numel() == 0 or x.abs().max() == 0:
        return
    hi, lo, inv = _split_h3(x[None])
    back = (hi.double() + lo.double()) * inv.double()
    err = (back[0] - x.double()).abs()
    # <= 2^-22 relative, floored at 2^-25 on the scaled axis (fp16 subnormals:
    # <= 2^-38 of the row max)
    bound = torch.maximum(x.double().abs() * 2.0 ** -22, 2.0 ** -25 * inv[0].double())
    assert bool((err <= bound).all()), (err - bound).max()
    normal = x.double().abs() >= x.double().abs().max() * 2.0 ** -10
    assert (err[normal] / x.double().abs()[normal]).mean() <= 2.0 ** -23  # ~2^-24 on average


def _gemm_pieces(a: torch.Tensor, b: torch.Tensor, terms) -> torch.Tensor:
    """sum over 16-deep k steps of the given piece products, each step's
    products exact (fp64) and added to an fp32 accumulator per step."""
    ah, al, ainv = _split_h3(a)
    bh, bl, binv = _split_h3(b)
    pa, pb = (ah.double(), al.double()), (bh.double(), bl.double())
    acc = torch.zeros(a.shape[0], b.shape[0], dtype=torch.float32)
    for k0 in range(0, a.shape[1], 16):
        s = sum(pa[i][:, k0:k0 + 16] @ pb[j][:, k0:k0 + 16].t() for i, j in terms)
        acc = (acc.double() + s).float()
    return acc.double() * ainv.double() * binv.double().t()


@pytest.mark.parametrize("mag", [1e-6, 1.0, 1e4])
def test_three_fp16_products_are_as_accurate_as_an_fp32_chain(mag):
    torch.manual_seed(0)
    a = torch.randn(64, 384) * mag
    b = torch.randn(48, 384) * 0.05
    ref = a.double() @ b.double().t()
    den = a.double().abs() @ b.double().abs().t()
    f32 = torch.zeros(64, 48)
    for k in range(384):  # fmaf chain: one rounding per product
        f32 = (f32.double() + a[:, k:k + 1].double() * b[:, k].double()[None]).float()
    e32 = ((f32.double() - ref).abs() / den).max().item()
    eh3 = ((_gemm_pieces(a, b, [(1, 0), (0, 1), (0, 0)]) - ref).abs() / den).max().item()
    eh2 = ((_gemm_pieces(a, b, [(0, 0)]) - ref).abs() / den).max().item()
    assert eh3 <= 1.5 * e32, (eh3, e32)
    assert eh2 > 20 * e32  # one piece alone (fp16 math) is not fp32


@pytest.mark.parametrize("wscale", [1e-4, 0.05, 30.0])
def test_head_scales_bound_every_key_and_value(wscale):
    torch.manual_seed(1)
    H, K = 3, 128
    w = torch.randn(3 * H * 64, K) * wscale
    b = torch.randn(3 * H * 64) * wscale
    gam, bet = 1 + 0.3 * torch.randn(K), 0.3 * torch.randn(K)
    wg, c1, c2 = ops.fold_layernorm(w, b, gam, bet)
    sc = ops.h3_head_scales(wg, c2, H)
    assert sc.shape == (2, H)
    e = torch.log2(sc)
    assert torch.equal(e, e.round())  # powers of two
    # the input attaining the bound of column j: x^ along the centred wg_j
    hd = H * 64
    xs = []
    for j in range(hd, 3 * hd, 17):
        v = wg[j].double() - wg[j].double().mean()
        xs.append(v * math.sqrt(K) / v.norm())
    xs.append(torch.randn(64, K, dtype=torch.float64))
    x = torch.cat([t.reshape(-1, K) for t in xs])
    y = torch.nn.functional.layer_norm(x, (K,), eps=1e-12) @ wg.double().t() + c2.double()
    kv = y[:, hd:].view(-1, 2, H, 64).abs().amax(dim=(0, 3))  # [K|V, head]
    scaled = kv * sc.double()
    assert bool((scaled < 2 ** 14 * (1 + 1e-6)).all()), scaled
    assert bool((scaled > 2 ** 11).all()), scaled  # tight enough: the aligned input reaches >= 1/8 of it
    assert ops.h3_head_scales(wg, c2, H) is sc  # cached per weight
