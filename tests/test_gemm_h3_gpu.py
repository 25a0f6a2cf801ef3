"""The fp16x3 ("h3") fp32 GEMM (csrc/hip/gemm_f32h.hip): activation rows
split by a pre-pass on per-row power-of-two scales (LayerNorm applied in
it), weights split once per tensor, three fp16 MFMAs per product.  Checked
against fp64 next to the exact-f32 MFMA GEMM on the same inputs (error
within 1.5x, max and mean), every epilogue and tail shape, rows spanning
1e-30 .. 1e30 in one matrix, and bit-identity of the two wave layouts."""
from __future__ import annotations

import pytest
import torch

from nos_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _with_math(m, fn):
    ops.set_f32_math(m)
    try:
        y = fn()
        torch.cuda.synchronize()
        return y
    finally:
        ops.set_f32_math("exact")


@pytest.mark.parametrize("M,N,K", [(3401, 1152, 384), (3401, 384, 1536), (512, 768, 3072)])
def test_h3_linear_is_as_accurate_as_exact_f32(M, N, K):
    torch.manual_seed(5)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    ref = x.cpu().double() @ w.cpu().double().t()
    errs = {}
    for m in ("exact", "x6", "h3"):
        e = (_with_math(m, lambda: ops.linear(x, w)).cpu().double() - ref).abs()
        errs[m] = (e.max().item(), e.mean().item())
    print("linear fp32 error vs fp64 (max, mean):", errs)
    assert errs["h3"][0] <= 1.5 * errs["exact"][0] and errs["h3"][1] <= 1.5 * errs["exact"][1], errs


@pytest.mark.parametrize("act", [None, "gelu", "relu"])
@pytest.mark.parametrize("resid", [False, True])
@pytest.mark.parametrize("M,N,K", [(77, 100, 64), (3401, 384, 384), (1, 1536, 384), (300, 130, 96)])
def test_h3_linear_epilogues_and_tails(M, N, K, act, resid):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV) * 3
    w = torch.randn(N, K, device=DEV) * 0.1
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV) if resid else None
    y = _with_math("h3", lambda: ops.linear(x, w, b, act=act, residual=r))
    ref = x.cpu().double() @ w.cpu().double().t() + b.cpu().double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    elif act == "relu":
        ref = torch.relu(ref)
    if resid:
        ref = ref + r.cpu().double()
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, ref.abs().max().item()), err


def test_h3_rows_of_any_magnitude():
    """Per-row scales: rows from 1e-30 to 1e30 (and a zero row) in one
    matrix, each within fp32 accuracy of its own fp64 result."""
    torch.manual_seed(9)
    M, N, K = 130, 96, 256
    mags = torch.logspace(-30, 30, M - 1, dtype=torch.float64)
    x = torch.randn(M, K, dtype=torch.float64)
    x[:-1] *= mags[:, None]
    x[-1] = 0
    w = torch.randn(N, K, dtype=torch.float64) * 0.05
    ref = x @ w.t()
    den = x.abs() @ w.abs().t()
    y = _with_math("h3", lambda: ops.linear(x.float().to(DEV), w.float().to(DEV))).cpu().double()
    rel = ((y - ref).abs() / den.clamp_min(1e-300))[:-1]
    assert rel.max().item() < 1e-6, rel.max().item()
    assert torch.count_nonzero(y[-1]) == 0


@pytest.mark.parametrize("act", [None, "gelu"])
@pytest.mark.parametrize("M,N,K", [(3401, 1152, 384), (77, 1536, 384), (5, 64, 1024)])
def test_h3_linear_layernorm(M, N, K, act):
    """LayerNorm in the split pre-pass: against the fp64 LN -> linear, and
    within 1.5x of the exact-f32 fused kernel's error (plus a floor)."""
    torch.manual_seed(N + K)
    x = torch.randn(M, K, device=DEV) * 4 + 1.5
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    g, be = 1 + 0.2 * torch.randn(K, device=DEV), 0.2 * torch.randn(K, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
    xd = torch.nn.functional.layer_norm(x.cpu().double(), (K,), g.cpu().double(), be.cpu().double(), 1e-12)
    ref = xd @ w.cpu().double().t() + b.cpu().double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    errs = {}
    for m in ("exact", "h3"):
        e = (_with_math(m, lambda: ops.linear_ln(x, wg, c1, c2, act=act)).cpu().double() - ref).abs()
        errs[m] = e.max().item()
    print("linear_ln error vs fp64:", errs)
    assert errs["h3"] <= 1.5 * errs["exact"] + 1e-6 * max(1.0, ref.abs().max().item()), errs


def test_h3_wave_layouts_are_bit_identical():
    torch.manual_seed(2)
    x = torch.randn(1000, 384, device=DEV)
    w = torch.randn(384, 384, device=DEV) * 0.05
    b = torch.randn(384, device=DEV)
    outs = []
    lays = ("4x1", "2x2", "256x128", "4x1r3", "4x1k16", "2x2k16", "2x2r3", "2x2n64")
    for lay in lays:
        ops.set_gemm_f32h3_layout(lay)
        try:
            outs.append(_with_math("h3", lambda: ops.linear(x, w, b, act="gelu", residual=x)))
        finally:
            ops.set_gemm_f32h3_layout("2x2")
    for lay, o in zip(lays[1:], outs[1:]):
        assert torch.equal(outs[0], o), lay


@pytest.mark.parametrize("B,S,H", [(1, 3401, 6), (2, 77, 3)])
def test_h3_qkv_projection_with_h3_attention(B, S, H):
    """The whole h3 path (LN pre-pass, h3 QKV GEMM writing the fp16 K / V
    planes, h3 attention) against fp64, within the exact path's error."""
    torch.manual_seed(S)
    K = 384
    x = torch.randn(B, S, K, device=DEV) * 2 + 0.5
    w = torch.randn(3 * H * 64, K, device=DEV) * 0.05
    b = torch.randn(3 * H * 64, device=DEV) * 0.2
    g, be = 1 + 0.2 * torch.randn(K, device=DEV), 0.2 * torch.randn(K, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
    xd = torch.nn.functional.layer_norm(x.cpu().double(), (K,), g.cpu().double(), be.cpu().double(), 1e-12)
    qkv = xd @ w.cpu().double().t() + b.cpu().double()
    q, k, v = qkv.view(B, S, 3, H, 64).unbind(2)
    p = torch.softmax((q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / 8.0, dim=-1)
    ref = (p @ v.transpose(1, 2)).transpose(1, 2).reshape(B, S, H * 64)
    errs = {}
    for name, m, var in (("exact", "exact", "w4k32o4"), ("h3", "h3", "h3n")):
        ops.set_f32_math(m)
        ops.set_attention_f32_variant(var)
        try:
            if ops.ln_qkv_fusable(x):
                y = ops.ln_qkv_attention(x, wg, c1, c2, H)
            else:
                y = ops.attention_qkv(ops.linear_ln(x, wg, c1, c2), H)
            torch.cuda.synchronize()
        finally:
            ops.set_f32_math("exact")
            ops.set_attention_f32_variant("auto")
        e = (y.cpu().double() - ref).abs()
        errs[name] = (e.max().item(), e.mean().item())
    print("h3 path error vs fp64 (max, mean):", errs)
    assert errs["h3"][0] <= 1.5 * errs["exact"][0] + 1e-7 and errs["h3"][1] <= 1.5 * errs["exact"][1], errs


def test_h3_mlp_plane_handoff_matches_fp64():
    """fc1 (LN-folded, GELU) writing fc2's A planes on the static scale from
    its weights, fc2 reading them: the fc1 -> fc2 chain against fp64, within
    the exact-f32 chain's error."""
    torch.manual_seed(4)
    M, K, F = 3401, 384, 1536
    x = torch.randn(M, K, device=DEV) * 2 + 0.3
    w1 = torch.randn(F, K, device=DEV) * 0.05
    b1 = torch.randn(F, device=DEV) * 0.1
    w2 = torch.randn(K, F, device=DEV) * 0.03
    b2 = torch.randn(K, device=DEV) * 0.1
    g, be = 1 + 0.2 * torch.randn(K, device=DEV), 0.2 * torch.randn(K, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w1, b1, g, be)
    xd = torch.nn.functional.layer_norm(x.cpu().double(), (K,), g.cpu().double(), be.cpu().double(), 1e-12)
    hid = torch.nn.functional.gelu(xd @ w1.cpu().double().t() + b1.cpu().double())
    ref = hid @ w2.cpu().double().t() + b2.cpu().double() + x.cpu().double()

    def exact():
        m = ops.linear_ln(x, wg, c1, c2, act="gelu")
        return ops.linear(m, w2, b2, residual=x)

    def handoff():
        m = ops.linear_ln_to_planes(x, wg, c1, c2, act="gelu")
        assert isinstance(m, ops.H3Planes) and m.rinv is None and m.shape == (M, F)
        return ops.linear_planes(m, w2, b2, residual=x)

    errs = {}
    for name, m, fn in (("exact", "exact", exact), ("h3", "h3", handoff)):
        e = (_with_math(m, fn).cpu().double() - ref).abs()
        errs[name] = (e.max().item(), e.mean().item())
    print("fc1 -> fc2 error vs fp64 (max, mean):", errs)
    assert errs["h3"][0] <= 1.5 * errs["exact"][0] and errs["h3"][1] <= 1.5 * errs["exact"][1], errs


@pytest.mark.parametrize("variant", ["h3n", "h3"])
def test_h3_yolos_with_plane_handoffs_matches_the_fp32_reference(variant):
    """YOLOS-small under the default h3 kernels, attention -> proj and fc1 ->
    fc2 handing their activations over as planes: logits and boxes within
    the exact-fp32 tolerance of the PyTorch fp32 model, and the compiled
    program of the same weights marks 24 hand-offs and agrees."""
    from nos_amd.models.yolos import YolosConfig, YolosDetector, make_demo_input

    cfg = YolosConfig.small()
    m = YolosDetector(cfg, backend="torch")
    m.reset_parameters(0)
    m = m.to(DEV).eval()
    x = make_demo_input(cfg, device=DEV, dtype=torch.float32, seed=0)
    with torch.no_grad():
        ref = m(x)
        m.backend = "native"
        ops.set_f32_math("h3")
        ops.set_attention_f32_variant(variant)
        try:
            got = m(x)
            torch.cuda.synchronize()
        finally:
            ops.set_f32_math("exact")
            ops.set_attention_f32_variant("auto")
    rng = (ref[0].max() - ref[0].min()).item()
    assert (got[0] - ref[0]).abs().max().item() <= 1e-4 * rng
    assert (got[1] - ref[1]).abs().max().item() <= 1e-4
