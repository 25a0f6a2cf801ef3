"""gfx950 kernels of general tenant programs (nos_amd/ops/tenant.py:
csrc/hip/tenant_ops.hip, attention_h3g.hip, the batched h3 GEMM) against
fp64 references of the same op.

The h3 kernels are fp32-class (two fp16 pieces per operand, three products,
fp32 accumulation): their error against fp64 is checked to stay within a
small multiple of torch's own fp32 result's error (TF32 off), like
tests/test_gemm_h3_gpu.py does for the YOLOS kernels."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from nos_amd.ops import tenant as T  # noqa: E402


@pytest.fixture(autouse=True)
def _no_tf32():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    yield
    T.set_attention_h3g_kvsplit(0)


def _err(got: torch.Tensor, ref64: torch.Tensor) -> float:
    return float((got.double() - ref64).abs().max() / ref64.abs().max().clamp_min(1e-30))


def _close_to_fp64(got, ref64, fp32_got, floor=5e-6, mult=4.0):
    e, e32 = _err(got, ref64), _err(fp32_got, ref64)
    assert e <= max(mult * e32, floor), f"h3 err {e:.3g} vs torch fp32 err {e32:.3g}"
    return e, e32


@pytest.mark.parametrize("cfg", [
    dict(n=2, c=3, h=32, w=30, oc=64, k=7, s=2, p=3, d=1),      # ResNet stem (K = 147 -> 160)
    dict(n=2, c=64, h=28, w=28, oc=64, k=3, s=1, p=1, d=1),
    dict(n=1, c=64, h=28, w=28, oc=128, k=3, s=2, p=1, d=1),
    dict(n=3, c=128, h=14, w=14, oc=256, k=1, s=1, p=0, d=1),   # 1x1: a transpose GEMM
    dict(n=1, c=32, h=17, w=19, oc=48, k=3, s=1, p=2, d=2),     # dilation, odd sizes
    dict(n=2, c=16, h=9, w=9, oc=24, k=5, s=1, p=2, d=1),       # runtime kernel size
])
@pytest.mark.parametrize("epi", ["plain", "bias_relu_resid", "bias_resid_relu"])
def test_conv2d_h3_matches_fp64(cfg, epi):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(cfg["n"], cfg["c"], cfg["h"], cfg["w"], device="cuda", generator=g)
    w = torch.randn(cfg["oc"], cfg["c"], cfg["k"], cfg["k"], device="cuda", generator=g) / math.sqrt(cfg["c"] * cfg["k"] ** 2)
    st, pd, dl = (cfg["s"],) * 2, (cfg["p"],) * 2, (cfg["d"],) * 2
    b = torch.randn(cfg["oc"], device="cuda", generator=g) if epi != "plain" else None
    ref64 = F.conv2d(x.double(), w.double(), None if b is None else b.double(), st, pd, dl)
    r = None
    act = None
    first = epi == "bias_resid_relu"
    if epi != "plain":
        act = "relu"
        r = torch.randn(ref64.shape, device="cuda", generator=g)
        ref64 = F.relu(ref64 + r.double()) if first else F.relu(ref64) + r.double()
    got = T.conv2d(x, w, b, st, pd, dl, act=act, residual=r, residual_first=first)
    f32 = F.conv2d(x, w, b, st, pd, dl)
    if epi != "plain":
        f32 = F.relu(f32 + r) if first else F.relu(f32) + r
    assert got.shape == ref64.shape
    _close_to_fp64(got, ref64, f32)


@pytest.mark.parametrize("n,c,oc,k,s,groups", [(1, 32, 32, 3, 1, 32), (2, 24, 48, 3, 2, 4), (2, 64, 64, 5, 1, 64),
                                              (1, 12, 36, 1, 1, 3)])
def test_grouped_conv2d_h3_matches_fp64(n, c, oc, k, s, groups):
    """Grouped / depthwise convolutions: one batched h3 GEMM per image over
    the groups, bias per group, residual before the ReLU."""
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, c, 19, 23, device="cuda", generator=g)
    w = torch.randn(oc, c // groups, k, k, device="cuda", generator=g) / math.sqrt(c // groups * k * k)
    b = torch.randn(oc, device="cuda", generator=g)
    pd = (k // 2, k // 2)
    ref = F.conv2d(x.double(), w.double(), b.double(), (s, s), pd, 1, groups)
    r = torch.randn(ref.shape, device="cuda", generator=g)
    ref64 = F.relu(ref + r.double())
    got = T.conv2d(x, w, b, (s, s), pd, (1, 1), act="relu", residual=r, residual_first=True, groups=groups)
    f32 = F.relu(F.conv2d(x, w, b, (s, s), pd, 1, groups) + r)
    assert got.shape == ref64.shape
    _close_to_fp64(got, ref64, f32)


@pytest.mark.parametrize("shapes", [((4, 100, 96), (4, 96, 70)), ((2, 3, 33, 64), (2, 3, 64, 40)),
                                    ((5, 64, 128), (128, 256)), ((300, 50), (3, 50, 64))])
def test_matmul_h3_matches_fp64(shapes):
    g = torch.Generator(device="cuda").manual_seed(2)
    a = torch.randn(shapes[0], device="cuda", generator=g)
    b = torch.randn(shapes[1], device="cuda", generator=g)
    ref64 = a.double() @ b.double()
    got = T.matmul(a, b)
    assert got.shape == ref64.shape
    _close_to_fp64(got, ref64, a @ b)


def _rope_tables(S, D, base=10000.0):
    inv = 1.0 / (base ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    f = torch.outer(torch.arange(S, dtype=torch.float64), inv)
    emb = torch.cat([f, f], dim=-1)
    return emb.cos().float().cuda().contiguous(), emb.sin().float().cuda().contiguous()


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 300, 8, 8), (2, 77, 4, 2), (1, 1030, 4, 1), (3, 1, 4, 4)])
@pytest.mark.parametrize("rope", [False, True])
def test_sdpa_h3_matches_fp64(D, causal, shape, rope):
    B, S, H, Hkv = shape
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(B, S, H, D, device="cuda", generator=g)
    k = torch.randn(B, S, Hkv, D, device="cuda", generator=g) * 2
    v = torch.randn(B, S, Hkv, D, device="cuda", generator=g)
    tabs = _rope_tables(S, D) if rope else None
    ref64 = T.sdpa_ref(q.double(), k.double(), v.double(), causal, None,
                       (tabs[0].double(), tabs[1].double()) if rope else None)
    f32 = T.sdpa_ref(q, k, v, causal, None, tabs)
    got = T.sdpa(q, k, v, causal=causal, rope=tabs)
    assert got.shape == (B, S, H, D) and torch.isfinite(got).all()
    _close_to_fp64(got, ref64, f32)


@pytest.mark.parametrize("nsplit", [1, 2, 3, 4])
def test_sdpa_key_splits_agree(nsplit):
    """Key splits (merged partials) give the same attention, causal rows
    whose split range is fully masked included."""
    g = torch.Generator(device="cuda").manual_seed(4)
    q = torch.randn(1, 700, 2, 128, device="cuda", generator=g)
    k = torch.randn(1, 700, 2, 128, device="cuda", generator=g)
    v = torch.randn(1, 700, 2, 128, device="cuda", generator=g)
    ref64 = T.sdpa_ref(q.double(), k.double(), v.double(), True)
    T.set_attention_h3g_kvsplit(nsplit)
    got = T.sdpa(q, k, v, causal=True)
    _close_to_fp64(got, ref64, T.sdpa_ref(q, k, v, True))


def test_sdpa_reads_strided_slices_of_a_fused_projection():
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn(2, 130, 3, 4, 64, device="cuda", generator=g)
    q, k, v = qkv.unbind(2)
    assert q.stride(1) == 3 * 4 * 64
    got = T.sdpa(q, k, v)
    ref64 = T.sdpa_ref(q.double(), k.double(), v.double())
    _close_to_fp64(got, ref64, T.sdpa_ref(q, k, v))


def test_linear_rms_matches_fp64():
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.randn(3, 70, 256, device="cuda", generator=g) * 5
    gam = 1 + 0.1 * torch.randn(256, device="cuda", generator=g)
    w = torch.randn(512, 256, device="cuda", generator=g) / 16
    wg = (w * gam[None, :]).contiguous()
    ref64 = T.linear_rms_ref(x.double(), wg.double(), eps=1e-6)
    got = T.linear_rms(x, wg, eps=1e-6)
    _close_to_fp64(got, ref64, T.linear_rms_ref(x, wg, eps=1e-6))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_row_kernels(dt):
    g = torch.Generator(device="cuda").manual_seed(7)
    x = (torch.randn(5, 33, 200, device="cuda", generator=g) * 3).to(dt)
    w = (1 + 0.1 * torch.randn(200, device="cuda", generator=g)).to(dt)
    tol = 1e-6 if dt == torch.float32 else 1e-2
    assert _err(T.rmsnorm(x, w, 1e-5), T.rmsnorm_ref(x.double(), w.double(), 1e-5)) < tol * 4
    assert _err(T.softmax(x), torch.softmax(x.double(), -1)) < tol * 4
    xs = (torch.randn(2, 9, 3, 64, device="cuda", generator=g)).to(dt)
    c, s = _rope_tables(9, 64)
    assert _err(T.rotary(xs, c, s), T.rope_ref(xs.double(), c.double(), s.double())) < tol * 4
    table = torch.randn(1000, 128, device="cuda", generator=g).to(dt)
    ids = torch.tensor([[0, 5, 999, 5], [1, 2, 3, 1000]], device="cuda")  # 1000: out of range -> zeros
    e = T.embedding(ids, table)
    assert torch.equal(e[0], table[[0, 5, 999, 5]]) and torch.equal(e[1, :3], table[[1, 2, 3]])
    assert not e[1, 3].any()


@pytest.mark.parametrize("n,hw", [(1, (80, 107)), (2, (64, 96))])
def test_patches_read_a_cropped_image_in_place(n, hw):
    """ViT patch rows straight from a non-contiguous crop of an fp32 image:
    the bf16 rows are bit-identical to torch's cast of the same views, the h3
    planes reconstruct the fp32 rows exactly (hi + lo carry 22 bits, the
    inputs are fp16-representable up to the row scale)."""
    from nos_amd import ops

    g = torch.Generator(device="cuda").manual_seed(5)
    img = torch.randn((n, 3, *hw), device="cuda", generator=g)
    p = 16
    hp, wp = hw[0] // p, hw[1] // p
    want = img[:, :, :hp * p, :wp * p].reshape(n, 3, hp, p, wp, p).permute(0, 2, 4, 1, 3, 5).reshape(n, hp * wp, -1)
    got = T.patches(img, p, p, torch.bfloat16)
    assert got.dtype == torch.bfloat16 and got.shape == want.shape
    assert torch.equal(got, want.to(torch.bfloat16))
    prev = ops.f32_math()
    ops.set_f32_math("h3")
    try:
        pl = T.patches(img, p, p)
    finally:
        ops.set_f32_math(prev)
    assert isinstance(pl, ops.H3Planes)
    rows = (pl.planes[0].float() + pl.planes[1].float()) * pl.rinv[:, None]
    err = (rows.view_as(want) - want).abs().max() / want.abs().max()
    assert float(err) < 1e-6
    torch.cuda.synchronize()


@pytest.mark.parametrize("op", ["relu", "sigmoid", "silu", "gelu", "tanh", "exp", "neg"])
@pytest.mark.parametrize("dts", [(torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16),
                                 (torch.float32, torch.float32)])
def test_cast_unary_matches_fp32_math(op, dts):
    """One-pass activation with independent input / output dtypes against
    torch's fp32 evaluation of the same input, rounded once."""
    src, dst = dts
    x = (torch.randn(3, 1001, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2)) * 3).to(src)
    got = T.unary(x, op, dst)
    ref = T.unary(x.cpu(), op, torch.float32).to(torch.float64)
    assert got.dtype == dst and got.shape == x.shape
    tol = 2 ** -7 if dst == torch.bfloat16 else 2e-6
    err = (got.double().cpu() - ref).abs() / ref.abs().clamp_min(1.0)
    assert float(err.max()) <= tol


def test_unary_reads_row_strided_slices_and_host_copies_them():
    """A column slice of a merged GEMM's output: ``unary`` reads its rows in
    place (nos_unary_rows), the server's host copy takes the covering rows."""
    from nos_amd.podserver.server import _host_array

    base = torch.randn(100, 96, device="cuda")
    for sl in (base[:, 92:], base[:, :92], base[5:50, 10:20]):
        for op, f in (("sigmoid", torch.sigmoid), ("relu", torch.relu)):
            got = T.unary(sl, op, torch.float32)
            assert got.is_contiguous() and torch.allclose(got, f(sl), rtol=1e-6, atol=1e-7)
        assert np.array_equal(_host_array(sl), sl.cpu().numpy())
    assert torch.equal(T.unary(base[:, :92].bfloat16(), "relu", torch.bfloat16), torch.relu(base[:, :92].bfloat16()))
