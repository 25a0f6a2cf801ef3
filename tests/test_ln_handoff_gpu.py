"""The LayerNorm hand-off between a pre-LN residual GEMM and the LN-GEMM
after it (no ``nos_split_rows_h3`` launch between them):
the residual GEMM writes its output's row statistics in its epilogue
(``nos_gemm_f32h3_stats``) and the LN-GEMM normalises and splits its fp32
input inside its own A load (``nos_gemm_f32h3_lna``).  Statistics against
fp64, the LN-GEMM against the split-pass path and an fp64 LayerNorm + GEMM,
every epilogue the consumers use (fp32 C, the attention's K / V planes, the
next GEMM's planes), and a YOLOS program with and without the hand-off."""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from nos_amd import ops  # noqa: E402


@pytest.fixture(autouse=True, params=[128, 64], ids=["bn128", "bn64"])
def _h3(request):
    """Every test on both tile widths of the hand-off GEMMs (ops.set_gemm_f32h3_hot_bn)."""
    torch.backends.cuda.matmul.allow_tf32 = False
    prev, prev_h, prev_bn = ops.f32_math(), ops.ln_handoff_active(), ops.stats_pw()
    ops.set_f32_math("h3")
    ops.set_gemm_f32h3_hot_bn(request.param)
    yield
    ops.set_f32_math(prev)
    ops.set_ln_handoff(prev_h)
    ops.set_gemm_f32h3_hot_bn(prev_bn)


def _parts(y64: torch.Tensor, pw: int) -> torch.Tensor:
    """(mean, M2) per part of pw columns, fp64."""
    out = []
    for p0 in range(0, y64.shape[1], pw):
        c = y64[:, p0:p0 + pw]
        m = c.mean(1)
        out.append(torch.stack([m, ((c - m[:, None]) ** 2).sum(1)], 1))
    return torch.stack(out, 1)


@pytest.mark.parametrize("ring, bn", [(2, 128), (3, 128), (2, 64)])
@pytest.mark.parametrize("M,N,K", [(3401, 384, 384), (3401, 384, 1536), (100, 768, 384), (257, 132, 64)])
def test_residual_gemm_writes_its_row_statistics(M, N, K, ring, bn):
    """Also on the 3-deep LDS ring (ops.set_gemm_f32h3_hot_ring) and on 128 x 64
    tiles (ops.set_gemm_f32h3_hot_bn: statistics parts of 64 columns): C
    bit-identical to the default."""
    prev = ops.stats_pw()
    ops.set_gemm_f32h3_hot_ring(ring)
    ops.set_gemm_f32h3_hot_bn(bn)
    try:
        y = _stats_case(M, N, K)
        ops.set_gemm_f32h3_hot_ring(2)
        ops.set_gemm_f32h3_hot_bn(128)
        assert torch.equal(y, _stats_case(M, N, K))
    finally:
        ops.set_gemm_f32h3_hot_ring(2)
        ops.set_gemm_f32h3_hot_bn(prev)


def _stats_case(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g) * 3 + 2
    ap, rinv = ops._split_rows_h3(x, ln=False)
    a = ops.H3Planes(ap, rinv, 0.0, (M, K))
    y_ref = ops.linear_planes(a, w, b, residual=r)
    y, st = ops.linear_planes(a, w, b, residual=r, row_stats=True)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)  # the statistics epilogue leaves C alone
    pw = ops.stats_pw()
    assert st.pw == pw and st.stats.shape == (M, math.ceil(N / pw), 2)
    ref = _parts(y.double(), pw)
    got = st.stats.double()
    scale = y.double().abs().amax(1, keepdim=True)
    assert ((got[..., 0] - ref[..., 0]).abs() <= 4e-6 * scale).all()
    assert ((got[..., 1] - ref[..., 1]).abs() <= 1e-5 * ref[..., 1] + 1e-30).all()
    return y


def _ln64(x, wg, c2, eps):
    x = x.double()
    xh = (x - x.mean(-1, keepdim=True)) / torch.sqrt(x.var(-1, unbiased=False, keepdim=True) + eps)
    return xh @ wg.double().t() + c2.double()


@pytest.mark.parametrize("M,K,N,offset", [(3401, 384, 1152, 0.0), (3401, 384, 1536, 5.0), (77, 768, 256, -3.0),
                                          (130, 1536, 384, 0.0)])
def test_ln_in_the_a_load_matches_the_split_pass(M, K, N, offset):
    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g) * 2 + offset
    wg = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    c2 = torch.randn(N, device="cuda", generator=g)
    ops.set_ln_handoff(False)
    y_split = ops.linear_ln(x, wg, wg.sum(1), c2, eps=1e-6)
    ops.set_ln_handoff(True)
    y_lna = ops.linear_ln(x, wg, wg.sum(1), c2, eps=1e-6)  # statistics from nos_row_stats
    st = ops.RowStats(torch.stack([x.double().mean(1), ((x.double() - x.double().mean(1, keepdim=True)) ** 2).sum(1)],
                                  1).float().view(M, 1, 2).contiguous(), K)
    y_pre = ops.linear_ln(x, wg, wg.sum(1), c2, eps=1e-6, pre=st)
    ref = _ln64(x, wg, c2, 1e-6)
    torch.cuda.synchronize()
    e_split = float((y_split.double() - ref).abs().max() / ref.abs().max())
    e_lna = float((y_lna.double() - ref).abs().max() / ref.abs().max())
    e_pre = float((y_pre.double() - ref).abs().max() / ref.abs().max())
    assert e_lna <= max(1.5 * e_split, 2e-6), (e_lna, e_split)
    assert e_pre <= max(1.5 * e_split, 2e-6), (e_pre, e_split)


def test_ln_in_the_a_load_feeds_the_attention_and_plane_outputs():
    """The QKV projection (K / V planes of the h3 attention) and fc1 (GELU,
    the next GEMM's planes) with the LN in their A load equal the split-pass
    versions to fp32 rounding of the statistics."""
    g = torch.Generator(device="cuda").manual_seed(7)
    B, S, H, K = 1, 3401, 6, 384
    x = torch.randn(B, S, K, device="cuda", generator=g)
    wq = torch.randn(3 * H * 64, K, device="cuda", generator=g) / K ** 0.5
    cq = torch.randn(3 * H * 64, device="cuda", generator=g) * 0.1
    w1 = torch.randn(1536, K, device="cuda", generator=g) / K ** 0.5
    c1 = torch.randn(1536, device="cuda", generator=g) * 0.1
    ops.set_attention_f32_variant("h3n")
    outs = {}
    for on in (False, True):
        ops.set_ln_handoff(on)
        att = ops.ln_qkv_attention(x, wq, wq.sum(1), cq, H, eps=1e-12)
        pl = ops.linear_ln_to_planes(x, w1, w1.sum(1), c1, act="gelu", eps=1e-12)
        outs[on] = (att.clone(), (pl.planes[0].float() + pl.planes[1].float()) * pl.rconst)
    torch.cuda.synchronize()
    for a, b in zip(outs[False], outs[True]):
        assert ((a - b).abs().max() / a.abs().max()) <= 2e-6


def test_yolos_program_with_and_without_the_handoff():
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver import program as PG

    prog, w = demo_tenant("fp32", 0, small=True)
    p = PG.parse(prog, w, gpu=True)
    x = p.input_tensor("cuda", torch.randn(p.inputs[0].shape).numpy())
    ops.set_attention_f32_variant("h3n")
    outs = {}
    for on in (False, True):
        ops.set_ln_handoff(on)
        cm = p.compile("cuda")
        # every LN; layer 0's statistics come from the patch GEMM's epilogue (its
        # rows of the token buffer) and the build (the constant cls / detection rows)
        assert cm.stats["ln_handoffs"] == 25
        with torch.no_grad():
            outs[on] = [o.clone() for o in cm(x)]
    torch.cuda.synchronize()
    for a, b in zip(outs[False], outs[True]):
        assert ((a - b).abs().max() / a.abs().max()) <= 1e-5


@pytest.mark.parametrize("M,N,K,act", [(3401, 384, 384, None), (257, 132, 64, "gelu"), (100, 1536, 384, "relu")])
def test_lds_epilogue_equals_the_register_epilogue(M, N, K, act):
    """Plain fp32-C GEMMs through the LDS epilogue (float4 row stores and
    residual loads): the same arithmetic in the same order, bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    outs = []
    for on in (False, True):
        ops.set_gemm_f32h3_lds_epilogue(on)
        try:
            outs.append(ops.linear(x, w, b, act=act, residual=r))
        finally:
            ops.set_gemm_f32h3_lds_epilogue(False)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_wide_lna_tiles_are_bit_identical():
    """fc1 (LN in the A load, GELU, the next GEMM's planes) on 128 x 256 tiles
    with 8 waves (ops.set_gemm_f32h3_lna_wide) equals the 128 x 128 form."""
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(1, 3401, 384, device="cuda", generator=g)
    w1 = torch.randn(1536, 384, device="cuda", generator=g) / 384 ** 0.5
    c1 = torch.randn(1536, device="cuda", generator=g) * 0.1
    ops.set_ln_handoff(True)
    outs = []
    for on in (False, True):
        ops.set_gemm_f32h3_lna_wide(on)
        try:
            pl = ops.linear_ln_to_planes(x, w1, w1.sum(1), c1, act="gelu", eps=1e-12)
            outs.append(pl.planes.clone())
        finally:
            ops.set_gemm_f32h3_lna_wide(False)
    assert torch.equal(outs[0], outs[1])
