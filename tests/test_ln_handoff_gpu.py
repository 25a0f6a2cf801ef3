"""The pre-LN residual GEMM that hands the next LN-GEMM its planes
(``nos_gemm_f32h3_ln_out``, VERDICT r4 item 2: no ``nos_split_rows_h3``
launch between the residual GEMMs and the LN-GEMMs of an encoder): its fp32
output and its planes equal the separate GEMM + split pass bit for bit, and a
YOLOS program run with the handoff equals the one without."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu

from nos_amd import ops  # noqa: E402


@pytest.fixture(autouse=True)
def _h3():
    prev, prev_h = ops.f32_math(), ops.ln_handoff_active()
    ops.set_f32_math("h3")
    yield
    ops.set_f32_math(prev)
    ops.set_ln_handoff(prev_h)


@pytest.mark.parametrize("M,N,K", [(3401, 384, 384), (3401, 384, 1536), (100, 768, 384), (257, 132, 64)])
def test_ln_out_equals_gemm_then_split(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N)
    x = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g) * 3
    ap, rinv = ops._split_rows_h3(x, ln=False)
    a = ops.H3Planes(ap, rinv, 0.0, (M, K))
    y_ref = ops.linear_planes(a, w, b, residual=r)
    p_ref, ri_ref = ops._split_rows_h3(y_ref, ln=True, eps=1e-12)
    y, lnp = ops.linear_planes(a, w, b, residual=r, ln_eps=1e-12)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref)
    assert torch.equal(lnp.rinv, ri_ref)
    if N <= 512:  # the split pass reduces such rows over a half-wave too: the same sums in the same order
        assert torch.equal(lnp.planes, p_ref)
    else:         # a full-wave reduction there: the same values up to fp32 rounding of the statistics
        v, v_ref = lnp.planes[0].float() + lnp.planes[1].float(), p_ref[0].float() + p_ref[1].float()
        assert ((v - v_ref).abs() <= 1e-5 * v_ref.abs().amax(dim=1, keepdim=True)).all()


def test_yolos_program_with_and_without_the_handoff_is_bit_identical():
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
        assert cm.stats["ln_handoffs"] == 23  # layer 0's LN reads the embeddings; the final LN a token slice
        with torch.no_grad():
            outs[on] = [o.clone() for o in cm(x)]
    torch.cuda.synchronize()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
