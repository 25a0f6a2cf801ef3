"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references.

Every case runs the native kernel (libnos_hip.so must be loaded: the ops fail
loudly on a GPU box without it) and compares with the fp32 reference of the
same op on the CPU.  Tolerances are bf16-output tolerances (outputs are
rounded to bf16: 2^-8 relative).
"""
from __future__ import annotations

import pytest
import torch

from nos_amd import ops

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(y: torch.Tensor, ref: torch.Tensor) -> float:
    return ((y.float().cpu() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-6)).item()


@pytest.fixture(autouse=True)
def _native():
    from nos_amd.ops import _lib

    _lib.require_native_on_gpu()
    torch.manual_seed(0)


@pytest.mark.parametrize("M,N,K,act,resid", [
    (3401, 1152, 384, None, False), (3401, 1536, 384, "gelu", False), (3401, 384, 1536, None, True),
    (3401, 384, 384, None, True), (100, 4, 384, "relu", False), (257, 200, 128, None, False),
    (1, 8, 64, None, False), (4096, 4096, 1024, None, False)])
@pytest.mark.parametrize("policy", ["throughput", "latency", "big", "wide"])
def test_linear(M, N, K, act, resid, policy):
    ops.set_gemm_policy(policy)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16) if resid else None
    y = ops.linear(x, w, b, act=act, residual=r)
    ref = ops.linear_ref(x.cpu().float(), w.cpu().float(), b.cpu().float(), act=act,
                         residual=r.cpu().float() if resid else None)
    ops.set_gemm_policy("throughput")
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("M,N,K,act", [(3401, 1152, 384, None), (3401, 1536, 384, "gelu"), (77, 100, 128, None),
                                       (1, 64, 64, None), (300, 384, 384, None)])
@pytest.mark.parametrize("policy", ["throughput", "latency", "big", "wide"])
def test_linear_layernorm_fused(M, N, K, act, policy):
    ops.set_gemm_policy(policy)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16) * 2 + 0.5
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    g = torch.randn(K, device=DEV, dtype=torch.bfloat16)
    be = torch.randn(K, device=DEV, dtype=torch.bfloat16)
    wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
    y = ops.linear_ln(x, wg, c1, c2, act=act)
    ln = torch.nn.functional.layer_norm(x.float().cpu(), (K,), g.float().cpu(), be.float().cpu(), 1e-12)
    ref = ops.linear_ref(ln, w.cpu().float(), b.cpu().float(), act=act)
    ops.set_gemm_policy("throughput")
    assert _rel(y, ref) < 2e-2


@pytest.mark.parametrize("M,N,K,act,resid,ln", [
    (3401, 1152, 384, None, False, True), (3401, 1536, 384, "gelu", False, True), (3401, 384, 1536, None, True, False),
    (257, 200, 128, "relu", False, False), (1000, 384, 64, None, True, False), (77, 100, 128, None, False, True)])
@pytest.mark.parametrize("persist", [1, 2, 13])
def test_linear_persistent_grid(M, N, K, act, resid, ln, persist):
    """Persistent bf16 GEMM grid: every workgroup walks several tiles of its
    XCD's chunk with the next tile's loads in flight during the epilogue.
    persist = 13 is an explicit grid of 13 workgroups (uneven over the XCDs)."""
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16) * 2 + 0.5
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16) if resid else None
    max_wg = persist if persist > 8 else 0
    if persist <= 8:
        ops.set_gemm_persistent(persist)
    try:
        if ln:
            g = torch.randn(K, device=DEV, dtype=torch.bfloat16)
            be = torch.randn(K, device=DEV, dtype=torch.bfloat16)
            wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
            y = ops.linear_ln(x, wg, c1, c2, act=act, max_wg=max_wg)
            xin = torch.nn.functional.layer_norm(x.float().cpu(), (K,), g.float().cpu(), be.float().cpu(), 1e-12)
        else:
            y = ops.linear(x, w, b, act=act, residual=r, max_wg=max_wg)
            xin = x.cpu().float()
    finally:
        ops.set_gemm_persistent(0)
    ref = ops.linear_ref(xin, w.cpu().float(), b.cpu().float(), act=act, residual=r.cpu().float() if resid else None)
    assert _rel(y, ref) < 2e-2


@pytest.mark.parametrize("B,S,H", [(1, 3401, 6), (2, 200, 2), (1, 64, 1), (1, 1000, 3), (1, 65, 2), (1, 1, 1),
                                   (3, 129, 4)])
def test_attention(B, S, H):
    qkv = torch.randn(B, S, 3 * H * 64, device=DEV, dtype=torch.bfloat16)
    o = ops.attention_qkv(qkv, H)
    ref = ops.attention_qkv(qkv.cpu().float(), H)
    assert o.shape == (B, S, H * 64)
    assert (o.float().cpu() - ref).abs().max().item() < 1e-2


def test_attention_large_logits_rescale_path():
    """Scores spanning many rescale thresholds (peaky rows) exercise the deferred-rescale branch."""
    B, S, H = 1, 777, 2
    qkv = torch.randn(B, S, 3 * H * 64, device=DEV, dtype=torch.bfloat16)
    qkv[..., : H * 64] *= 6.0
    # increasing key norms along the sequence -> the running max keeps growing
    ramp = torch.linspace(0.2, 3.0, S, device=DEV).view(1, S, 1)
    qkv[..., H * 64: 2 * H * 64] = (qkv[..., H * 64: 2 * H * 64].float() * ramp).bfloat16()
    o = ops.attention_qkv(qkv, H)
    ref = ops.attention_qkv(qkv.cpu().float(), H)
    assert (o.float().cpu() - ref).abs().max().item() < 2e-2


def test_attention_strided_views():
    """q/k/v as column views of one packed [B, S, 3*hid] tensor (no copies) and a padded output."""
    B, S, H = 2, 300, 3
    hid = H * 64
    qkv = torch.randn(B, S, 3 * hid, device=DEV, dtype=torch.bfloat16)
    out = torch.zeros(B, S, hid + 64, device=DEV, dtype=torch.bfloat16)
    q, k, v = (qkv[..., i * hid:(i + 1) * hid].unflatten(-1, (H, 64)) for i in range(3))
    ops.attention(q, k, v, out=out[..., :hid].unflatten(-1, (H, 64)))
    ref = ops.attention_ref(q.cpu().float(), k.cpu().float(), v.cpu().float())
    assert (out[..., :hid].float().cpu() - ref.reshape(B, S, hid)).abs().max().item() < 1e-2
    assert out[..., hid:].abs().max().item() == 0  # padding untouched


@pytest.mark.parametrize("variant", ["w4k64", "w4k64g2", "w4k32", "w4k32o4", "w4k32g2", "w2k64", "w8k64", "x6", "x6n",
                                     "x6k2", "x6k3", "x6k4", "auto"])
@pytest.mark.parametrize("B,S,H", [(1, 3401, 6), (2, 77, 3), (1, 1, 1), (1, 33, 2), (3, 300, 2), (1, 129, 1)])
def test_attention_fp32_exact(B, S, H, variant):
    """fp32 MFMA attention against an fp64 reference: exact-f32 numerics."""
    qkv = torch.randn(B, S, 3 * H * 64, device=DEV, dtype=torch.float32)
    ops.set_attention_f32_variant(variant)
    try:
        y = ops.attention_qkv(qkv, H)
    finally:
        ops.set_attention_f32_variant("auto")
    q, k, v = qkv.cpu().double().view(B, S, 3, H, 64).unbind(2)
    p = torch.softmax((q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / 8.0, dim=-1)
    ref = (p @ v.transpose(1, 2)).transpose(1, 2).reshape(B, S, H * 64)
    assert y.dtype == torch.float32
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("scale_in", [1.0, 4.0])
def test_attention_fp32_split_is_as_accurate_as_exact_f32(scale_in):
    """The bf16x6 split kernel (three bf16 pieces per fp32 operand, six exact
    piece products) against fp64, next to the exact-f32 MFMA kernel on the
    same inputs: its error may not exceed the exact kernel's by more than 50 %
    (mean and max), at YOLOS-small's shape, plain and with logits ~ +-100."""
    torch.manual_seed(3)
    B, S, H = 1, 3401, 6
    qkv = torch.randn(B, S, 3 * H * 64, device=DEV) * scale_in
    q, k, v = qkv.cpu().double().view(B, S, 3, H, 64).unbind(2)
    p = torch.softmax((q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / 8.0, dim=-1)
    ref = (p @ v.transpose(1, 2)).transpose(1, 2).reshape(B, S, H * 64)
    errs = {}
    for variant in ("w4k32o4", "x6"):
        ops.set_attention_f32_variant(variant)
        try:
            y = ops.attention_qkv(qkv, H)
        finally:
            ops.set_attention_f32_variant("auto")
        e = (y.cpu().double() - ref).abs()
        errs[variant] = (e.max().item(), e.mean().item())
    print("attention fp32 error vs fp64 (max, mean):", errs)
    assert errs["x6"][0] <= 1.5 * errs["w4k32o4"][0] + 1e-7, errs
    assert errs["x6"][1] <= 1.5 * errs["w4k32o4"][1], errs


@pytest.mark.parametrize("M,N,K", [(3401, 1152, 384), (3401, 384, 1536)])
def test_linear_fp32_split_is_as_accurate_as_exact_f32(M, N, K):
    """bf16x6 split GEMM vs the exact-f32 MFMA GEMM, both against fp64 on the
    same inputs: max and mean error within 1.5x of the exact kernel's."""
    torch.manual_seed(5)
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    ref = x.cpu().double() @ w.cpu().double().t()
    errs = {}
    for m in ("exact", "x6"):
        ops.set_f32_math(m)
        try:
            e = (ops.linear(x, w).cpu().double() - ref).abs()
        finally:
            ops.set_f32_math("exact")
        errs[m] = (e.max().item(), e.mean().item())
    print("linear fp32 error vs fp64 (max, mean):", errs)
    assert errs["x6"][0] <= 1.5 * errs["exact"][0] and errs["x6"][1] <= 1.5 * errs["exact"][1], errs


@pytest.mark.parametrize("tile", [-1, 0, 1, 2, 3, 5, 7])
@pytest.mark.parametrize("M,N,K,kind", [(3401, 1152, 384, "ln"), (3401, 384, 1536, "resid"), (257, 200, 96, "gelu"),
                                        (100, 92, 64, "ln"), (3401, 1152, 384, "qkv"), (64, 64, 32, "plain")])
def test_linear_fp32_x6_pipelined_loop_is_bit_identical(tile, M, N, K, kind):
    """The software-pipelined x6 K loop (next step's LDS reads and A split
    under the current step's MFMAs) accumulates in the plain loop's order:
    every tile config, epilogue and K (one stage, two, many) bit for bit."""
    from nos_amd.ops import _lib

    torch.manual_seed(M + N + K)
    x = torch.randn(1, M, K, device=DEV) * 2 + 0.5
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    r = torch.randn(1, M, N, device=DEV)
    g, be = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, g, be)

    def run():
        if kind == "ln":
            return (ops.linear_ln(x, wg, c1, c2, act="gelu"),)
        if kind == "qkv":
            H = N // 192
            qkv, ws = ops.linear_ln_qkv_x6(x, wg, c1, c2, H)
            return (qkv[..., :N // 3].clone(), ws[:M * 6 * (N // 3)].clone())  # the planes' S rows (no padding)
        if kind == "resid":
            return (ops.linear(x, w, b, residual=r),)
        return (ops.linear(x, w, b, act="gelu" if kind == "gelu" else None),)

    ops.set_f32_math("x6")
    ops.set_attention_f32_variant("x6n")
    _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(tile), "set_tile")
    try:
        ops.set_gemm_f32x6_pipeline(False)
        ref = run()
        ops.set_gemm_f32x6_pipeline(True)
        got = run()
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_f32x6_pipeline(True)
        _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(-1), "set_tile")
        ops.set_f32_math("exact")
        ops.set_attention_f32_variant("auto")
    for a, c in zip(ref, got):
        assert torch.equal(a, c)


@pytest.mark.parametrize("stage,tile", [(1, -1), (2, -1), (0, 3), (0, 5), (0, 7)])
@pytest.mark.parametrize("M,N,K,ln", [(3401, 1152, 384, True), (3401, 384, 1536, False), (257, 200, 96, False),
                                      (100, 92, 384, True)])
def test_linear_fp32_split_stage_configs(stage, tile, M, N, K, ln):
    """The x6 GEMM's other K-stage configs (1: BK 32 in a 3-deep ring, 2: BK 64
    -- K % 64 != 0 falls back to BK 32) and the 128x64 4x1-wave tile against
    fp64 at the exact-f32 tolerance."""
    from nos_amd.ops import _lib

    x = torch.randn(M, K, device=DEV) * 2 + 0.5
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    ops.set_f32_math("x6")
    _lib.check(_lib.lib().nos_gemm_f32x6_set_stage(stage), "set_stage")
    _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(tile), "set_tile")
    try:
        if ln:
            g, be = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
            wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
            y = ops.linear_ln(x, wg, c1, c2, act="gelu")
            xd = torch.nn.functional.layer_norm(x.cpu().double(), (K,), g.cpu().double(), be.cpu().double(), 1e-12)
            ref = torch.nn.functional.gelu(xd @ w.cpu().double().t() + b.cpu().double())
        else:
            y = ops.linear(x, w, b)
            ref = x.cpu().double() @ w.cpu().double().t() + b.cpu().double()
    finally:
        _lib.check(_lib.lib().nos_gemm_f32x6_set_stage(0), "set_stage")
        _lib.check(_lib.lib().nos_gemm_f32x6_set_tile(-1), "set_tile")
        ops.set_f32_math("exact")
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


def test_attention_fp32_strided_and_large_logits():
    B, S, H = 2, 129, 6
    base = torch.randn(B, S, 3 * H * 64 + 64, device=DEV) * 4.0  # padded rows: ld != 3*H*64, logits ~ +-100
    qkv = base[:, :, : 3 * H * 64]
    y = ops.attention_qkv(qkv, H)
    ref = ops.attention_ref(*(t.cpu() for t in qkv.view(B, S, 3, H, 64).unbind(2))).reshape(B, S, H * 64)
    assert torch.isfinite(y).all()
    assert (y.cpu() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,K,act,resid", [
    (3401, 1152, 384, None, False), (3401, 1536, 384, "gelu", False), (3401, 384, 1536, None, True),
    (3401, 384, 384, None, True), (100, 92, 384, "relu", False), (100, 4, 384, None, False), (257, 200, 96, None, True),
    (8 * 3401, 384, 1536, None, True), (1, 8, 32, None, False), (3401, 100, 384, None, False)])
@pytest.mark.parametrize("policy", ["throughput", "latency", "small"])
@pytest.mark.parametrize("math_", ["exact", "x6"])
def test_linear_fp32_exact(M, N, K, act, resid, policy, math_):
    """fp32 GEMM (exact-f32 MFMA, and the bf16x6 split) against an fp64
    reference at the exact-f32 tolerance, every tile shape."""
    x = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV) if resid else None
    ops.set_gemm_f32_policy(policy)
    ops.set_f32_math(math_)
    try:
        y = ops.linear(x, w, b, act=act, residual=r)
    finally:
        ops.set_gemm_f32_policy("latency")
        ops.set_f32_math("exact")
    ref = x.cpu().double() @ w.cpu().double().t() + b.cpu().double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    elif act == "relu":
        ref = ref.clamp_min(0)
    if resid:
        ref = ref + r.cpu().double()
    assert y.dtype == torch.float32 and y.shape == (M, N)
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("M,N,K,act", [(3401, 1152, 384, None), (3401, 1536, 384, "gelu"), (77, 100, 384, None),
                                       (1, 64, 64, None), (300, 384, 384, None)])
@pytest.mark.parametrize("math_", ["exact", "x6"])
def test_linear_layernorm_fused_fp32(M, N, K, act, math_):
    x = torch.randn(M, K, device=DEV) * 2 + 0.5
    w = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV)
    g = torch.randn(K, device=DEV)
    be = torch.randn(K, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, g, be)
    ops.set_f32_math(math_)
    try:
        y = ops.linear_ln(x, wg, c1, c2, act=act, eps=1e-12)
    finally:
        ops.set_f32_math("exact")
    xd = x.cpu().double()
    ln = torch.nn.functional.layer_norm(xd, (K,), g.cpu().double(), be.cpu().double(), 1e-12)
    ref = ln @ w.cpu().double().t() + b.cpu().double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    err = (y.cpu().double() - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


def test_yolos_fp32_native_attention_matches_torch():
    from nos_amd.models.yolos import YolosConfig, YolosDetector, demo_input_hw, make_demo_input

    cfg = YolosConfig.small()
    m = YolosDetector(cfg, backend="native")
    m.reset_parameters(1)
    m = m.to(DEV, torch.float32).eval()
    x = make_demo_input(cfg, device=DEV, dtype=torch.float32, hw=demo_input_hw(), seed=1)
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        logits, boxes = m(x)
        m.backend = "torch"
        rl, rb = m(x)
    assert (logits - rl).abs().max().item() < 1e-3 * max(1.0, rl.abs().max().item())
    assert (boxes - rb).abs().max().item() < 1e-4


def test_layernorm_strided_x_and_residual():
    """x and residual are row-strided views of wider buffers: the
    kernel reads each with its own stride and writes a dense sum."""
    rows, D = 300, 384
    xb = torch.randn(rows, D + 64, device=DEV, dtype=torch.bfloat16)
    rb = torch.randn(rows, D + 128, device=DEV, dtype=torch.bfloat16)
    x, r = xb[:, :D], rb[:, 64:64 + D]
    g = torch.randn(D, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(D, device=DEV, dtype=torch.bfloat16)
    y, s = ops.layernorm(x, g, b, 1e-12, residual=r)
    ry, rs = ops.layernorm_ref(x.cpu(), g.cpu(), b.cpu(), 1e-12, residual=r.cpu())
    assert s.is_contiguous() and _rel(s, rs) < 1e-2 and _rel(y, ry) < 2e-2
    with pytest.raises(ValueError):
        ops.layernorm(x, g.float(), b, 1e-12)


def test_layernorm_with_residual_sum():
    x = torch.randn(3401, 384, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(3401, 384, device=DEV, dtype=torch.bfloat16)
    g = torch.randn(384, device=DEV, dtype=torch.bfloat16)
    bb = torch.randn(384, device=DEV, dtype=torch.bfloat16)
    y, s = ops.layernorm(x, g, bb, 1e-12, residual=r)
    ref_s = x.cpu().float() + r.cpu().float()
    assert (s.float().cpu() - ref_s).abs().max().item() < 3e-2
    # the residual stream is bf16 (as in the model): normalise the rounded sum
    ref_y = torch.nn.functional.layer_norm(ref_s.bfloat16().float(), (384,), g.cpu().float(), bb.cpu().float(),
                                           1e-12)
    assert _rel(y, ref_y) < 1e-2


def test_yolos_native_matches_torch_path():
    from nos_amd.models.yolos import YolosConfig, YolosDetector, demo_input_hw, make_demo_input

    cfg = YolosConfig.small()
    m = YolosDetector(cfg)
    m.reset_parameters(0)
    m = m.to(DEV, torch.bfloat16).eval()
    x = make_demo_input(cfg, device=DEV, hw=demo_input_hw(), seed=0)
    with torch.no_grad():
        lg, bx = m(x)
        m.backend = "torch"
        lr, br = m(x)
    assert (lg.float() - lr.float()).abs().max().item() < 0.05 * max(1.0, lr.float().abs().max().item())
    assert (bx.float() - br.float()).abs().max().item() < 2e-2


def test_graphed_tenants_on_cumask_streams():
    from nos_amd.gpu.topology import split_even
    from nos_amd.models.tenants import InferenceTenants, TenantSpec
    from nos_amd.models.yolos import YolosConfig, demo_input_hw
    from nos_amd.ops.streams import device_info

    n_cus = device_info(0)["num_cus"]
    specs = [TenantSpec(f"p{i}", s.cus()) for i, s in enumerate(split_even(2))]
    ts = InferenceTenants(specs, n_cus, YolosConfig.small(), demo_input_hw(), use_graphs=True)
    ts.prepare()
    dt = ts.run(2)
    ts.close()
    assert dt > 0


def test_cumask_stream_roundtrip():
    from nos_amd.ops.streams import CUMaskedStream

    cus = list(range(0, 256, 2))
    s = CUMaskedStream(cus, 256)
    try:
        assert s.get_mask() == cus
        x = torch.randn(1024, 1024, device=DEV)
        with torch.cuda.stream(s.torch):
            y = x @ x
        s.synchronize()
        assert torch.isfinite(y).all()
    finally:
        s.close()


def test_probes_report_sane_numbers():
    from nos_amd.ops import probes

    stream = torch.cuda.current_stream().cuda_stream
    summary = probes.placement_summary(probes.placement(stream))
    assert len(summary["xccs"]) == 8
    assert probes.hbm_gbps(stream) > 1000
    assert probes.mfma_peak_tflops(stream, 1024) > 500


@pytest.mark.parametrize("budget", [8, 32, 40])
def test_slice_sized_persistent_grids_are_bit_identical(budget):
    """With a CU budget (a CU-mask slice's popcount, ops.set_cu_budget) the fp32
    GEMMs, the fp32 attention and the bf16 GEMM launch at most occupancy x
    budget workgroups that each walk a chunk of tiles (nos::xcd_chunk): the
    output must equal the one-workgroup-per-tile launch bit for bit (the tile
    math is the same; only the tile -> workgroup mapping changes)."""
    torch.manual_seed(budget)
    x = torch.randn(3401, 384, device=DEV)
    w = torch.randn(1152, 384, device=DEV) * 0.05
    b = torch.randn(1152, device=DEV)
    r = torch.randn(3401, 1152, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, torch.randn(384, device=DEV), torch.randn(384, device=DEV))
    qkv = torch.randn(1, 3401, 3 * 6 * 64, device=DEV)
    xb, wb, rb = x.bfloat16(), w.bfloat16(), r.bfloat16()

    def run():
        outs = []
        for m in ("exact", "x6"):
            ops.set_f32_math(m)
            for pol in ("small", "latency", "throughput"):
                ops.set_gemm_f32_policy(pol)
                outs += [ops.linear(x, w, b, act="gelu", residual=r), ops.linear_ln(x, wg, c1, c2, act="gelu")]
        ops.set_f32_math("exact")
        ops.set_gemm_f32_policy("latency")
        for var in ("w4k32", "w4k64g2", "w4k32o4", "x6n", "x6k2"):
            ops.set_attention_f32_variant(var)
            outs.append(ops.attention_qkv(qkv, 6))
        ops.set_attention_f32_variant("auto")
        outs.append(ops.linear(xb, wb, None, residual=rb))
        torch.cuda.synchronize()
        return outs

    assert ops.cu_budget() == 0
    ref = run()
    ops.set_cu_budget(budget)
    try:
        got = run()
    finally:
        ops.set_cu_budget(0)
    for a, c in zip(ref, got):
        assert torch.equal(a, c)


@pytest.mark.parametrize("B,S,H", [(1, 3401, 6), (2, 77, 3), (3, 33, 2)])
@pytest.mark.parametrize("variant", ["x6n", "x6"])
def test_qkv_projection_writing_the_attention_planes_is_bit_identical(B, S, H, variant):
    """LN-QKV GEMM whose epilogue writes K/V as the bf16x6 attention's planes
    (no fp32 K/V, no split kernel) == the unfused LN GEMM + x6 attention, bit
    for bit (the same pieces of the same fp32 values), padding rows between
    batches included."""
    torch.manual_seed(B * S)
    K = 384
    x = torch.randn(B, S, K, device=DEV) * 2 + 0.5
    w = torch.randn(3 * H * 64, K, device=DEV) * 0.05
    b = torch.randn(3 * H * 64, device=DEV)
    wg, c1, c2 = ops.fold_layernorm(w, b, torch.randn(K, device=DEV), torch.randn(K, device=DEV))
    ops.set_f32_math("x6")
    ops.set_attention_f32_variant(variant)
    try:
        ref = ops.attention_qkv(ops.linear_ln(x, wg, c1, c2), H)
        qkv, ws = ops.linear_ln_qkv_x6(x, wg, c1, c2, H)
        got = ops.attention_presplit(qkv, ws, H)
        torch.cuda.synchronize()
    finally:
        ops.set_f32_math("exact")
        ops.set_attention_f32_variant("auto")
    assert torch.equal(got, ref)


@pytest.mark.parametrize("variant", ["x6n", "x6"])
def test_attention_planes_padding_rows_never_reach_the_output(variant):
    """Garbage in the planes' padding rows past S of each batch (NaN here)
    never reaches the output: the kernel's tail tile re-reads the last key
    instead of the padding rows (no memset per call), so the result stays
    bit-identical to the unfused path."""
    torch.manual_seed(7)
    B, S, H, K = 2, 77, 3, 384
    x = torch.randn(B, S, K, device=DEV)
    w = torch.randn(3 * H * 64, K, device=DEV) * 0.05
    wg, c1, c2 = ops.fold_layernorm(w, torch.randn(3 * H * 64, device=DEV), torch.randn(K, device=DEV),
                                    torch.randn(K, device=DEV))
    ops.set_f32_math("x6")
    ops.set_attention_f32_variant(variant)
    try:
        ref = ops.attention_qkv(ops.linear_ln(x, wg, c1, c2), H)
        qkv, ws = ops.linear_ln_qkv_x6(x, wg, c1, c2, H)
        skvp = (S + 31) // 32 * 32
        row = 6 * H * 64  # int16 elements per token row of the six planes
        planes = ws[:B * skvp * row].view(B, skvp, row)
        planes[:, S:, :] = 0x7FC0  # bf16 NaN in every padding row
        got = ops.attention_presplit(qkv, ws, H)
        torch.cuda.synchronize()
    finally:
        ops.set_f32_math("exact")
        ops.set_attention_f32_variant("auto")
    assert torch.isfinite(got).all() and torch.equal(got, ref)
