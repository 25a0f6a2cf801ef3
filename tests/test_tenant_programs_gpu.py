"""General tenants on gfx950 kernels: a ResNet-18 conv net and a Llama decoder
(head_dim 128, causal, grouped-query, rotary) as pod-server programs, each
against an fp64 evaluation of its own torch module, and co-hosted with YOLOS
in one GPU pod server (HIP graphs) -- VERDICT r4 "next round" item 1."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from nos_amd import ops  # noqa: E402
from nos_amd.models.llama_program import llama_config, llama_model, llama_program  # noqa: E402
from nos_amd.models.resnet import resnet18, resnet_tenant  # noqa: E402
from nos_amd.podserver import program as PG  # noqa: E402


@pytest.fixture(autouse=True)
def _h3():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    prev = ops.f32_math()
    ops.set_f32_math("h3")
    yield
    ops.set_f32_math(prev)


def _err(got, ref64) -> float:
    return float((got.double() - ref64).abs().max() / ref64.abs().max())


def test_resnet18_program_on_gpu_matches_fp64():
    m = resnet18(seed=0)
    prog, w = resnet_tenant("fp32", 0)
    cm = PG.parse(prog, w, gpu=True).compile("cuda")
    assert cm.stats["kernels"] == 21  # 20 convs (BN, residual, ReLU fused) + fc
    x = torch.randn(1, 3, 224, 224, device="cuda")
    with torch.no_grad():
        got = cm(x)[0]
        ref64 = m.double().cuda()(x.double())
        f32 = m.float()(x)
    e, e32 = _err(got, ref64), _err(f32, ref64)
    assert e <= max(4 * e32, 1e-5), (e, e32)


def test_llama_program_on_gpu_matches_fp64():
    m = llama_model(llama_config(False), 0)
    prog, w = llama_program(m, 64)
    cm = PG.parse(prog, w, gpu=True).compile("cuda")
    ids = torch.randint(0, m.config.vocab_size, (1, 64), device="cuda")
    with torch.no_grad():
        got = cm(ids.int())[0]
        m = m.cuda()
        f32 = m(ids).logits
        ref64 = m.double()(ids).logits
    e, e32 = _err(got, ref64), _err(f32, ref64)
    assert e <= max(4 * e32, 1e-5), (e, e32)


def test_gpu_pod_server_cohosts_three_model_families(tmp_path):
    """YOLOS (the demo tenant), ResNet-18 and a Llama decoder in ONE GPU pod
    server, graphs captured, each tenant answering with its module's result;
    the static estimate bounds every measured build footprint."""
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    lm = llama_model(llama_config(False), 0)
    progs = {"yolos": demo_tenant("fp32", 0, small=False), "resnet": resnet_tenant("fp32", 0),
             "llama": llama_program(lm, 64)}
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=4, memory_gb=64).start()
    try:
        clients = {}
        for name, (prog, w) in progs.items():
            c = clients[name] = PodClient(srv.path, connect_timeout_s=30)
            rep = c.register(name, prog, w, memory_limit_gb=4)
            est = PG.parse(prog, w, gpu=True).bytes_estimate_for(srv.kernel_config) / 2 ** 30
            # (+16 MB: the caching allocator's per-allocation rounding of ~100 small tensors)
            assert rep["footprint_gb"] <= est + 0.016, (name, rep["footprint_gb"], est)
        x = np.random.default_rng(0).standard_normal((1, 3, 224, 224)).astype(np.float32)
        ids = np.random.default_rng(1).integers(0, lm.config.vocab_size, (1, 64)).astype(np.int32)
        for _ in range(3):  # replays
            out_r, _ = clients["resnet"].infer(x, outputs=True)
            out_l, _ = clients["llama"].infer(ids, outputs=True)
            clients["yolos"].infer()
        with torch.no_grad():
            ref_r = resnet18(seed=0)(torch.from_numpy(x)).numpy()
            ref_l = lm(torch.from_numpy(ids).long()).logits.numpy()
        assert np.abs(out_r[0] - ref_r).max() <= 1e-4 * np.abs(ref_r).max()
        assert np.abs(out_l[0] - ref_l).max() <= 1e-4 * np.abs(ref_l).max()
        for c in clients.values():
            c.close()
    finally:
        srv.stop()


@pytest.mark.parametrize("family", ["resnet", "llama"])
def test_bf16_tenant_programs_run_on_gpu(family):
    """bf16 programs of the new families: bf16 weights / activations, the
    GEMM-class ops on the fp32 kernels over an fp32 copy (never less precise
    than asked); close to the fp32 module at bf16 tolerance."""
    if family == "resnet":
        m = resnet18(seed=0)
        prog, w = resnet_tenant("bf16", 0)
        x = torch.randn(1, 3, 224, 224)
        with torch.no_grad():
            ref = m(x)
        inp = x.cuda()
    else:
        lm = llama_model(llama_config(False), 0)
        prog, w = llama_program(lm, 64, dtype="bf16")
        ids = torch.randint(0, lm.config.vocab_size, (1, 64))
        with torch.no_grad():
            ref = lm(ids).logits
        inp = ids.int().cuda()
    cm = PG.parse(prog, w, gpu=True).compile("cuda")
    with torch.no_grad():
        got = cm(inp)[0].float().cpu()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max() <= 0.05 * ref.abs().max(), float((got - ref).abs().max() / ref.abs().max())


def test_grouped_conv_program_on_gpu_matches_fp64():
    """Depthwise + grouped convolutions exported from torch.nn run on the h3
    kernels within 4x torch-fp32's error against fp64."""
    from test_tenant_programs import MobileBlock

    from nos_amd.podserver.export import export

    m = MobileBlock().eval()
    x = torch.randn(2, 16, 20, 20)
    prog, w = export(m, x, name="mobile")
    cm = PG.parse(prog, w, gpu=True).compile("cuda")
    xc = x.cuda()
    with torch.no_grad():
        got = cm(xc)[0]
        mc = m.cuda()
        f32 = mc(xc)
        ref64 = mc.double()(xc.double())
    e, e32 = _err(got, ref64), _err(f32, ref64)
    assert e <= max(4 * e32, 1e-5), (e, e32)


def test_gpu_tenant_shape_variants_share_weights(tmp_path):
    """A decoder registered at sequence lengths 64 / 32 / 16 over one weight
    payload on the GPU server: one captured graph per shape, each request
    replays the graph of its input's shape and matches the module; the build
    footprint stays inside the variants' combined static estimate and well
    below three separate tenants' weights."""
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    lm = llama_model(llama_config(False), 0)
    progs = [llama_program(lm, s, rope_len=64) for s in (64, 32, 16)]
    w = progs[0][1]
    srv = PodServer(tmp_path / "s.sock", device="cuda", lanes=4, memory_gb=64).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=30)
        rep = c.register("llm", progs[0][0], w, memory_limit_gb=4, variants=[p for p, _ in progs[1:]])
        assert rep["input_shapes"] == [[1, 64], [1, 32], [1, 16]]
        parsed = PG.parse_variants([p for p, _ in progs], w, gpu=True)
        est = (sum(p.bytes_estimate_for(srv.kernel_config) for p in parsed) - 2 * parsed[0].param_bytes) / 2 ** 30
        assert rep["footprint_gb"] <= est + 0.016, (rep["footprint_gb"], est)
        t = next(iter(srv.tenants.values()))
        assert all(v.graph is not None for v in t.alts.values()) and t.graph is not None
        for s in (16, 64, 32, 16):
            ids = np.random.default_rng(s).integers(0, lm.config.vocab_size, (1, s)).astype(np.int32)
            out, _ = c.infer(ids, outputs=True)
            with torch.no_grad():
                ref = lm(torch.from_numpy(ids).long()).logits.numpy()
            assert out[0].shape == ref.shape
            assert np.abs(out[0] - ref).max() <= 1e-4 * np.abs(ref).max()
        c.close()
    finally:
        srv.stop()


def test_bare_fp32_attention_runs_the_h3_flash_kernel():
    """A post-LN block's attention (its QKV projection reads the residual
    stream, so no LayerNorm folds into it) under h3 math: the per-row-scale
    h3 flash kernel, within 4x torch fp32's error against fp64."""
    from nos_amd.podserver.program import Builder

    g = np.random.default_rng(3)
    S, D, H = 333, 384, 6
    b = Builder("bare-attn")
    x = b.input("x", [1, S, D])
    wq = b.param("wqkv", (g.standard_normal((3 * D, D)) / D ** 0.5).astype(np.float32))
    bq = b.param("bqkv", (g.standard_normal(3 * D) * 0.1).astype(np.float32))
    wo = b.param("wo", (g.standard_normal((D, D)) / D ** 0.5).astype(np.float32))
    a = b.op("attention", b.op("linear", x, wq, bq), heads=H)
    y = b.op("add", b.op("linear", a, wo), x, out="y")
    prog, w = b.build([y])
    p = PG.parse(prog, w, gpu=True)
    cm = p.compile("cuda")
    assert any(s.kind == "attention" for s in cm.steps)
    xt = torch.from_numpy(g.standard_normal((1, S, D)).astype(np.float32))
    with torch.no_grad():
        got = cm(xt.cuda())[0]
        ps = {k: v.double() for k, v in p.tensors("cpu").items()}
        qkv = xt.double() @ ps["wqkv"].t() + ps["bqkv"]
        q, k, v = qkv.view(1, S, 3, H, D // H).unbind(2)
        att = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q, k) / (D // H) ** 0.5, -1)
        o = torch.einsum("bhqk,bkhd->bqhd", att, v).reshape(1, S, D)
        ref64 = o @ ps["wo"].t() + xt.double()
        f32 = p.reference(xt)[0]
    e, e32 = _err(got.cpu(), ref64), _err(f32, ref64)
    assert e <= max(4 * e32, 1e-5), (e, e32)
