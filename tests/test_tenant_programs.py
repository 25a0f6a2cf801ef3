"""General pod-server tenants on the CPU: a torch.nn conv net (exported with
torch.fx) and a ``transformers`` Llama decoder as programs, compiled by the
server's graph compiler and co-hosted with YOLOS in one pod server.  Each is
compared with its own torch fp32 module.  GPU runs (gfx950 kernels, fp64
references): tests/test_tenant_programs_gpu.py."""
from __future__ import annotations

import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from nos_amd.models.llama_program import llama_config, llama_model, llama_program
from nos_amd.models.resnet import resnet_tenant, resnet_tiny
from nos_amd.models.yolos_program import demo_tenant
from nos_amd.podserver import program as PG
from nos_amd.podserver.client import PodClient, PodServerError
from nos_amd.podserver.export import ExportError, export
from nos_amd.podserver.server import PodServer


@pytest.fixture(scope="module")
def llama():
    m = llama_model(llama_config(False), 0)
    return m, llama_program(m, 64)


def test_resnet_program_matches_the_module():
    prog, w = resnet_tenant("fp32", 0, small=False)
    p = PG.parse(prog, w, gpu=True)
    cm = p.compile("cpu")
    # every conv + BN (+ residual) (+ ReLU) is one kernel step
    assert cm.stats["batchnorm_folded"] == 6 and cm.stats["residual_fused"] == 2 and cm.stats["activation_fused"] == 5
    assert sum(1 for s in cm.steps if s.kind == "conv2d") == 6
    x = torch.randn(1, 3, 32, 32)
    with torch.no_grad():
        ref = resnet_tiny(0)(x)
    assert torch.allclose(cm(x)[0], ref, atol=1e-5, rtol=1e-5)
    assert torch.allclose(p.reference(x)[0], ref, atol=1e-5, rtol=1e-5)


class MobileBlock(nn.Module):
    """Depthwise-separable and grouped convolutions (MobileNet / ResNeXt
    style): depthwise 3x3 + BN + ReLU, pointwise 1x1, grouped 3x3 stride 2."""

    def __init__(self, c=16):
        super().__init__()
        self.dw = nn.Conv2d(c, c, 3, padding=1, groups=c, bias=False)
        self.bn = nn.BatchNorm2d(c)
        self.pw = nn.Conv2d(c, 2 * c, 1)
        self.gc = nn.Conv2d(2 * c, 2 * c, 3, stride=2, padding=1, groups=4)
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2 * c, 10)
        g = torch.Generator().manual_seed(0)
        with torch.no_grad():
            for p in self.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.2)
            self.bn.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
            self.bn.running_var.copy_(torch.rand(c, generator=g) + 0.5)

    def forward(self, x):
        x = torch.relu(self.bn(self.dw(x)))
        x = torch.relu(self.pw(x))
        x = self.gc(x)
        return self.fc(torch.flatten(self.pool(x), 1))


def test_grouped_and_depthwise_convs_export_and_match():
    m = MobileBlock().eval()
    x = torch.randn(2, 16, 20, 20)
    prog, w = export(m, x, name="mobile")
    p = PG.parse(prog, w, gpu=True)
    cm = p.compile("cpu")
    assert cm.stats["batchnorm_folded"] == 1
    assert [n.attrs.get("groups", 1) for n in p.nodes if n.op == "conv2d"] == [16, 1, 4]
    with torch.no_grad():
        ref = m(x)
    assert torch.allclose(cm(x)[0], ref, atol=1e-5, rtol=1e-5)


def test_llama_program_matches_hf(llama):
    m, (prog, w) = llama
    p = PG.parse(prog, w, gpu=True)
    cm = p.compile("cpu")
    L = m.config.num_hidden_layers
    assert cm.stats["linears_merged"] == 5 * L            # q / k / v and gate / up
    assert cm.stats["rmsnorm_folded"] == 2 * L + 1 and cm.stats["rotary_fused"] == L
    assert cm.stats["residual_fused"] == 2 * L
    ids = torch.randint(0, m.config.vocab_size, (1, 64))
    with torch.no_grad():
        ref = m(ids).logits
    assert torch.allclose(cm(ids.int())[0], ref, atol=2e-5, rtol=1e-5)
    assert torch.allclose(p.reference(ids.int())[0], ref, atol=2e-5, rtol=1e-5)
    assert p.id_bound() == m.config.vocab_size


def test_llama_bf16_program_tracks_the_fp32_module(llama):
    m, _ = llama
    prog, w = llama_program(m, 64, dtype="bf16")
    cm = PG.parse(prog, w, gpu=True).compile("cpu")
    ids = torch.randint(0, m.config.vocab_size, (1, 64))
    with torch.no_grad():
        ref = m(ids).logits
    out = cm(ids.int())[0].float()
    assert (out - ref).abs().max() < 0.05 * ref.abs().max()


def test_export_refuses_what_a_program_cannot_express():
    class Same(nn.Module):
        def __init__(self):
            super().__init__()
            self.c = nn.Conv2d(8, 8, 3, padding="same")

        def forward(self, x):
            return self.c(x)

    with pytest.raises(ExportError, match="explicit padding"):
        export(Same(), torch.zeros(1, 8, 8, 8))

    class Odd(nn.Module):
        def __init__(self):
            super().__init__()
            self.e = nn.Embedding(10, 4)

        def forward(self, x):
            return self.e(x)

    with pytest.raises(ExportError, match="Embedding"):
        export(Odd(), torch.zeros(1, 3, dtype=torch.long))


@pytest.mark.parametrize("node,match", [
    ({"op": "conv2d", "inputs": ["x", "w4"], "output": "y", "attrs": {"groups": 2}}, "OC % groups"),
    ({"op": "softmax", "inputs": ["x"], "output": "y", "attrs": {"dim": 0}}, "last dim"),
    ({"op": "sdpa", "inputs": ["q32", "q32", "q32"], "output": "y"}, "head_dim 64 or 128"),
    ({"op": "embedding", "inputs": ["x", "w2"], "output": "y"}, "ids must be i32"),
    ({"op": "rotary", "inputs": ["q32", "w2", "w2"], "output": "y"}, "cos / sin"),
    ({"op": "matmul", "inputs": ["x", "w4"], "output": "y"}, r"\[\.\.\., M, K\]"),
])
def test_new_ops_are_validated_at_parse_time(node, match):
    b = PG.Builder("bad")
    b.input("x", [1, 4, 6, 6])
    b.param("w4", np.zeros((4, 4, 3, 3), np.float32))
    b.param("w2", np.zeros((4, 4), np.float32))
    b.param("q32", np.zeros((1, 8, 2, 32), np.float32))
    prog, w = b.build(["x"])
    prog["nodes"].append(node)
    prog["outputs"] = [node["output"]]
    with pytest.raises(PG.ProgramError, match=match):
        PG.parse(prog, w, gpu=True)


def test_one_pod_server_cohosts_yolos_a_conv_net_and_a_decoder(tmp_path, llama):
    """The MPS-client analogue beyond ViT encoders: three model families in
    one server process, each replying with its own module's outputs."""
    m, lprog = llama
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=2, memory_gb=40).start()
    try:
        clients = {}
        for name, prog in (("yolos", demo_tenant("fp32", 0, small=False)),
                           ("resnet", resnet_tenant("fp32", 0, small=False)), ("llama", lprog)):
            c = clients[name] = PodClient(srv.path, connect_timeout_s=5)
            rep = c.register(name, *prog, memory_limit_gb=2)
            assert rep["compile"]["kernels"] > 0
        assert len(srv.tenants) == 3
        x = np.random.default_rng(0).standard_normal((1, 3, 32, 32)).astype(np.float32)
        out, _ = clients["resnet"].infer(x, outputs=True)
        with torch.no_grad():
            ref = resnet_tiny(0)(torch.from_numpy(x)).numpy()
        np.testing.assert_allclose(out[0], ref, atol=1e-5, rtol=1e-5)
        ids = np.random.default_rng(1).integers(0, m.config.vocab_size, (1, 64)).astype(np.int32)
        out, _ = clients["llama"].infer(ids, outputs=True)
        with torch.no_grad():
            ref = m(torch.from_numpy(ids).long()).logits.numpy()
        np.testing.assert_allclose(out[0], ref, atol=2e-5, rtol=1e-5)
        with pytest.raises(PodServerError, match="token ids must lie"):
            clients["llama"].infer(np.full((1, 64), m.config.vocab_size, np.int32))
        clients["yolos"].infer()
        for c in clients.values():
            c.close()
    finally:
        srv.stop()


def test_estimate_counts_the_new_ops_workspaces(llama):
    _, (prog, w) = llama
    p = PG.parse(prog, w, gpu=True)
    q = copy.deepcopy(prog)
    for n in q["nodes"]:
        if n["op"] == "sdpa":
            n["op"], n["inputs"], n["attrs"] = "add", n["inputs"][:2], {}
    # same graph with the attention replaced by an elementwise op: the attention workspace is gone
    assert p.bytes_estimate > PG.parse(q, w).bytes_estimate


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_vit_patch_extraction_is_one_step_on_the_uncropped_image(dtype):
    """YOLOS at an input that is not a whole number of patches: the crop
    slice, the bf16 cast and the reshape / permute / reshape chain become one
    ``patches`` step that reads the original fp32 image (the kernel crops via
    strides and casts as it writes); outputs match the unfused reference."""
    from nos_amd.models.yolos import YolosConfig
    from nos_amd.models.yolos_program import yolos_program, yolos_weights

    cfg = YolosConfig.test()
    p = cfg.patch_size
    hw = (cfg.image_size[0] + p // 2, cfg.image_size[1] + 3)
    prog = PG.parse(*yolos_program(cfg, yolos_weights(cfg, 3), hw, dtype))
    m = prog.compile("cpu")
    assert m.stats["patchify_fused"] == 1
    first = [s for s in m.steps if s.kind == "patches"]
    assert len(first) == 1 and first[0].inputs == [m.input_name]
    assert first[0].attrs["hp"] == hw[0] // p and first[0].attrs["wp"] == hw[1] // p
    assert not any(s.kind in ("cast", "relayout") and s.inputs == [m.input_name] for s in m.steps)
    x = torch.from_numpy(np.random.default_rng(1).standard_normal((1, 3, *hw)).astype(np.float32))
    tol = dict(rtol=1e-4, atol=1e-5) if dtype == "fp32" else dict(rtol=0.1, atol=0.1)
    for o, r in zip(m(x), prog.reference(x)):
        np.testing.assert_allclose(o.float().numpy(), r.float().numpy(), **tol)


def test_bf16_heads_cast_and_sigmoid_are_one_step():
    """The bf16 YOLOS box head's cast to fp32 and sigmoid compile to one
    ``unary`` step (fp32 math, one rounding) matching the reference."""
    prog = PG.parse(*demo_tenant("bf16", 2, small=False))
    m = prog.compile("cpu")
    assert m.stats["cast_unary_fused"] == 1
    u = [s for s in m.steps if s.kind == "unary"]
    assert len(u) == 1 and u[0].attrs == {"op": "sigmoid", "dtype": "fp32"} and u[0].output == "pred_boxes"
    assert not any(s.kind in ("cast", "sigmoid") for s in m.steps)
    x = torch.from_numpy(np.random.default_rng(4).standard_normal(prog.inputs[0].shape).astype(np.float32))
    outs = m(x)
    assert outs[1].dtype == torch.float32
    for o, r in zip(outs, prog.reference(x)):
        np.testing.assert_allclose(o.float().numpy(), r.float().numpy(), rtol=0.1, atol=0.1)


def test_a_tenant_serves_several_input_shapes_over_one_weight_payload(tmp_path, llama):
    """Shape buckets: a decoder at sequence lengths 64 / 32 / 16 and a ViT at
    two image sizes register once each (one weight payload, one graph per
    shape); every request runs the variant its input shape names and matches
    the module at that shape; unknown shapes fail that request only."""
    from nos_amd.models.yolos import YolosConfig
    from nos_amd.models.yolos_program import yolos_program, yolos_weights

    m, (p64, w) = llama
    variants = [llama_program(m, s, rope_len=64) for s in (32, 16)]
    assert all(vw == w for _, vw in variants)
    cfg = YolosConfig.test()
    yw = yolos_weights(cfg, 5)
    y0, yp = yolos_program(cfg, yw, cfg.image_size)
    hw1 = (cfg.image_size[0] + 32, cfg.image_size[1] - 16)
    y1, yp1 = yolos_program(cfg, yw, hw1)
    assert yp1 == yp
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=2, memory_gb=40).start()
    try:
        lc = PodClient(srv.path, connect_timeout_s=5)
        rep = lc.register("llm", p64, w, memory_limit_gb=4, variants=[p for p, _ in variants])
        assert rep["input_shapes"] == [[1, 64], [1, 32], [1, 16]]
        for s in (16, 64, 32):
            ids = np.random.default_rng(s).integers(0, m.config.vocab_size, (1, s)).astype(np.int32)
            out, _ = lc.infer(ids, outputs=True)
            with torch.no_grad():
                ref = m(torch.from_numpy(ids).long()).logits.numpy()
            assert out[0].shape == ref.shape
            np.testing.assert_allclose(out[0], ref, atol=2e-5, rtol=1e-5)
        with pytest.raises(PodServerError, match="no program variant takes the input shape"):
            lc.infer(np.zeros((1, 48), np.int32))
        yc = PodClient(srv.path, connect_timeout_s=5)
        rep = yc.register("vit", y0, yp, memory_limit_gb=2, variants=[y1])
        assert rep["input_shapes"] == [[1, 3, *cfg.image_size], [1, 3, *hw1]]
        for shape, prog in (((1, 3, *hw1), y1), ((1, 3, *cfg.image_size), y0)):
            x = np.random.default_rng(7).standard_normal(shape).astype(np.float32)
            outs, _ = yc.infer(x, outputs=True)
            ref = PG.parse(prog, yp).reference(torch.from_numpy(x))
            for o, r in zip(outs, ref):
                np.testing.assert_allclose(o, r.numpy(), rtol=1e-4, atol=1e-5)
        lc.infer()   # no input: the primary shape's resident input
        lc.close()
        yc.close()
    finally:
        srv.stop()


def test_variants_must_share_their_weights():
    from nos_amd.models.yolos import YolosConfig
    from nos_amd.models.yolos_program import yolos_program, yolos_weights

    cfg = YolosConfig.test()
    y0, yp = yolos_program(cfg, yolos_weights(cfg, 5), cfg.image_size)
    with pytest.raises(PG.ProgramError, match="two variants take the input shape"):
        PG.parse_variants([y0, y0], yp)
    other = copy.deepcopy(y0)
    other["inputs"][0]["shape"] = [1, 3, 64, 64]
    other["params"][0]["shape"] = [1] + other["params"][0]["shape"][1:]
    with pytest.raises(PG.ProgramError):
        PG.parse_variants([y0, other], yp)
    with pytest.raises(PG.ProgramError, match="1 to 8 program variants"):
        PG.parse_variants([y0] * 9, yp)


def test_compiled_program_drops_the_derived_weight_memo():
    """The memo of derived weights (shared by a tenant's shape variants during
    the build) holds the source tensors; a compiled program must not keep it,
    or every raw weight a fold replaced stays allocated (GPU footprint)."""
    import weakref

    import torch

    from nos_amd.podserver import program as PG

    b = PG.Builder("bnfold")
    x = b.input("x", [1, 8, 6, 6])
    w = b.param("w", np.random.default_rng(0).standard_normal((4, 8, 3, 3)) * 0.1)
    h = b.op("conv2d", x, w, padding=[1, 1])
    h = b.op("batchnorm", h, b.param("g", np.ones(4)), b.param("be", np.zeros(4)), b.param("mu", np.zeros(4)),
             b.param("var", np.ones(4)), eps=1e-5)
    prog, wts = b.build([h])
    p = PG.parse(prog, wts)
    params = p.tensors("cpu")
    raw = weakref.ref(params["w"])
    derived: dict = {}
    c = p.compile("cpu", params=params, derived=derived)
    assert c._derived is None and derived
    del params, derived
    import gc

    gc.collect()
    assert raw() is None, "the raw conv weight outlived the build"
    assert torch.is_tensor(c(p.input_tensor("cpu"))[0])
