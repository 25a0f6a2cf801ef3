"""The pod server on the MI355X: tenants ship programs (op graph + weights)
whose inferences run as HIP-graph replays on the server's lanes.  Checks that
a YOLOS-small fp32 program's results are bit-identical to YolosDetector run
eagerly with the same weights and kernels, that two architectures (YOLOS +
the bf16 GEMM-MLP probe) co-hosted each match their own eager output, that
memory admission refuses a tenant that exceeds its slice, and that more
clients than lanes all make progress.  The server runs inside the test
process; its clients are threads with sockets and never touch the GPU."""
from __future__ import annotations

import threading
import time

import numpy as np
import pytest
import torch

from nos_amd import ops

pytestmark = pytest.mark.gpu


def _yolos(seed: int, dtype: str = "fp32"):
    from nos_amd.models.yolos_program import demo_tenant

    return demo_tenant(dtype, seed, small=True)


@pytest.fixture
def server(tmp_path):
    from nos_amd.ops import _lib
    from nos_amd.podserver.server import PodServer

    _lib.require_native_on_gpu()
    srv = PodServer(tmp_path / "gpu-0" / "server.sock", device="cuda", lanes=2, max_tenants=8).start()
    yield srv
    srv.stop()
    # the server set process-wide kernel configs: back to the library defaults
    ops.set_gemm_policy("throughput")
    ops.set_gemm_f32_policy("latency")
    ops.set_attention_f32_variant("auto")
    ops.set_f32_math("exact")
    ops.set_gemm_f32x6_tile("policy")


def test_server_replays_match_the_eager_model(server):
    from nos_amd.models.yolos import YolosConfig, YolosDetector
    from nos_amd.models.yolos_program import yolos_weights
    from nos_amd.podserver.client import PodClient

    c = PodClient(server.path, connect_timeout_s=10)
    rep = c.register("pod-a", *_yolos(3), memory_limit_gb=10)
    assert rep["server"]["kernel_config"]["f32_math"] == "h3"
    assert rep["compile"]["qkv_attention_fused"] == 12 and rep["compile"]["layernorm_folded"] == 25
    # the heads' first GEMMs (both ReLU) merge into one, ReLU fused, the final LN folded into it
    assert rep["compile"]["linears_merged"] == 2
    # ... and their second / third layers into block-diagonal GEMMs (2 + 2)
    assert rep["compile"]["linears_blockdiag_merged"] == 4
    assert rep["compile"]["plane_handoffs"] == 25
    assert 0.05 < rep["footprint_gb"] < 10
    x = np.random.default_rng(1).standard_normal(rep["input_shape"]).astype(np.float32)
    outs, meta = c.infer(x, outputs=True)
    assert meta["gpu_us"] > 0
    # a lone tenant replays its solo graph: the eager reference runs under the
    # same (whole-GPU) configs, which are process-wide
    assert next(iter(server.tenants.values())).solo_completed == 1
    cfg = YolosConfig.small()
    m = YolosDetector(cfg)
    m.load_numpy(yolos_weights(cfg, 3))
    m = m.cuda().eval()
    server._apply_config(server.solo_config)
    try:
        with torch.no_grad():
            ref = m(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
    finally:
        server._apply_config(server.kernel_config)
    # the encoder runs the same kernels in the same order; the last layer only on
    # the 100 detection tokens (row-slice pushdown: its attention may then split
    # the keys differently), so fp32-class agreement rather than bit equality
    assert rep["compile"]["row_slices_pushed"] >= 8
    for o, r in zip(outs, ref):
        r = r.float().cpu().numpy()
        assert np.abs(o - r).max() <= 1e-5 * (np.abs(r).max() + 1)
    c.close()


def test_two_architectures_cohosted_each_match_their_eager_output(server):
    """YOLOS-small fp32 and the bf16 GEMM-MLP probe tenant in one server:
    each tenant's replayed outputs equal its own program run eagerly (same
    kernels, same configs) bit for bit."""
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.client import PodClient

    yolos, mlp = _yolos(4), PG.mlp_program(dim=1024, layers=4, batch=256, dtype="bf16", seed=5)
    a, b = PodClient(server.path, connect_timeout_s=10), PodClient(server.path, connect_timeout_s=10)
    ra = a.register("yolos", *yolos, memory_limit_gb=10)
    rb = b.register("mlp", *mlp, memory_limit_gb=2)
    assert rb["compile"]["layernorm_folded"] == 4 and rb["compile"]["residual_fused"] == 4
    rng = np.random.default_rng(6)
    xa = rng.standard_normal(ra["input_shape"]).astype(np.float32)
    xb = rng.standard_normal(rb["input_shape"]).astype(np.float32)
    oa, _ = a.infer(xa, outputs=True)  # one at a time: each replays its solo graph
    ob, _ = b.infer(xb, outputs=True)
    server._apply_config(server.solo_config)
    try:
        with torch.no_grad():
            for (prog, w), x, o in ((yolos, xa, oa), (mlp, xb, ob)):
                P = PG.parse(prog, w, gpu=True)
                ref = P.compile("cuda")(P.input_tensor("cuda", x))
                torch.cuda.synchronize()
                for oo, r in zip(o, ref):
                    assert np.array_equal(oo, r.float().cpu().numpy())
                # and near the unfused fp32 reference (bf16: per-op rounding)
                eag = P.reference(torch.from_numpy(x))
                err = np.abs(o[0] - eag[0].numpy()).max() / np.abs(eag[0].numpy()).max()
                assert err < (3e-2 if "mlp" in P.name else 1e-4), (P.name, err)
    finally:
        server._apply_config(server.kernel_config)
    # concurrent load: a request may replay the co-tenancy graph (other kernel
    # configs: sums in another order), so within fp32 accuracy of the solo run
    res, stop = [], threading.Event()

    def hammer():
        while not stop.is_set():
            b.infer()

    th = threading.Thread(target=hammer)
    th.start()
    try:
        for _ in range(4):
            res.append(a.infer(xa, outputs=True)[0][0])
    finally:
        stop.set()
        th.join(timeout=30)
    for r in res:
        assert np.abs(r - oa[0]).max() <= 1e-4 * (np.abs(oa[0]).max() + 1e-6)
    a.close()
    b.close()


def test_a_tenant_larger_than_its_slice_is_refused(server):
    from nos_amd.podserver.client import PodClient, PodServerError

    c = PodClient(server.path, connect_timeout_s=10)
    prog = _yolos(0)
    # weights (~0.09 GB) larger than the slice: refused before they are read
    with pytest.raises(PodServerError, match="PayloadTooLarge"):
        c.register("tiny-slice", *prog, memory_limit_gb=0.05)
    with pytest.raises(PodServerError, match="slice has 0.2 GB"):  # the static estimate
        c.register("tiny-slice", *prog, memory_limit_gb=0.2)
    # past the estimate, the measured peak of the build decides: an estimate
    # of 0 lets the build run, and the real footprint (~0.47 GB) refuses it
    import nos_amd.podserver.program as PG

    orig = PG.Program.bytes_estimate
    try:
        PG.Program.bytes_estimate = property(lambda self: 0)
        with pytest.raises(PodServerError, match="slice has 0.2 GB"):
            c.register("tiny-slice", *prog, memory_limit_gb=0.2)
    finally:
        PG.Program.bytes_estimate = orig
    assert not server.tenants and server.stats()["pending"] == 0
    c.register("ok", *prog, memory_limit_gb=10)  # the refused build left nothing behind
    c.infer()
    c.close()


def test_more_clients_than_lanes_all_progress(server):
    from nos_amd.podserver.client import PodClient

    n = 5
    clients = [PodClient(server.path, connect_timeout_s=10) for _ in range(n)]
    for i, c in enumerate(clients):
        c.register(f"p{i}", *_yolos(i), memory_limit_gb=10)
    counts, stop = [0] * n, threading.Event()

    def loop(i):
        while not stop.is_set():
            clients[i].infer()
            counts[i] += 1

    th = [threading.Thread(target=loop, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    time.sleep(3.0)
    stop.set()
    for t in th:
        t.join(timeout=30)
    assert min(counts) > 10, counts
    assert max(counts) <= 1.5 * min(counts) + 2, counts  # FIFO service: equal shares
    for c in clients:
        c.close()


def test_a_lone_tenant_replays_its_solo_graph_with_the_same_results(server):
    """A tenant alone on the GPU replays the graph captured under the whole-GPU
    configs (key splits, latency tiles); its outputs stay within fp32
    accuracy of the co-tenancy graph's (a key split only reorders the sums)."""
    from nos_amd.podserver.client import PodClient

    assert server.solo_config is not None and server.solo_config != server.kernel_config
    c = PodClient(server.path, connect_timeout_s=10)
    rep = c.register("solo", *_yolos(5), memory_limit_gb=10)
    x = np.random.default_rng(2).standard_normal(rep["input_shape"]).astype(np.float32)
    outs, _ = c.infer(x, outputs=True)
    t = next(iter(server.tenants.values()))
    assert t.solo_graph is not None and t.solo_completed == 1
    # the co-tenancy graph on the same input, replayed directly
    with torch.no_grad(), torch.cuda.stream(server._setup_stream):
        t.graph.replay()
    server._setup_stream.synchronize()
    for o, r in zip(outs, t.outputs):
        r = r.float().cpu().numpy()
        assert np.abs(o - r).max() <= 1e-4 * (np.abs(r).max() + 1e-6)
    c.close()


def test_both_graphs_follow_every_new_input(server):
    """Each replay of a tenant's co-tenancy and solo graphs computes on the
    input just written, bit-identical to the eager program under the same
    configs, input after input (regression: a memset node in the captured
    graph made replays return an earlier input's outputs,
    profiles/r04_graph_memset_staleness.json)."""
    from nos_amd.podserver import program as PG

    prog = _yolos(6)
    t = server._build(99, {"pod": "g"}, PG.parse(*prog, gpu=True), 10.0, None)
    try:
        rng = np.random.default_rng(9)
        s = server._lanes[0]
        for _ in range(3):
            x = torch.from_numpy(rng.standard_normal(tuple(t.x.shape)).astype(np.float32))
            for graph, outs, cfg in ((t.graph, t.outputs, server.kernel_config),
                                     (t.solo_graph, t.solo_outputs, server.solo_config)):
                with torch.no_grad(), torch.cuda.stream(s):
                    t.x.copy_(x.view(t.x.shape).to(t.x.dtype))  # the server's _run: copy, then replay
                    graph.replay()
                s.synchronize()
                server._apply_config(cfg)
                try:
                    with torch.no_grad():
                        ref = t.model(t.x)
                    torch.cuda.synchronize()
                finally:
                    server._apply_config(server.kernel_config)
                for o, r in zip(outs, ref):
                    assert torch.equal(o, r)
    finally:
        server._free(t)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_a_torch_transformer_encoder_tenant(server, dtype):
    """A third architecture: a tenant's own ``nn.TransformerEncoder``
    (pre-LN, GELU) shipped as a program, against the same module run by
    PyTorch in fp32 on the CPU (on the GPU, PyTorch's fused encoder fast path
    is itself only ~1e-4 accurate)."""
    from nos_amd.models.encoder_program import encoder_program, random_encoder_weights
    from nos_amd.podserver.client import PodClient

    L, hid, heads, mlp, S = 2, 256, 4, 1024, 200
    w = random_encoder_weights(L, hid, mlp, seed=8)
    layer = torch.nn.TransformerEncoderLayer(hid, heads, mlp, dropout=0.0, activation="gelu", batch_first=True,
                                             norm_first=True)
    enc = torch.nn.TransformerEncoder(layer, L, norm=torch.nn.LayerNorm(hid), enable_nested_tensor=False)
    enc.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()})
    enc = enc.eval()
    c = PodClient(server.path, connect_timeout_s=10)
    rep = c.register("enc", *encoder_program(w, L, heads, (2, S, hid), dtype), memory_limit_gb=2)
    assert rep["compile"]["qkv_attention_fused"] == L
    x = np.random.default_rng(5).standard_normal(rep["input_shape"]).astype(np.float32)
    out, _ = c.infer(x, outputs=True)
    with torch.no_grad():
        ref = enc(torch.from_numpy(x)).numpy()
    err = np.abs(out[0] - ref).max() / np.abs(ref).max()
    assert err < (1e-4 if dtype == "fp32" else 3e-2), err
    c.close()
