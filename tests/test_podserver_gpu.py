"""The pod server on the MI355X: tenants' YOLOS-small fp32 inferences run as
HIP-graph replays on the server's lanes.  Checks that the server's results are
bit-identical to the same model run eagerly with the same kernels, that its
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


@pytest.fixture
def server(tmp_path):
    from nos_amd.ops import _lib
    from nos_amd.podserver.server import PodServer

    _lib.require_native_on_gpu()
    srv = PodServer(tmp_path / "gpu-0.sock", device="cuda", lanes=2, max_tenants=8).start()
    yield srv
    srv.stop()
    # the server set process-wide kernel configs: back to the library defaults
    ops.set_gemm_policy("throughput")
    ops.set_gemm_f32_policy("latency")
    ops.set_attention_f32_variant("auto")
    ops.set_f32_math("exact")
    ops.set_gemm_f32x6_tile("policy")


def test_server_replays_match_the_eager_model_bit_for_bit(server):
    from nos_amd.models.pod import _build
    from nos_amd.models.yolos import demo_input_hw
    from nos_amd.podserver.client import PodClient

    c = PodClient(server.path, connect_timeout_s=10)
    rep = c.register("pod-a", seed=3, memory_limit_gb=10)
    assert rep["server"]["kernel_config"]["f32_math"] == "x6"
    assert 0.05 < rep["footprint_gb"] < 10
    x = np.random.default_rng(1).standard_normal(rep["input_shape"]).astype(np.float32)
    outs, meta = c.infer(x, outputs=True)
    assert meta["gpu_us"] > 0
    # a lone tenant replays its solo graph: the eager reference runs under the
    # same (whole-GPU) configs, which are process-wide
    assert next(iter(server.tenants.values())).solo_completed == 1
    m, _ = _build("fp32", 3, demo_input_hw(), "cuda")
    server._apply_config(server.solo_config)
    try:
        with torch.no_grad():
            ref = m(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
    finally:
        server._apply_config(server.kernel_config)
    for o, r in zip(outs, ref):
        assert np.array_equal(o, r.float().cpu().numpy())
    c.close()


def test_a_tenant_larger_than_its_slice_is_refused(server):
    from nos_amd.podserver.client import PodClient, PodServerError

    c = PodClient(server.path, connect_timeout_s=10)
    with pytest.raises(PodServerError, match="slice has 0.05 GB"):
        c.register("tiny-slice", memory_limit_gb=0.05)
    assert not server.tenants
    c.register("ok", memory_limit_gb=10)  # the refused build left nothing behind
    c.infer()
    c.close()


def test_more_clients_than_lanes_all_progress(server):
    from nos_amd.podserver.client import PodClient

    n = 5
    clients = [PodClient(server.path, connect_timeout_s=10) for _ in range(n)]
    for i, c in enumerate(clients):
        c.register(f"p{i}", seed=i, memory_limit_gb=10)
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
    rep = c.register("solo", seed=5, memory_limit_gb=10)
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
