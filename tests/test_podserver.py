"""Pod server (nos_amd/podserver, the MPS analogue) on the CPU: wire protocol,
tenant admission (server capacity, memory slices), result parity with running
the model in the pod itself, fair service of concurrent clients, tenant
cleanup on disconnect, and the control-plane path that hands pods a
pod-server slice (device plugin env, no device nodes; slice count per GPU
bounded by the server's tenants, not the HWS process slots).  GPU runs of the
same server: tests/test_podserver_gpu.py."""
from __future__ import annotations

import socket
import threading
import time

import numpy as np
import pytest
import torch

from nos_amd.api import constants as C
from nos_amd.podserver import protocol as P
from nos_amd.podserver.client import PodClient, PodServerError
from nos_amd.podserver.server import PodServer


@pytest.fixture
def server(tmp_path):
    srv = PodServer(tmp_path / "gpu-0.sock", device="cpu", lanes=2, max_tenants=3, memory_gb=30).start()
    yield srv
    srv.stop()


def test_protocol_round_trips_json_and_arrays():
    a, b = socket.socketpair()
    arrs = [np.arange(6, dtype=np.float32).reshape(2, 3), np.ones((1, 4), np.float32)]
    descs, payload = P.pack_arrays(arrs)
    P.send_msg(a, {"op": "x", "outputs": descs}, payload)
    obj, data = P.recv_msg(b)
    back = P.unpack_arrays(obj["outputs"], data)
    assert obj["op"] == "x" and all(np.array_equal(x, y) for x, y in zip(arrs, back))
    a.close()
    with pytest.raises(ConnectionError):
        P.recv_msg(b)
    b.close()


def test_outputs_match_the_model_run_in_the_pod_itself(server):
    from nos_amd.models.pod import _build
    from nos_amd.models.yolos import demo_input_hw

    c = PodClient(server.path, connect_timeout_s=5)
    rep = c.register("pod-a", seed=7, memory_limit_gb=10)
    assert rep["tenant"] >= 1 and rep["server"]["lanes"] == 2
    x = np.random.default_rng(0).standard_normal(rep["input_shape"]).astype(np.float32)
    outs, meta = c.infer(x, outputs=True)
    m, _ = _build("fp32", 7, demo_input_hw(), "cpu")
    with torch.no_grad():
        ref = m(torch.from_numpy(x))
    assert len(outs) == len(ref)
    for o, r in zip(outs, ref):
        np.testing.assert_array_equal(o, r.numpy())
    # the resident input stays: a request without an input reuses it
    outs2, _ = c.infer(outputs=True)
    np.testing.assert_array_equal(outs2[0], outs[0])
    assert meta["queue_us"] >= 0 and meta["gpu_us"] > 0
    c.close()


def test_admission_bounds_tenants_and_slice_memory(server):
    cs = [PodClient(server.path, connect_timeout_s=5) for _ in range(4)]
    for i in range(2):
        cs[i].register(f"p{i}", memory_limit_gb=10)
    with pytest.raises(PodServerError, match="does not fit"):  # 10 + 10 + 20 > 30 GB
        cs[2].register("big", memory_limit_gb=20)
    cs[2].register("p2", memory_limit_gb=10)
    with pytest.raises(PodServerError, match="server full"):
        cs[3].register("p3", memory_limit_gb=1)
    with pytest.raises(PodServerError, match="register first"):
        cs[3].infer()
    cs[0].close()  # a departing tenant frees its place
    deadline = time.monotonic() + 5
    while len(server.tenants) > 2 and time.monotonic() < deadline:
        time.sleep(0.01)
    cs[3].register("p3", memory_limit_gb=1)
    assert sorted(t.pod for t in server.tenants.values()) == ["p1", "p2", "p3"]
    for c in cs[1:]:
        c.close()


def test_disconnect_without_close_unregisters_the_tenant(server):
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("gone")
    c.infer()
    c.sock.close()  # the pod was killed
    c.sock = None
    deadline = time.monotonic() + 5
    while server.tenants and time.monotonic() < deadline:
        time.sleep(0.01)
    assert not server.tenants


def test_wrong_input_size_fails_only_that_request(server):
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("a")
    with pytest.raises(PodServerError, match="input has 3 values"):
        c.infer(np.zeros(3, np.float32))
    c.infer()  # the tenant still works
    c.close()


def test_concurrent_clients_are_served_fairly(server):
    """More clients than lanes, each back to back: the FIFO gives every tenant
    the same share (within one request of each other per round)."""
    n, stop = 3, threading.Event()
    counts = [0] * n
    clients = [PodClient(server.path, connect_timeout_s=5) for _ in range(n)]
    for i, c in enumerate(clients):
        c.register(f"p{i}", seed=i)

    def loop(i):
        while not stop.is_set():
            clients[i].infer()
            counts[i] += 1

    th = [threading.Thread(target=loop, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    time.sleep(2.0)
    stop.set()
    for t in th:
        t.join()
    assert min(counts) > 0
    assert max(counts) - min(counts) <= max(2, 0.25 * max(counts)), counts
    st = clients[0].stats()
    assert sorted(t["completed"] for t in st["tenants"]) == sorted(counts)
    for c in clients:
        c.close()


def test_client_reports_a_missing_server(tmp_path):
    with pytest.raises(PodServerError, match="no pod server"):
        PodClient(tmp_path / "none.sock", connect_timeout_s=0.3)
    with pytest.raises(PodServerError, match="NOS_AMD_POD_SERVER"):
        PodClient.from_env({})


def test_client_side_never_imports_torch():
    import subprocess
    import sys

    code = ("import sys; import nos_amd.podserver.client, nos_amd.podserver.protocol, nos_amd.models.pod; "
            "print('torch' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "False"


# ----------------------------------------------------------------- control plane
def test_device_plugin_allocates_pod_server_slices_without_device_nodes():
    from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
    from nos_amd.gpu.fakesmi import FakeSmi

    p = NosAmdDevicePlugin("n1", FakeSmi(gpus=2, node="n1"), mode=C.PARTITIONING_CUMASK, cu_policy="shared",
                           pod_server_dir="/run/nos-amd/podserver")
    p.set_config("n1-1", {"gpus": [{"index": 1, "slices": [{"profile": "10gb", "replicas": 3}]}]})
    devs = p.list_devices("amd.com/gpu-10gb")
    assert len(devs) == 3
    a = p.allocate("amd.com/gpu-10gb", [devs[0].id])
    assert a.envs == {C.ENV_POD_SERVER: "/run/nos-amd/podserver/gpu-1.sock", C.ENV_MEMORY_LIMIT_GB: "10"}
    assert a.devices == [] and a.mounts == ["/run/nos-amd/podserver"]
    # a proportional CU policy hands the tenant's CU mask to the server, not to HIP
    q = NosAmdDevicePlugin("n1", FakeSmi(gpus=1, node="n1"), mode=C.PARTITIONING_CUMASK, cu_policy="even",
                           pod_server_dir="/run/ps")
    q.set_config("n1-1", {"gpus": [{"index": 0, "slices": [{"profile": "10gb", "replicas": 4}]}]})
    b = q.allocate("amd.com/gpu-10gb", [q.list_devices("amd.com/gpu-10gb")[0].id])
    assert C.ENV_POD_CU_MASK in b.envs and C.ENV_CU_MASK not in b.envs
    assert bin(int(b.envs[C.ENV_POD_CU_MASK], 16)).count("1") == 64


def test_pod_server_node_schedules_slices_by_memory_not_hws_slots():
    from nos_amd.bench_support import control_plane_plan, schedulable_pods

    # 10 GB slices on one 288 GB MI355X: 8 GPU processes (HWS) vs 28 server tenants (memory)
    assert schedulable_pods(1, 10)["schedulable_fractional_pods_per_node"] == 8
    assert schedulable_pods(1, 10, pod_server_tenants=48)["schedulable_fractional_pods_per_node"] == 28
    # ... and the server's tenant count bounds it when memory does not
    assert schedulable_pods(1, 5, pod_server_tenants=16)["schedulable_fractional_pods_per_node"] == 16
    _, info = control_plane_plan(2, 28, 10, 256, local_gpu=1, cu_policy="shared", capacity_probe=False,
                                 pod_server_tenants=48, pod_server_dir="/tmp/psx")
    assert info["placed_pods"] == 56 and info["pending_pods"] == 0
    assert len(info["envs"]) == 28
    assert all(e[C.ENV_POD_SERVER] == "/tmp/psx/gpu-1.sock" and C.ENV_VISIBLE_DEVICES not in e
               for e in info["envs"])


def test_podserver_binary_supervises_one_server_per_gpu(tmp_path):
    """``nos_amd.cmd.podserver --gpus 0,1`` (the DaemonSet entry point): one
    server per GPU at <socket-dir>/gpu-<i>.sock, stopped by SIGTERM."""
    import os
    import signal
    import subprocess
    import sys

    from nos_amd.cmd.podserver import socket_path

    env = {**os.environ, "OMP_NUM_THREADS": "1"}
    p = subprocess.Popen([sys.executable, "-m", "nos_amd.cmd.podserver", "--gpus", "0,1", "--device", "cpu",
                          "--socket-dir", str(tmp_path), "--lanes", "1"], env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        for g in (0, 1):
            c = PodClient(socket_path(tmp_path, g), connect_timeout_s=60)
            c.register(f"p{g}")
            c.infer()
            assert c.stats()["server"]["device"] == "cpu"
            c.close()
    finally:
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 0


def test_manifests_render_the_pod_server_and_its_configs():
    import yaml

    from nos_amd.api import config as cfgmod
    from nos_amd.cmd import manifests as m

    out = m.render(m.apply_set(m.merge_values(m.DEFAULT_VALUES, {}), "gpuPartitioner.podServer.enabled=true"))
    ds = [o for o in yaml.safe_load_all(out["podserver/daemonset.yaml"]) if o and o["kind"] == "DaemonSet"][0]
    spec = ds["spec"]["template"]["spec"]
    assert spec["nodeSelector"] == {C.LABEL_GPU_PARTITIONING: C.PARTITIONING_CUMASK}
    assert spec["containers"][0]["args"][:2] == ["--gpus", "all"]

    def embedded(key, fname):
        cm = [o for o in yaml.safe_load_all(out[key]) if o and o["kind"] == "ConfigMap"][0]
        return cfgmod.parse(yaml.safe_load(cm["data"][fname]))

    assert embedded("gpuagent/daemonset.yaml", "gpu_agent_config.yaml").pod_server_tenants == 48
    assert embedded("deviceplugin/daemonset.yaml", "device_plugin_config.yaml").pod_server_socket_dir == \
        C.DEFAULT_POD_SERVER_SOCKET_DIR
    with pytest.raises(ValueError, match="lanes"):
        m.render(m.apply_set(m.merge_values(m.DEFAULT_VALUES, {"gpuPartitioner": {"podServer": {
            "enabled": True, "lanes": 64}}}), "namespace=nos-system"))


def test_server_exports_prometheus_metrics(server):
    from nos_amd.observability import metrics as M

    c = PodClient(server.path, connect_timeout_s=5)
    c.register("metered")
    for _ in range(3):
        c.infer()
    text = M.exposition().decode()
    assert 'nos_podserver_tenants{gpu="cpu"} 1.0' in text
    assert 'nos_podserver_inferences_total{gpu="cpu",pod="metered"} 3.0' in text
    assert "nos_podserver_request_seconds_count" in text
    c.close()
    deadline = time.monotonic() + 5
    while server.tenants and time.monotonic() < deadline:
        time.sleep(0.01)
    text = M.exposition().decode()
    assert 'pod="metered"' not in text and 'nos_podserver_tenants{gpu="cpu"} 0.0' in text


def test_lanes_know_when_a_tenant_runs_alone(server, monkeypatch):
    """The lane passes ``alone`` (no other job running or queued) to the run:
    a lone client always runs alone (its solo graph on a GPU); clients that
    keep the lanes busy mostly do not.  stop() leaves no tenant behind."""
    seen: list[bool] = []
    orig = server._run

    def spy(job, lane, alone=False):
        seen.append(alone)
        time.sleep(0.01)  # long enough for co-tenants' jobs to overlap
        return orig(job, lane, alone)

    monkeypatch.setattr(server, "_run", spy)
    c = PodClient(server.path, connect_timeout_s=5)
    c.register("solo")
    for _ in range(5):
        c.infer()
    assert seen == [True] * 5
    seen.clear()
    others = [PodClient(server.path, connect_timeout_s=5) for _ in range(2)]
    for i, o in enumerate(others):
        o.register(f"co{i}")
    stop = threading.Event()

    def loop(cl):
        while not stop.is_set():
            cl.infer()

    th = [threading.Thread(target=loop, args=(cl,)) for cl in [c, *others]]
    for t in th:
        t.start()
    time.sleep(1.0)
    stop.set()
    for t in th:
        t.join()
    assert seen.count(False) > len(seen) // 2, seen.count(False)
    assert server._busy == 0
    server.stop()
    assert server.tenants == {}
