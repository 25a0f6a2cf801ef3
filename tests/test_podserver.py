"""Pod server (nos_amd/podserver, the MPS analogue) on the CPU: wire protocol,
tenant programs (op graph + weights) of two architectures co-hosted and
matching each tenant's own eager output, tenant admission (server capacity,
memory slices, reservation before the build), fair service of concurrent
clients, tenant cleanup on disconnect, and the control-plane path that hands
pods a pod-server slice (device plugin env + allocation token, no device
nodes; slice count per GPU bounded by the server's tenants, not the HWS
process slots).  Allocation tokens, eviction and server crashes:
tests/test_podserver_admission.py.  GPU runs: tests/test_podserver_gpu.py."""
from __future__ import annotations

import socket
import threading
import time

import numpy as np
import pytest
import torch

from nos_amd.api import constants as C
from nos_amd.models.yolos_program import demo_tenant
from nos_amd.podserver import program as PG
from nos_amd.podserver import protocol as P
from nos_amd.podserver.client import PodClient, PodServerError
from nos_amd.podserver.server import PodServer

YOLOS = demo_tenant("fp32", 0, small=False)  # the tiny YOLOS test config (program, weights)


def reg(c: PodClient, pod: str, limit: float = 10, seed: int = 0, prog=None):
    p, w = prog or (YOLOS if seed == 0 else demo_tenant("fp32", seed, small=False))
    return c.register(pod, p, w, memory_limit_gb=limit)


@pytest.fixture
def server(tmp_path):
    srv = PodServer(tmp_path / "gpu-0" / "server.sock", device="cpu", lanes=2, max_tenants=3, memory_gb=30).start()
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


def test_outputs_match_the_tenants_own_eager_model(server):
    """A YOLOS program runs in the server and returns what the same weights
    give in YolosDetector and in the program's own unfused eager reference."""
    from nos_amd.models.yolos import YolosConfig, YolosDetector
    from nos_amd.models.yolos_program import yolos_weights

    c = PodClient(server.path, connect_timeout_s=5)
    prog = demo_tenant("fp32", 7, small=False)
    rep = reg(c, "pod-a", prog=prog)
    assert rep["tenant"] >= 1 and rep["server"]["lanes"] == 2 and rep["program"].startswith("yolos")
    # the graph compiler folded the LNs into the GEMMs (the final one into the
    # two detection heads' merged first GEMM) and fused QKV + attention
    assert rep["compile"]["layernorm_folded"] == 5 and rep["compile"]["qkv_attention_fused"] == 2
    assert rep["compile"]["plane_handoffs"] == 5 and rep["compile"]["linears_merged"] == 2
    # the heads' second and third layers: one block-diagonal GEMM per level
    assert rep["compile"]["linears_blockdiag_merged"] == 4
    # (+1 residual: the position embeddings, distributed over the token cat, into the patch GEMM)
    assert rep["compile"]["residual_fused"] == 5 and rep["compile"]["activation_fused"] == 4
    assert rep["compile"]["adds_distributed"] == 1
    x = np.random.default_rng(0).standard_normal(rep["input_shape"]).astype(np.float32)
    outs, meta = c.infer(x, outputs=True)
    m = YolosDetector(YolosConfig.test(), backend="torch")
    m.load_numpy(yolos_weights(YolosConfig.test(), 7))
    with torch.no_grad():
        ref = m(torch.from_numpy(x))
    eager = PG.parse(*prog).reference(torch.from_numpy(x))
    assert len(outs) == len(ref) == 2
    for o, r, e in zip(outs, ref, eager):
        np.testing.assert_allclose(o, r.numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(o, e.numpy(), rtol=1e-4, atol=1e-6)
    # the resident input stays: a request without an input reuses it
    outs2, _ = c.infer(outputs=True)
    np.testing.assert_array_equal(outs2[0], outs[0])
    assert meta["queue_us"] >= 0 and meta["gpu_us"] > 0
    c.close()


def test_two_architectures_share_a_server_and_each_matches_its_eager_output(server):
    """YOLOS (fp32) and the GEMM-MLP probe tenant (bf16, BASELINE config 4's
    workload) co-hosted, interleaved requests."""
    a, b = PodClient(server.path, connect_timeout_s=5), PodClient(server.path, connect_timeout_s=5)
    mlp = PG.mlp_program(dim=128, layers=2, batch=32, dtype="bf16", seed=3)
    ra = reg(a, "yolos", prog=YOLOS)
    rb = b.register("mlp", *mlp, memory_limit_gb=1)
    assert ra["program"] != rb["program"] and rb["compile"]["layernorm_folded"] == 2
    rng = np.random.default_rng(4)
    for _ in range(2):
        xa = rng.standard_normal(ra["input_shape"]).astype(np.float32)
        xb = rng.standard_normal(rb["input_shape"]).astype(np.float32)
        ob, _ = b.infer(xb, outputs=True)
        oa, _ = a.infer(xa, outputs=True)
        ea = PG.parse(*YOLOS).reference(torch.from_numpy(xa))
        eb = PG.parse(*mlp).reference(torch.from_numpy(xb))
        np.testing.assert_allclose(oa[0], ea[0].numpy(), rtol=1e-4, atol=1e-6)
        # bf16 activations against the fp32 reference: bf16 rounding per op
        err = np.abs(ob[0] - eb[0].numpy()).max() / np.abs(eb[0].numpy()).max()
        assert ob[0].shape == (32, 128) and err < 3e-2, err
    st = a.stats()
    assert sorted(t["program"] for t in st["tenants"]) == sorted([ra["program"], rb["program"]])
    a.close()
    b.close()


def test_admission_bounds_tenants_and_slice_memory(server):
    cs = [PodClient(server.path, connect_timeout_s=5) for _ in range(4)]
    with pytest.raises(PodServerError, match="memory slice"):  # no slice: refused, not unaccounted
        reg(cs[0], "p0", limit=0)
    for i in range(2):
        reg(cs[i], f"p{i}", limit=10)
    with pytest.raises(PodServerError, match="does not fit"):  # 10 + 10 + 20 > 30 GB
        reg(cs[2], "big", limit=20)
    reg(cs[2], "p2", limit=10)
    with pytest.raises(PodServerError, match="server full"):
        reg(cs[3], "p3", limit=1)
    with pytest.raises(PodServerError, match="register first"):
        cs[3].infer()
    cs[0].close()  # a departing tenant frees its place
    deadline = time.monotonic() + 5
    while len(server.tenants) > 2 and time.monotonic() < deadline:
        time.sleep(0.01)
    reg(cs[3], "p3", limit=1)
    assert sorted(t.pod for t in server.tenants.values()) == ["p1", "p2", "p3"]
    for c in cs[1:]:
        c.close()


def test_disconnect_without_close_unregisters_the_tenant(server):
    c = PodClient(server.path, connect_timeout_s=5)
    reg(c, "gone")
    c.infer()
    c.sock.close()  # the pod was killed
    c.sock = None
    deadline = time.monotonic() + 5
    while server.tenants and time.monotonic() < deadline:
        time.sleep(0.01)
    assert not server.tenants


def test_wrong_input_size_fails_only_that_request(server):
    c = PodClient(server.path, connect_timeout_s=5)
    reg(c, "a")
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
        reg(c, f"p{i}", seed=i)

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
            "from nos_amd.models.yolos_program import demo_tenant; demo_tenant('bf16', 1); "
            "from nos_amd.podserver.program import mlp_program, parse; parse(*mlp_program(64, 1, 8)); "
            "print('torch' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "False"


# ----------------------------------------------------------------- control plane
def test_device_plugin_allocates_pod_server_slices_without_device_nodes(tmp_path):
    import json

    from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.podserver.allocations import lookup, records_dir

    root = tmp_path / "ps"
    p = NosAmdDevicePlugin("n1", FakeSmi(gpus=2, node="n1"), mode=C.PARTITIONING_CUMASK, cu_policy="shared",
                           pod_server_dir=str(root))
    p.set_config("n1-1", {"gpus": [{"index": 1, "slices": [{"profile": "10gb", "replicas": 3}]}]})
    devs = p.list_devices("amd.com/gpu-10gb")
    assert len(devs) == 3
    a = p.allocate("amd.com/gpu-10gb", [devs[0].id], owner="default/pod-a/main")
    tok = a.envs.pop(C.ENV_POD_TOKEN)
    assert a.envs == {C.ENV_POD_SERVER: f"{root}/gpu-1/server.sock", C.ENV_MEMORY_LIMIT_GB: "10"}
    # no device nodes, and only this GPU's socket directory is mounted (not the records)
    assert a.devices == [] and a.mounts == [f"{root}/gpu-1"]
    rec, path = lookup(records_dir(root, 1), tok)
    assert rec["memory_gb"] == 10 and rec["device_ids"] == [devs[0].id] and rec["cu_mask"] is None
    assert (path.stat().st_mode & 0o777) == 0o600 and tok not in path.read_text()
    assert lookup(records_dir(root, 0), tok) is None  # the record is GPU 1's only
    b = p.allocate("amd.com/gpu-10gb", [devs[1].id])
    assert b.envs[C.ENV_POD_TOKEN] != tok
    p.release([devs[0].id])  # the pod went away: its record goes, the server evicts the tenant
    assert not path.exists() and lookup(records_dir(root, 1), b.envs[C.ENV_POD_TOKEN]) is not None
    # a proportional CU policy hands the tenant's CU mask to the server (record), not to HIP
    q = NosAmdDevicePlugin("n1", FakeSmi(gpus=1, node="n1"), mode=C.PARTITIONING_CUMASK, cu_policy="even",
                           pod_server_dir=str(tmp_path / "q"))
    q.set_config("n1-1", {"gpus": [{"index": 0, "slices": [{"profile": "10gb", "replicas": 4}]}]})
    b = q.allocate("amd.com/gpu-10gb", [q.list_devices("amd.com/gpu-10gb")[0].id])
    assert C.ENV_POD_CU_MASK in b.envs and C.ENV_CU_MASK not in b.envs
    rec = json.loads(next((tmp_path / "q" / ".allocations" / "gpu-0").glob("*.json")).read_text())
    assert rec["cu_mask"] == b.envs[C.ENV_POD_CU_MASK] and bin(int(rec["cu_mask"], 16)).count("1") == 64


def test_pod_server_node_schedules_slices_by_memory_not_hws_slots(tmp_path):
    from nos_amd.bench_support import control_plane_plan, schedulable_pods

    # 10 GB slices on one 288 GB MI355X: 8 GPU processes (HWS) vs 28 server tenants (memory)
    assert schedulable_pods(1, 10)["schedulable_fractional_pods_per_node"] == 8
    assert schedulable_pods(1, 10, pod_server_tenants=48)["schedulable_fractional_pods_per_node"] == 28
    # ... and the server's tenant count bounds it when memory does not
    assert schedulable_pods(1, 5, pod_server_tenants=16)["schedulable_fractional_pods_per_node"] == 16
    _, info = control_plane_plan(2, 28, 10, 256, local_gpu=1, cu_policy="shared", capacity_probe=False,
                                 pod_server_tenants=48, pod_server_dir=str(tmp_path))
    assert info["placed_pods"] == 56 and info["pending_pods"] == 0
    assert len(info["envs"]) == 28
    assert all(e[C.ENV_POD_SERVER] == f"{tmp_path}/gpu-1/server.sock" and C.ENV_VISIBLE_DEVICES not in e
               for e in info["envs"])
    assert len({e[C.ENV_POD_TOKEN] for e in info["envs"]}) == 28  # one token per allocation
    assert len(list((tmp_path / ".allocations" / "gpu-1").glob("*.json"))) == 28


def test_podserver_binary_supervises_one_server_per_gpu(tmp_path):
    """``nos_amd.cmd.podserver --gpus 0,1`` (the DaemonSet entry point): one
    server per GPU at <socket-dir>/gpu-<i>/server.sock, stopped by SIGTERM."""
    import os
    import signal
    import subprocess
    import sys

    from nos_amd.cmd.podserver import socket_path

    env = {**os.environ, "OMP_NUM_THREADS": "1"}
    p = subprocess.Popen([sys.executable, "-m", "nos_amd.cmd.podserver", "--gpus", "0,1", "--device", "cpu",
                          "--socket-dir", str(tmp_path), "--lanes", "1", "--open-admission"], env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        for g in (0, 1):
            c = PodClient(socket_path(tmp_path, g), connect_timeout_s=60)
            reg(c, f"p{g}")
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
    args = spec["containers"][0]["args"]
    assert args[:2] == ["--gpus", "all"]
    # the PodResources reaper is on in deployment: flag + the kubelet socket's directory
    assert args[args.index("--pod-resources-socket") + 1] == C.KUBELET_PODRESOURCES_SOCKET
    mounts = {v["mountPath"] for v in spec["containers"][0]["volumeMounts"]}
    assert "/var/lib/kubelet/pod-resources" in mounts
    assert any(v.get("hostPath", {}).get("path") == "/var/lib/kubelet/pod-resources" for v in spec["volumes"])

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
    reg(c, "metered")
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
    reg(c, "solo")
    for _ in range(5):
        c.infer()
    assert seen == [True] * 5
    seen.clear()
    others = [PodClient(server.path, connect_timeout_s=5) for _ in range(2)]
    for i, o in enumerate(others):
        reg(o, f"co{i}")
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


def test_chart_defaults_pod_server_nodes_to_shared_cus():
    """cuPolicy "auto": shared CUs when the pod server is enabled (its tenants
    share the lanes' graphs, MPS's default), proportional masks otherwise; an
    explicit policy wins."""
    import yaml

    from nos_amd.cmd import manifests as m

    def policy(values):
        out = m.render(values)
        cm = [o for o in yaml.safe_load_all(out["deviceplugin/daemonset.yaml"]) if o and o["kind"] == "ConfigMap"][0]
        return yaml.safe_load(cm["data"]["device_plugin_config.yaml"])["cuPolicy"]

    assert policy({}) == "proportional"
    assert policy({"gpuPartitioner": {"podServer": {"enabled": True}}}) == "shared"
    assert policy({"gpuPartitioner": {"cuPolicy": "even", "podServer": {"enabled": True}}}) == "even"


def test_node_labeler_removes_the_pod_server_label_when_disabled():
    from nos_amd.agents.devices import NodeLabeler
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.kube import objects as ko
    from nos_amd.runtime.manager import Request
    from nos_amd.sim.apiserver import ApiServer

    api = ApiServer()
    api.create({"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1", "labels": {}}})
    smi = FakeSmi(gpus=1, node="n1")
    NodeLabeler(api, "n1", smi, pod_server_tenants=48).reconcile(Request("n1"))
    assert ko.labels(api.get("Node", "n1"))[C.LABEL_POD_SERVER_TENANTS] == "48"
    NodeLabeler(api, "n1", smi, pod_server_tenants=0).reconcile(Request("n1"))
    labels = ko.labels(api.get("Node", "n1"))
    assert C.LABEL_POD_SERVER_TENANTS not in labels and labels[C.LABEL_AMD_COUNT] == "1"


def test_host_array_of_row_strided_outputs():
    """Column slices of a merged result go to the host as their covering row
    block (no contiguous copy); other layouts as before."""
    import numpy as np
    import torch

    from nos_amd.podserver.server import _host_array

    base = torch.arange(100 * 96, dtype=torch.float32).view(100, 96)
    for t in (base[:, :92], base[:, 92:], base[10:20, 3:7], base.t(), base):
        assert np.array_equal(_host_array(t), t.contiguous().numpy())
