"""Pod-server admission and failure handling (CPU):

* allocation tokens (podserver/allocations.py): a tenant registers only with
  the token the device plugin minted, gets the slice of the plugin's record
  whatever it claims, one tenant per token, and loses its tenant when its pod
  is deleted from the kubelet (record removed) or when PodResources no longer
  lists its devices -- reference: the MPS replica's slice fixed by the device
  plugin, ``internal/partitioning/mps/partitioner.go:123-157``, device usage
  from PodResources, ``pkg/resource/client.go:39-87``;
* slot and memory reservation before the (slow) build: concurrent
  registrations never over-commit;
* program validation: whatever a client sends is refused before anything is
  allocated unless it is a well-formed program over the whitelisted ops;
* server crashes: the supervisor restarts a killed server, a client with
  ``reconnect_s`` re-registers and carries on, and a pod without it exits
  non-zero (so the kubelet restarts it).
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from nos_amd.api import constants as C
from nos_amd.models.yolos_program import demo_tenant
from nos_amd.podserver import program as PG
from nos_amd.podserver.allocations import AllocationStore, records_dir, socket_path
from nos_amd.podserver.client import PodClient, PodServerError, PodServerGone
from nos_amd.podserver.server import PodServer

YOLOS = demo_tenant("fp32", 0, small=False)


def _wait(cond, timeout=10.0):
    deadline = time.monotonic() + timeout
    while not cond():
        if time.monotonic() > deadline:
            return False
        time.sleep(0.02)
    return True


@pytest.fixture
def tokened(tmp_path):
    """A GPU-1 server reading the records an AllocationStore writes."""
    store = AllocationStore(tmp_path)
    srv = PodServer(socket_path(tmp_path, 1), device="cpu", lanes=1, max_tenants=4, memory_gb=40,
                    allocations_dir=records_dir(tmp_path, 1), reap_interval_s=0.05).start()
    yield store, srv
    srv.stop()


def test_tokens_bind_tenants_to_their_allocation(tokened):
    store, srv = tokened
    store.write(1, "tok-a", {"memory_gb": 10, "cu_mask": None, "device_ids": ["g1::10gb::0"]})
    store.write(1, "tok-zero", {"memory_gb": 0, "device_ids": ["g1::0gb::0"]})
    store.write(0, "tok-gpu0", {"memory_gb": 10, "device_ids": ["g0::10gb::0"]})
    c = PodClient(srv.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="no allocation token"):
        c.register("p", *YOLOS, env={})
    with pytest.raises(PodServerError, match="unknown allocation token"):
        c.register("p", *YOLOS, token="forged")
    with pytest.raises(PodServerError, match="unknown allocation token"):  # another GPU's allocation
        c.register("p", *YOLOS, token="tok-gpu0")
    with pytest.raises(PodServerError, match="no memory slice"):
        c.register("p", *YOLOS, token="tok-zero")
    # the slice is the record's, whatever the client claims
    rep = c.register("p", *YOLOS, token="tok-a", memory_limit_gb=100, cu_mask="ffff")
    assert rep["memory_limit_gb"] == 10 and rep["cu_mask"] is None
    c.infer()
    d = PodClient(srv.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="already holds a tenant"):
        d.register("p-again", *YOLOS, token="tok-a")
    c.close()  # the token is free again once its tenant left
    assert _wait(lambda: not srv.tenants)
    d.register("p-again", *YOLOS, token="tok-a")
    d.close()


def test_a_released_allocation_evicts_its_tenant(tokened):
    store, srv = tokened
    store.write(1, "tok-b", {"memory_gb": 10, "device_ids": ["g1::10gb::1"]})
    store.write(1, "tok-c", {"memory_gb": 10, "device_ids": ["g1::10gb::2"]})
    b, c = PodClient(srv.path, connect_timeout_s=5), PodClient(srv.path, connect_timeout_s=5)
    b.register("b", *YOLOS, token="tok-b")
    c.register("c", *YOLOS, token="tok-c")
    b.infer()
    assert store.remove_devices(["g1::10gb::1"]) == 1
    assert _wait(lambda: len(srv.tenants) == 1)
    with pytest.raises(PodServerGone):
        b.infer()
    c.infer()  # the other tenant is untouched
    assert srv.stats()["evictions"] == 1
    c.close()


def test_pod_resources_eviction_without_records(tmp_path):
    from nos_amd.resource.client import ContainerDevices, ContainerResources, PodResources

    class Lister:
        pods = [PodResources("p", "ns", [ContainerResources("c", [ContainerDevices("amd.com/gpu-10gb", ["d1"])])])]

        def list(self):
            return list(self.pods)

    store = AllocationStore(tmp_path)
    path = store.write(0, "tok", {"memory_gb": 10, "device_ids": ["d1"]})
    lister = Lister()
    srv = PodServer(socket_path(tmp_path, 0), device="cpu", lanes=1, memory_gb=40,
                    allocations_dir=records_dir(tmp_path, 0), pod_resources=lister, reap_interval_s=3600).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=5)
        c.register("p", *YOLOS, token="tok")
        assert srv.reap_once() == 0
        lister.pods = []  # the kubelet no longer runs a pod with d1 (the plugin has not synced yet)
        assert path.exists() and srv.reap_once() == 1
        assert _wait(lambda: not srv.tenants)
    finally:
        srv.stop()


def test_a_pod_deleted_from_the_kubelet_simulator_loses_its_tenant(tmp_path):
    """End to end through the control plane: scheduler -> device plugin
    Allocate (token + record) -> pod registers with its env -> the pod is
    deleted -> kubelet teardown releases the devices -> the record goes ->
    the server evicts the tenant."""
    from nos_amd.api.config import GpuPartitionerConfig
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.sim.cluster import SimCluster

    cl = SimCluster(partitioner_config=GpuPartitionerConfig(cuPolicy="shared"))
    cl.add_node("n0", C.PARTITIONING_CUMASK, smi=FakeSmi(gpus=1, node="n0"), pod_server_tenants=48,
                pod_server_dir=str(tmp_path))
    cl.settle(30)
    for i in range(2):
        cl.submit_pod(f"tenant-{i}", {f"{C.AMD_SLICE_RESOURCE_PREFIX}10gb": 1})
    cl.settle(600, until=lambda: not cl.pending_pods())
    envs = {k: rc.envs for k, conts in cl.nodes["n0"].kubelet.running_containers().items() for rc in conts}
    assert len(envs) == 2
    srv = PodServer(socket_path(tmp_path, 0), device="cpu", lanes=1, memory_gb=288,
                    allocations_dir=records_dir(tmp_path, 0), reap_interval_s=0.05).start()
    try:
        clients = {}
        for key, env in envs.items():
            assert env[C.ENV_POD_SERVER] == str(srv.path)
            c = clients[key] = PodClient.from_env(env, connect_timeout_s=5)
            rep = c.register(key, *YOLOS, env=env)
            assert rep["memory_limit_gb"] == 10
            c.infer()
        gone, stays = sorted(envs)
        cl.api.delete("Pod", gone.split("/", 1)[1], gone.split("/", 1)[0])
        cl.settle(60)
        assert _wait(lambda: len(srv.tenants) == 1)
        assert next(iter(srv.tenants.values())).pod == stays
        with pytest.raises(PodServerGone):
            clients[gone].infer()
        clients[stays].infer()
        clients[stays].close()
    finally:
        srv.stop()


def test_concurrent_registrations_cannot_overcommit(tmp_path, monkeypatch):
    """Slots and slice memory are reserved before the build: 6 clients racing
    for a 3-tenant, 30 GB server while each build takes a while."""
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, max_tenants=3, memory_gb=30).start()
    orig = srv._build

    def slow_build(*a, **kw):
        time.sleep(0.3)
        return orig(*a, **kw)

    monkeypatch.setattr(srv, "_build", slow_build)
    try:
        results: list[str] = []
        clients = [PodClient(srv.path, connect_timeout_s=5) for _ in range(6)]

        def go(i):
            try:
                clients[i].register(f"p{i}", *YOLOS, memory_limit_gb=8 if i % 2 else 12)
                results.append("ok")
            except PodServerError as e:
                results.append(str(e))

        th = [threading.Thread(target=go, args=(i,)) for i in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        ok = results.count("ok")
        assert 1 <= ok <= 3 and len(srv.tenants) == ok
        assert sum(t.memory_limit_gb for t in srv.tenants.values()) <= 30
        assert all(r == "ok" or "server full" in r or "does not fit" in r for r in results), results
        assert srv.stats()["pending"] == 0
        for c in clients:
            c.close()
    finally:
        srv.stop()


@pytest.mark.parametrize("mutate,match", [
    (lambda p, w: p["nodes"].append({"op": "exec", "inputs": ["pixel_values"], "output": "z"}), "not one the pod"),
    (lambda p, w: p["nodes"].insert(0, {"op": "relu", "inputs": ["later"], "output": "y"}), "not defined before"),
    (lambda p, w: p["params"][0].update(offset=len(w)), "outside the"),
    (lambda p, w: p["params"][1].update(offset=p["params"][0]["offset"]), "overlap"),
    (lambda p, w: p["params"][0].update(shape=[3, 3]), "nbytes"),
    (lambda p, w: p["nodes"][-1]["attrs"].update(evil=1), "unknown attributes"),
    (lambda p, w: p.update(outputs=["nope"]), "outputs must name"),
    (lambda p, w: p.update(format="pickle"), "format"),
    (lambda p, w: p["nodes"].append({"op": "reshape", "inputs": ["pixel_values"], "output": "r",
                                     "attrs": {"shape": [7, 7]}}), "cannot reshape"),
    (lambda p, w: p["nodes"].append({"op": "linear", "inputs": ["pixel_values", "patch_w"], "output": "l"}),
     "weight"),
])
def test_malformed_programs_are_refused_before_anything_is_built(mutate, match):
    import copy

    p, w = copy.deepcopy(YOLOS[0]), YOLOS[1]
    mutate(p, w)
    with pytest.raises(PG.ProgramError, match=match):
        PG.parse(p, w)


def test_gpu_kernel_constraints_are_checked_at_parse_time():
    p, w = PG.mlp_program(dim=96, layers=1, batch=8, dtype="bf16")  # K = 96: not a multiple of 64
    PG.parse(p, w)  # fine for the CPU reference path
    with pytest.raises(PG.ProgramError, match="K % 64"):
        PG.parse(p, w, gpu=True)
    b = PG.Builder("attn")
    x = b.input("x", [1, 16, 3 * 2 * 32])
    b.op("attention", x, heads=2, out="a")
    with pytest.raises(PG.ProgramError, match="head_dim 64"):
        PG.parse(*b.build(["a"]), gpu=True)


def test_static_estimate_refuses_a_program_larger_than_its_slice(tmp_path):
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=5)
        big = PG.mlp_program(dim=512, layers=2, batch=4096, dtype="fp32")
        est = PG.parse(*big).bytes_estimate / 2 ** 30
        with pytest.raises(PodServerError, match="static estimate"):
            c.register("big", *big, memory_limit_gb=round(est / 2, 3))
        assert not srv.tenants and srv.stats()["pending"] == 0
        c.register("big", *big, memory_limit_gb=round(est * 2, 3))
        c.close()
    finally:
        srv.stop()


def test_weights_may_fill_the_slice_but_not_exceed_it(tmp_path, monkeypatch):
    """A register request's payload is bounded by the tenant's slice, not by
    the 1 GiB cap on input images (multi-GB models on big slices); past the
    slice the server drains the payload and replies with an error on the
    same connection, which then registers a smaller program."""
    from nos_amd.podserver import protocol as P

    monkeypatch.setattr(P, "MAX_PAYLOAD", 1 << 16)  # weights well past it, inputs too
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=5)
        prog, w = PG.mlp_program(dim=256, layers=2, batch=8, dtype="fp32")
        assert len(w) > 1 << 16
        with pytest.raises(PodServerError, match="PayloadTooLarge"):
            c.register("big", prog, w, memory_limit_gb=len(w) / 2 / 2 ** 30)
        rep = c.register("ok", prog, w, memory_limit_gb=1)  # same connection, still in step
        assert rep["tenants"] == 1
        with pytest.raises(PodServerError, match="PayloadTooLarge"):  # an input over MAX_PAYLOAD
            c.infer(np.zeros((1 << 15,), np.float32))
        c.infer()
        c.close()
    finally:
        srv.stop()


# ----------------------------------------------------------------- crashes
def _supervised(tmp_path):
    env = {**os.environ, "OMP_NUM_THREADS": "1"}
    return subprocess.Popen([sys.executable, "-m", "nos_amd.cmd.podserver", "--gpus", "0", "--device", "cpu",
                             "--socket-dir", str(tmp_path), "--lanes", "1", "--open-admission"], env=env,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def test_supervisor_restarts_a_killed_server_and_clients_reregister(tmp_path):
    sup = _supervised(tmp_path)
    try:
        path = socket_path(tmp_path, 0)
        keep = PodClient(path, connect_timeout_s=60, reconnect_s=60)
        keep.register("keep", *YOLOS, memory_limit_gb=10)
        plain = PodClient(path, connect_timeout_s=5)
        plain.register("plain", *YOLOS, memory_limit_gb=10)
        x = np.random.default_rng(0).standard_normal(keep.info["input_shape"]).astype(np.float32)
        before, _ = keep.infer(x, outputs=True)
        pid = keep.stats()["pid"]
        os.kill(pid, signal.SIGKILL)  # the server dies mid-run
        with pytest.raises(PodServerGone):
            plain.infer()
        after, _ = keep.infer(x, outputs=True)  # waits for the restart, registers again, retries
        assert keep.reconnects == 1 and keep.stats()["pid"] != pid
        np.testing.assert_array_equal(before[0], after[0])
        keep.close()
    finally:
        sup.send_signal(signal.SIGTERM)
        assert sup.wait(timeout=60) == 0


def test_a_pod_exits_nonzero_when_its_server_dies(tmp_path):
    from nos_amd.models.pod import STATE_READY, StatusBoard

    srv = subprocess.Popen([sys.executable, "-m", "nos_amd.cmd.podserver", "--gpu", "0", "--device", "cpu",
                            "--socket-dir", str(tmp_path), "--lanes", "1", "--open-admission"],
                           env={**os.environ, "OMP_NUM_THREADS": "1"}, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
    board = StatusBoard(tmp_path / "board", pods=1)
    env = {**os.environ, C.ENV_POD_SERVER: str(socket_path(tmp_path, 0)), C.ENV_MEMORY_LIMIT_GB: "10",
           "OMP_NUM_THREADS": "1"}
    pod = subprocess.Popen([sys.executable, "-m", "nos_amd.models.pod", "--status", str(tmp_path / "board"),
                            "--slot", "0", "--out", str(tmp_path), "--device", "cpu"], env=env,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        assert _wait(lambda: board.states()[0] == STATE_READY and board.counts()[0] > 2, timeout=120)
        srv.kill()
        assert pod.wait(timeout=60) == 1
        assert b"connection lost" in pod.stderr.read()
    finally:
        for p in (pod, srv):
            if p.poll() is None:
                p.kill()


# ----------------------------------------------------------------- claims before payloads
def _raw_register(path, token, npay, send=None):
    """A register request announcing ``npay`` payload bytes, of which only
    ``send`` are sent (default all): the server's claim happens on the header."""
    import json
    import socket
    import struct

    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(str(path))
    prog, w = PG.mlp_program(dim=64, layers=1, batch=8, dtype="fp32")
    w = w + bytes(npay - len(w)) if npay > len(w) else w[:npay]
    js = json.dumps({"op": "register", "pod": "raw", "token": token, "program": prog, "memory_limit_gb": 1}).encode()
    s.sendall(struct.pack(">IQ", len(js), len(w)) + js)
    s.sendall(w[:len(w) if send is None else send])
    return s, w


def test_a_token_is_claimed_before_its_payload_is_read(tokened):
    """one valid token on many connections, each sending slice-sized
    weights, must not make the server buffer N x slice bytes.  The first
    connection's header claims the token; a second register with it is refused
    while the first payload is still in flight."""
    from nos_amd.podserver import protocol as P

    store, srv = tokened
    store.write(1, "tok-x", {"memory_gb": 10, "device_ids": ["g1::10gb::7"]})
    a, w = _raw_register(srv.path, "tok-x", 1 << 20, send=1 << 10)   # stalls mid-payload
    assert _wait(lambda: "tok-x" in srv._tokens and srv.stats()["pending"] == 1)
    c = PodClient(srv.path, connect_timeout_s=5)
    with pytest.raises(PodServerError, match="registration in flight"):
        c.register("again", *YOLOS, token="tok-x")
    a.sendall(w[1 << 10:])                                            # the first one completes
    rep, _ = P.recv_msg(a)
    assert rep["ok"], rep
    assert len(srv.tenants) == 1 and srv._inflight_bytes == 0
    a.close()
    c.close()


def test_register_bytes_in_flight_are_capped(tmp_path):
    from nos_amd.podserver import protocol as P

    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40,
                    max_inflight_register_gb=1.5 / 1024).start()   # 1.5 MiB
    try:
        a, w = _raw_register(srv.path, None, 1 << 20, send=10)       # 1 MiB claimed, stalled
        assert _wait(lambda: srv._inflight_bytes == 1 << 20)
        b, _ = _raw_register(srv.path, None, 1 << 20)                # would make 2 MiB: refused, drained
        rep, _ = P.recv_msg(b)
        assert not rep["ok"] and "in flight" in rep["error"]
        assert srv.stats()["pending"] == 1
        a.sendall(w[10:])
        assert P.recv_msg(a)[0]["ok"]
        assert srv._inflight_bytes == 0 and srv.stats()["pending"] == 0
        b2, _ = _raw_register(srv.path, None, 1 << 20)               # room again
        assert P.recv_msg(b2)[0]["ok"]
        for s in (a, b, b2):
            s.close()
    finally:
        srv.stop()


def test_a_dropped_connection_releases_its_claim(tokened):
    store, srv = tokened
    store.write(1, "tok-d", {"memory_gb": 10, "device_ids": ["g1::10gb::8"]})
    a, _ = _raw_register(srv.path, "tok-d", 1 << 20, send=100)
    assert _wait(lambda: srv.stats()["pending"] == 1)
    a.close()                                                        # mid-payload
    assert _wait(lambda: srv.stats()["pending"] == 0 and not srv._tokens and srv._inflight_bytes == 0)
    c = PodClient(srv.path, connect_timeout_s=5)
    c.register("p", *YOLOS, token="tok-d")                           # the token is usable again
    c.close()


def test_a_stalled_register_payload_times_out_and_frees_its_claim(tmp_path):
    """a client that sends only a register header (or
    part of its payload) and stalls must not hold its slot, slice and
    in-flight bytes forever: the payload has a deadline, then the claim is
    released and the connection closed."""
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40, max_inflight_register_gb=1.5 / 1024,
                    register_timeout_s=0.5, register_min_mb_s=1e6).start()
    try:
        a, _ = _raw_register(srv.path, None, 1 << 20, send=0)         # header only
        assert _wait(lambda: srv._inflight_bytes == 1 << 20)
        assert _wait(lambda: srv._inflight_bytes == 0 and srv.stats()["pending"] == 0, timeout=10)
        a.settimeout(5)
        assert a.recv(1) == b""                                      # the server closed it
        a.close()
        c = PodClient(srv.path, connect_timeout_s=5)                   # the budget is free again
        c.register("p", *YOLOS, memory_limit_gb=10)
        c.close()
    finally:
        srv.stop()


def test_a_bad_memory_limit_type_is_an_error_reply_not_a_dropped_connection(tmp_path):
    """a list for memory_limit_gb under open admission."""
    from nos_amd.podserver import protocol as P
    import socket

    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40).start()
    try:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect(str(srv.path))
        prog, w = YOLOS
        P.send_msg(s, {"op": "register", "pod": "x", "program": prog, "memory_limit_gb": [1, 2]}, w)
        rep, _ = P.recv_msg(s)
        assert not rep["ok"] and "AdmissionError" in rep["error"]
        P.send_msg(s, {"op": "stats"})                                # the connection is still in step
        assert P.recv_msg(s)[0]["ok"]
        s.close()
    finally:
        srv.stop()


def test_integer_data_for_an_fp32_tenant_goes_as_values(tmp_path):
    """the wire carries no dtype of its own, so the
    client converts by the registered program's input type (a uint8 image
    for an fp32 model arrives as float32 values, not reinterpreted bits) and
    the server refuses a request that names another type."""
    from nos_amd.podserver import protocol as P
    import socket

    prog, w = PG.mlp_program(dim=32, layers=1, batch=2, dtype="fp32", seed=0)
    srv = PodServer(tmp_path / "s.sock", device="cpu", lanes=1, memory_gb=40).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=5)
        rep = c.register("p", prog, w, memory_limit_gb=1)
        assert rep["input_dtype"] == "f32" and c.input_dtype == "f32"
        shape = rep["input_shape"]
        xi = (np.arange(int(np.prod(shape))) % 7).reshape(shape).astype(np.uint8)
        oi, _ = c.infer(xi, outputs=True)
        of, _ = c.infer(xi.astype(np.float32), outputs=True)
        assert np.array_equal(oi[0], of[0])
        # a raw request naming the wrong type is refused
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect(str(srv.path))
        P.send_msg(s, {"op": "register", "pod": "q", "program": prog, "memory_limit_gb": 1}, w)
        assert P.recv_msg(s)[0]["ok"]
        P.send_msg(s, {"op": "infer", "shape": shape, "dtype": "i32"}, xi.astype(np.int32).tobytes())
        rep2, _ = P.recv_msg(s)
        assert not rep2["ok"] and "takes 'f32'" in rep2["error"]
        s.close()
        c.close()
    finally:
        srv.stop()


# ----------------------------------------------------------------- device plugin restart
def _pod_server_plugin(root, smi):
    from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin

    p = NosAmdDevicePlugin("n1", smi, mode=C.PARTITIONING_CUMASK, cu_policy="even", pod_server_dir=str(root),
                           adopt_records=True)
    p.set_config("n1-1", {"gpus": [{"index": 0, "slices": [{"profile": "10gb", "replicas": 4}]}]})
    return p


def test_plugin_restart_keeps_live_records_and_their_cu_slots(tmp_path):
    """records survive a device-plugin restart -- the new
    process adopts them (devices stay allocated, CU slots stay put), a new pod
    gets a non-overlapping mask, orphan records are deleted, and records of
    pods PodResources no longer lists are released."""
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.podserver.allocations import lookup

    smi = FakeSmi(gpus=1, node="n1")
    root = tmp_path / "ps"
    p1 = _pod_server_plugin(root, smi)
    ids = sorted(d.id for d in p1.list_devices("amd.com/gpu-10gb"))
    toks, masks = {}, {}
    for did in ids[:3]:
        a = p1.allocate("amd.com/gpu-10gb", [did], owner=f"ns/{did}")
        toks[did], masks[did] = a.envs[C.ENV_POD_TOKEN], a.envs[C.ENV_POD_CU_MASK]
    slots1 = {did: p1.cu_slots[did].slots for did in ids[:3]}
    # an orphan: a record for a device no slice table has any more
    AllocationStore(root).write(0, "tok-orphan", {"memory_gb": 10, "device_ids": ["gone::10gb::0"]})
    del p1                                                           # the plugin process restarts

    p2 = _pod_server_plugin(root, smi)
    assert {did: p2.allocated[did] for did in ids[:3]} == {did: f"ns/{did}" for did in ids[:3]}
    assert {did: p2.cu_slots[did].slots for did in ids[:3]} == slots1
    for did in ids[:3]:
        assert lookup(records_dir(root, 0), toks[did]) is not None   # records kept, tenants keep running
    assert lookup(records_dir(root, 0), "tok-orphan") is None        # orphan deleted
    new = p2.allocate("amd.com/gpu-10gb", [ids[3]], owner="ns/new")
    new_cus = set(p2.cus_of(ids[3]))
    assert new_cus and all(not (new_cus & set(p2.cus_of(did))) for did in ids[:3])
    assert int(new.envs[C.ENV_POD_CU_MASK], 16) & int(masks[ids[0]], 16) == 0
    # PodResources: the pod of ids[0] is gone -> its record goes (its tenant is evicted)
    p2.sync_allocated(set(ids[1:]))
    assert lookup(records_dir(root, 0), toks[ids[0]]) is None
    assert lookup(records_dir(root, 0), toks[ids[1]]) is not None


def test_pod_server_allocations_are_mounted_read_only(tmp_path):
    from nos_amd.deviceplugin.grpc_server import _ResourceServicer
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.grpcapi.protos import deviceplugin as pb

    p = _pod_server_plugin(tmp_path / "ps", FakeSmi(gpus=1, node="n1"))

    class Owner:
        plugin = p

    ids = [d.id for d in p.list_devices("amd.com/gpu-10gb")]
    req = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=[i]) for i in ids[:2]])
    rep = _ResourceServicer(Owner(), "amd.com/gpu-10gb").Allocate(req, None)
    mounts = [m for cr in rep.container_responses for m in cr.mounts]
    assert len(mounts) == 2 and all(m.read_only for m in mounts)
    assert all(m.host_path == str(tmp_path / "ps" / "gpu-0") for m in mounts)


# ----------------------------------------------------------------- estimate + overflow
@pytest.mark.parametrize("shape", [[2 ** 62, 4], [2 ** 63, 1], [2 ** 40, 2 ** 40]])
def test_huge_shapes_are_refused_not_wrapped(shape):
    b = PG.Builder("huge")
    b.input("x", shape)
    b.op("relu", "x", out="y")
    with pytest.raises(PG.ProgramError, match="over|more than"):
        PG.parse(*b.build(["y"]))


def test_mixed_permute_dims_are_a_program_error():
    b = PG.Builder("perm")
    b.input("x", [2, 3])
    b.op("permute", "x", dims=[1, "0"], out="y")
    with pytest.raises(PG.ProgramError, match="permutation"):
        PG.parse(*b.build(["y"]))


def test_constant_folded_chains_count_as_persistent_weights():
    """A chain of all-constant nodes is materialised at load time: the static
    estimate must count every folded value, not release it like an activation."""
    b = PG.Builder("fold")
    x = b.input("x", [4, 64])
    w = b.param("w", np.ones((1, 64), np.float32))
    big = [b.op("expand", w, shape=[4096, 64])]
    for _ in range(4):
        big.append(b.op("mul", big[-1], big[-1]))
    y = b.op("add", x, b.op("slice", big[-1], dim=0, start=0, end=4))
    p = PG.parse(*b.build([y]))
    assert p.foldable() >= set(big)
    assert p.bytes_estimate >= sum(p.values[v].nbytes for v in big)
    import torch

    m = p.compile("cpu")
    assert set(big).isdisjoint(m.consts)           # dead folded values were freed
    assert torch.allclose(m(torch.zeros(4, 64))[0], torch.ones(4, 64))


def test_simulated_plugins_sharing_a_records_dir_keep_each_others_records(tmp_path):
    """bench.py plans several placements over one pod-server directory (the
    main fleet + the latency-table rows, one server): without adopt_records a
    later plugin must not delete an earlier plugin's records as orphans."""
    from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
    from nos_amd.gpu.fakesmi import FakeSmi
    from nos_amd.podserver.allocations import lookup

    root = tmp_path / "ps"
    toks = []
    for reps in (4, 1):
        p = NosAmdDevicePlugin("n1", FakeSmi(gpus=1, node="n1"), mode=C.PARTITIONING_CUMASK, cu_policy="shared",
                               pod_server_dir=str(root))
        p.set_config("n1-1", {"gpus": [{"index": 0, "slices": [{"profile": "10gb", "replicas": reps}]}]})
        for d in p.list_devices("amd.com/gpu-10gb"):
            toks.append(p.allocate("amd.com/gpu-10gb", [d.id]).envs[C.ENV_POD_TOKEN])
    assert all(lookup(records_dir(root, 0), t) is not None for t in toks)
