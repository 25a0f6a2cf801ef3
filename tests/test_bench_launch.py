"""The exact multi-GPU launch path of bench.py (python -m torch.distributed.run
... bench.py --gpus N), rehearsed on the CPU: gloo instead of RCCL, tiny
YOLOS pods on the CPU.  Every rank places its pods through the control plane,
starts them as processes, runs its lockstep DP trainer pod, and rank 0 prints
ONE JSON line aggregated over ranks."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _run(n: int, port: int, pods: int = 3, timeout: int = 600, **env_extra) -> list[dict]:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", str(n), "--device", "cpu",
           "--steps", "4", "--warmup", "1", "--step-s", "0.4", "--ref-pod-s", "0", "--pods-per-gpu", str(pods)]
    env = {**os.environ, "OMP_NUM_THREADS": "1", **env_extra}
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


@pytest.mark.timeout(900)
def test_torchrun_two_ranks_aggregate_one_json_line():
    lines = _run(2, 29611)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    base = json.loads((REPO / "BASELINE.json").read_text())
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 1
    # 3 pods per GPU: 2 inference pods + the DP trainer pod, all observed running, on both ranks
    assert d["value"] == 6 and d["config"]["pods_placed_per_node"] == 6
    assert d["trainer_pods"]["rank0"]["running"] and d["trainer_pods"]["per_node_allreduce_gb_per_s"] > 0
    assert d["ms_per_step"] == pytest.approx(400, rel=0.2)
    assert d["aggregate_inf_per_s"] > 0 and d["scaling"] == "weak"


@pytest.mark.timeout(900)
def test_trainer_job_that_cannot_form_falls_back_on_every_rank():
    """A trainer pod that fails before READY (here: an injected init fault) makes
    EVERY rank re-run the window without trainer pods; the line records why."""
    lines = _run(2, 29617, NOS_AMD_TRAINER_FAULT="init")
    assert len(lines) == 1
    d = lines[0]
    assert d["trainer_pods"] is None and "failed to start" in d["trainer_error"]
    assert d["config"]["collective_tenant"] is False
    assert d["value"] == 6 and d["aggregate_inf_per_s"] > 0  # 3 inference pods per rank


@pytest.mark.timeout(600)
def test_latency_table_rows_are_self_consistent():
    """bench.py --table: one aligned window per (mode, pods); pods / mean latency == throughput in every row."""
    cmd = [sys.executable, "bench.py", "--device", "cpu", "--steps", "2", "--warmup", "1", "--step-s", "0.3",
           "--ref-pod-s", "0", "--extra-bf16-s", "0", "--pods-per-gpu", "2", "--table", "1,3",
           "--table-window-s", "2"]
    r = subprocess.run(cmd, cwd=REPO, env={**os.environ, "OMP_NUM_THREADS": "1"}, capture_output=True, text=True,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    rows = d["latency_table"]
    # server mode (the default) adds pod-server rows in front of the process-pod rows
    assert [(t["mode"], t["pods"]) for t in rows] == [("server", 1), ("server", 3), ("shared", 1), ("shared", 3),
                                                      ("cumask", 1), ("cumask", 3)]
    for t in rows:
        assert t["concurrent"] == t["pods"]
        assert t["pods_over_latency"] == pytest.approx(t["inf_per_s"], rel=1e-3)


def test_fold_gpus_maps_every_rank_onto_the_visible_gpus(monkeypatch):
    """NOS_AMD_BENCH_FOLD_GPUS=1 (multi-rank rehearsal on fewer GPUs): rank r's
    pods get HIP_VISIBLE_DEVICES = r % visible GPUs; without it, the control
    plane's own GPU index."""
    import importlib
    import types

    sys.path.insert(0, str(REPO))
    bench = importlib.import_module("bench")
    args = types.SimpleNamespace()
    envs, _ = bench.plan(args, 2, 1, 36, 2, "shared")
    assert {e["HIP_VISIBLE_DEVICES"] for e in envs} == {"1"}
    monkeypatch.setenv("NOS_AMD_BENCH_FOLD_GPUS", "1")
    envs, _ = bench.plan(args, 2, 1, 36, 2, "shared")
    assert {e["HIP_VISIBLE_DEVICES"] for e in envs} == {"0"}  # no GPU here: one visible device


def test_util_sampler_reads_the_rank_gpu_on_a_permuted_node():
    """HIP enumerates the 8 GPUs in another order than amd-smi: the sampler of
    the rank on HIP device h must read the amd-smi index whose hip_id is h."""
    import importlib
    import time

    from nos_amd.gpu.fakesmi import FakeSmi

    sys.path.insert(0, str(REPO))
    bench = importlib.import_module("bench")
    order = [3, 7, 0, 5, 1, 6, 2, 4]  # hip id of amd-smi index i
    smi = FakeSmi(gpus=8, hip_order=order)
    smi.activity_gfx = [10 * (i + 1) for i in range(8)]  # index i reads 10(i+1) %
    for hip in range(8):
        s = bench.UtilSampler(hip, period_s=0.005, smi=smi)
        t0 = time.monotonic()
        time.sleep(0.05)
        s.close()
        idx = order.index(hip)
        assert s.index == idx and s.mean(t0, time.monotonic())[0] == 10 * (idx + 1)
    # the pod-server supervisor starts GPU i's server on GPU i's HIP id
    from nos_amd.cmd.podserver import _gpu_indices

    assert _gpu_indices("all", smi) == [(i, order[i]) for i in range(8)]
    assert _gpu_indices("2,5", smi) == [(2, order[2]), (5, order[5])]


@pytest.mark.timeout(1500)
def test_torchrun_eight_ranks_server_mode_one_socket_per_rank():
    """The driver's 8-GPU launch of the default (server) mode, rehearsed on
    the CPU: 8 ranks, each with its own pod server socket, its pods, and
    slot 0 of every GPU a DP trainer of one world-8 job; one JSON line; no GPU
    ever holds more GPU processes than the HWS limit (rank + server +
    trainer)."""
    lines = _run(8, 29631, pods=2, timeout=1400)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 8 and d["value"] == 16 and d["config"]["mode"] == "server"
    socks = d["pod_server_sockets"]
    assert len(socks) == 8 and len(set(socks)) == 8 and all(s.endswith("/server.sock") for s in socks)
    assert d["trainer_pods"]["rank0"]["running"] and d["trainer_pods"]["per_node_allreduce_gb_per_s"] > 0
    assert d["max_gpu_processes_per_gpu"] <= d["hws_max_concurrent_processes_per_gpu"]
    assert d["max_gpu_processes_per_gpu"] == 3  # this rank + its pod server + the trainer pod
