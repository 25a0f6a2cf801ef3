"""BASELINE config 5 harness (nos_amd/quotabench.py, ``bench.py --quota``):
ElasticQuota borrowing and CapacityScheduling fair-share preemption acting on
running tenants, rehearsed on the CPU.

Reference: victim selection ``pkg/scheduler/plugins/capacityscheduling/
capacity_scheduling.go:468-675``; ``status.used`` and the in-quota /
over-quota labels ``internal/controllers/elasticquota/elasticquota.go:38-72``.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from nos_amd.quotabench import RecordingRuntime, scenario_for

REPO = Path(__file__).resolve().parent.parent


def test_borrow_then_preempt_then_replace_on_a_full_node(tmp_path):
    """28 slice slots: team-a borrows 6 slices past its min, team-b claims its
    min, exactly the 6 borrowed slices are taken back, and at every step the
    EQ status.used and the pod labels describe the tenants actually running."""
    sc = scenario_for(28, pod_server_dir=str(tmp_path))
    rt = RecordingRuntime()
    res = sc.run(rt)
    a = res["phase_a"]
    assert a["ok"] and a["team-a"]["running_pods"] == 20
    assert (a["team-a"]["in_quota"], a["team-a"]["over_quota"]) == (14, 6)
    assert a["team-a"]["status_used_gb"] == a["team-a"]["tenant_gb"] == 200
    assert a["team-a"]["pods_match_tenants"]
    b = res["phase_b"]
    assert b["ok"] and b["preemptions"] == 6 and b["victims"] == 6 and b["victims_over_quota_only"]
    for team in ("team-a", "team-b"):
        t = b[team]
        assert t["running_pods"] == t["tenants_running"] == 14 and t["in_quota"] == 14 and t["over_quota"] == 0
        assert t["status_used_gb"] == t["tenant_gb"] == 140 and t["pods_match_tenants"]
    assert res["concurrent_tenants"] == 28
    # the victims' allocation records are gone (their pod-server tenants get evicted),
    # the 28 running tenants' records remain
    assert len(list((tmp_path / ".allocations" / "gpu-0").glob("*.json"))) == 28
    assert b["preemption_to_running_s"]["n"] == 6


@pytest.mark.timeout(600)
def test_bench_quota_runs_real_pod_processes_against_a_pod_server():
    """``bench.py --quota --device cpu``: the kubelet starts every admitted pod
    as a pod process (numpy-only client) against a CPU pod server; the
    borrowers' processes are stopped by preemption and the lender's pods run."""
    cmd = [sys.executable, "bench.py", "--quota", "--device", "cpu", "--pods-per-gpu", "6"]
    r = subprocess.run(cmd, cwd=REPO, env={**os.environ, "OMP_NUM_THREADS": "1"}, capture_output=True, text=True,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["metric"].startswith("config5")
    assert d["phase_a"]["ok"] and d["phase_a"]["team-a"]["over_quota"] == 1
    b = d["phase_b"]
    assert b["ok"] and b["preemptions"] >= 1 and b["victims"] == 1 and b["victims_over_quota_only"]
    assert b["team-a"]["tenants_running"] == b["team-b"]["tenants_running"] == 3
    assert b["team-b"]["pods_match_tenants"] and b["team-a"]["pods_match_tenants"]
    assert d["concurrent_tenants"] == 6 and d["pod_server"]["device"] == "cpu"


def test_composed_config5_rehearsal_on_an_8gpu_node(tmp_path):
    """config 5 as ONE scenario on an 8-GPU pod-server node
    -- one DP trainer pod per GPU, team-a's tenants in three bursts borrowing
    team-b's quota, pending CPX pods forcing a (simulated) repartition of an
    amdpart node, then team-b claiming its min by preemption."""
    from nos_amd.quotabench import RecordingRuntime, composed_for

    sc = composed_for(8, pod_server_dir=str(tmp_path), part_gpus=2, part_pods=12)
    res = sc.run(RecordingRuntime())
    assert res["phase_trainers"]["ok"] and res["phase_trainers"]["trainers"] == 8
    a = res["phase_a"]
    assert a["ok"] and a["team-a"]["tenants_running"] == sc.team_a_pods and a["team-a"]["over_quota"] > 0
    assert a["team-a"]["status_used_gb"] == a["team-a"]["tenant_gb"] == sc.team_a_pods * 10
    p = res["phase_repartition"]
    assert p["ok"] and p["pods_running"] == 12 and p["mode_switches"] >= 2 and set(p["modes_after"]) == {"CPX"}
    b = res["phase_b"]
    assert b["ok"] and b["victims"] == b["preemptions"] == a["team-a"]["over_quota"] and b["victims_over_quota_only"]
    assert b["team-b"]["tenants_running"] == sc.team_b_pods and b["team-a"]["over_quota"] == 0
    for ns in ("team-a", "team-b"):
        assert b[ns]["status_used_gb"] == b[ns]["tenant_gb"] and b[ns]["pods_match_tenants"]
    assert res["concurrent_tenants"] == 8 + 2 * sc.team_b_pods  # trainers + both teams at their min


@pytest.mark.timeout(600)
def test_bench_quota_composed_runs_trainer_and_tenant_processes():
    cmd = [sys.executable, "bench.py", "--quota", "--composed", "--device", "cpu", "--pods-per-gpu", "6"]
    r = subprocess.run(cmd, cwd=REPO, env={**os.environ, "OMP_NUM_THREADS": "1"}, capture_output=True, text=True,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["metric"].startswith("config5 composed")
    assert d["phase_trainers"]["ok"] and d["phase_a"]["ok"] and d["phase_repartition"]["ok"] and d["phase_b"]["ok"]
    assert d["phase_repartition"]["mode_switches"] == 1 and d["phase_b"]["preemptions"] >= 1
    assert d["concurrent_tenants"] == 7  # the trainer + 3 + 3
    assert "server_footprint_gb" in d["phase_b"]["quota_vs_footprint"]["team-b"]
    # the DP trainer keeps stepping through every phase
    assert all(d[p]["trainer"]["steps"] >= 1 for p in ("phase_a", "phase_b"))


def test_composed_config5_with_an_isolated_team_b_on_an_8gpu_node(tmp_path):
    """team-b on an isolated CU pool (cuPolicy split): its
    slices' masks are disjoint from each other and from the shared pool that
    team-a's tenants and the trainers get, on every GPU; team-a bursts in
    beside it (borrowing the slots team-b leaves)."""
    from nos_amd.bench_support import cus_from_hex
    from nos_amd.quotabench import RecordingRuntime, composed_for

    sc = composed_for(8, pod_server_dir=str(tmp_path), isolate_team_b=True)
    rt = RecordingRuntime()
    res = sc.run(rt)
    assert res["config"]["team_b_isolated"] and res["config"]["team_b_gb"] == 12
    assert res["phase_b_alone"]["ok"] and res["phase_b_alone"]["team-b"]["tenants_running"] == sc.team_b_pods
    a = res["phase_a"]
    assert a["ok"] and a["team-a"]["tenants_running"] == sc.team_a_pods and a["team-a"]["over_quota"] > 0
    started = {k: t.env for k, t in rt.tenants.items()}
    by_gpu: dict[str, dict[str, set]] = {}
    for k, env in started.items():
        if k.startswith(("team-a/", "team-b/")):
            gpu = env["NOS_AMD_POD_SERVER"].rsplit("gpu-", 1)[-1].split("/", 1)[0]
            by_gpu.setdefault(gpu, {})[k] = set(cus_from_hex(env["NOS_AMD_POD_CU_MASK"]))
        elif k.startswith("training/"):
            assert env.get("ROC_GLOBAL_CU_MASK"), "the trainer runs on the shared pool"
    assert len(by_gpu) == 8
    for masks in by_gpu.values():
        shared = [m for k, m in masks.items() if k.startswith("team-a/")]
        iso = [m for k, m in masks.items() if k.startswith("team-b/")]
        assert shared and iso and all(m == shared[0] for m in shared)          # one shared pool
        for i, m in enumerate(iso):
            assert not (m & shared[0]) and all(not (m & o) for o in iso[i + 1:])  # isolated, disjoint
            assert len(m) % 8 == 0                                               # XCD-symmetric


def test_partition_pods_start_as_tenants_and_finish(tmp_path):
    """The repartitioned node's pods also start as (recorded) pod-server
    tenants, then finish before team-b arrives."""
    from nos_amd.quotabench import RecordingRuntime, composed_for

    sc = composed_for(2, pod_server_dir=str(tmp_path), part_gpus=1, part_pods=8,
                      part_tenants=lambda key: {"NOS_AMD_POD_KIND": "partition"})
    rt = RecordingRuntime()
    res = sc.run(rt)
    assert res["phase_repartition"]["ok"] and res["config"]["part_pods_run_as"] == "pod-server tenants"
    parts = [k for k in rt.tenants if k.startswith("part/")]
    assert len(parts) == 8 and not (set(parts) & rt.running())
    assert res["phase_c"]["seconds"] >= 0
    assert not any(k.startswith("team-a/") for k in rt.running())


@pytest.mark.parametrize("gpus", [1, 2])
def test_isolated_team_b_fits_small_nodes(tmp_path, gpus):
    """The isolated variant on the node sizes the GPU bench runs (1 GPU):
    team-a borrows only up to the quotas' total min, so every tenant it
    submits is admitted (CapacityScheduling rejects borrowing past it)."""
    from nos_amd.quotabench import RecordingRuntime, composed_for

    sc = composed_for(gpus, pod_server_dir=str(tmp_path), isolate_team_b=True)
    res = sc.run(RecordingRuntime())
    assert res["phase_b_alone"]["ok"] and res["phase_a"]["ok"] and res["phase_a"]["team-a"]["over_quota"] > 0
    assert res["concurrent_tenants"] == sc.team_a_pods + sc.team_b_pods + gpus
