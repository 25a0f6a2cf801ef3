"""Pod-process measurement protocol (nos_amd/podbench.py, nos_amd/models/pod.py).

The pods run the tiny YOLOS test config on the CPU here; on a GPU box the same
protocol runs the fp32 YOLOS-small pods of bench.py."""
import os
import time

import pytest

from nos_amd.podbench import PodFleet, PodLauncher, WindowStats, PodResult, progress


def test_progress_interpolates_between_completions():
    times = [1.0, 2.0, 4.0]
    assert progress(times, 0.0, 0.0) == 0.0
    assert progress(times, 0.5, 0.0) == pytest.approx(0.5)
    assert progress(times, 1.0, 0.0) == pytest.approx(1.0)
    assert progress(times, 3.0, 0.0) == pytest.approx(2.5)
    assert progress(times, 9.0, 0.0) == 3.0
    # the count inside a window is additive over sub-windows
    a = progress(times, 3.0, 0.0) - progress(times, 0.7, 0.0)
    b = progress(times, 1.9, 0.0) - progress(times, 0.7, 0.0)
    c = progress(times, 3.0, 0.0) - progress(times, 1.9, 0.0)
    assert a == pytest.approx(b + c)


def test_window_latency_identity():
    w = WindowStats(10.0, [PodResult(0, 50.0, 0.2, 0.3, True), PodResult(1, 25.0, 0.4, 0.5, True)])
    # mean per-request latency: pods / latency == throughput exactly
    assert w.throughput == pytest.approx(7.5)
    assert len(w.pods) / w.mean_latency_s == pytest.approx(w.throughput)
    assert w.concurrent == 2


@pytest.mark.timeout(300)
@pytest.mark.parametrize("use_launcher", [True, False])
def test_cpu_pod_fleet_end_to_end(tmp_path, use_launcher):
    launcher = PodLauncher() if use_launcher else None
    envs = [{"NOS_AMD_MEMORY_LIMIT_GB": "10", "HIP_VISIBLE_DEVICES": "0"} for _ in range(3)]
    fleet = PodFleet(envs, dtype="fp32", workdir=str(tmp_path), device="cpu", launcher=launcher,
                     extra_env={"OMP_NUM_THREADS": "1"})
    try:
        fleet.start()
        fleet.wait_ready(timeout_s=240)
        time.sleep(0.3)
        t0 = time.monotonic()
        time.sleep(1.5)
        t1 = time.monotonic()
        time.sleep(0.3)
        fleet.stop()
        w = fleet.window(t0, t1)
    finally:
        fleet.close()
        if launcher:
            launcher.close()
    assert len(w.pods) == 3
    for p in w.pods:
        assert p.completed > 1, p
        assert p.info["memory_limit_gb"] == "10"
        assert p.info["hip_visible_devices"] == "0"
    assert w.concurrent == 3
    assert len(w.pods) / w.mean_latency_s == pytest.approx(w.throughput)


def test_failed_pod_is_reported(tmp_path):
    fleet = PodFleet([{}], dtype="nope", workdir=str(tmp_path), device="cpu")
    try:
        fleet.start()
        with pytest.raises(RuntimeError, match="pod 0 failed"):
            fleet.wait_ready(timeout_s=120)
    finally:
        fleet.close()


def test_running_criterion_allows_bursty_idle_at_the_window_end(tmp_path):
    """A bursty pod may be idle when the window closes; one that stopped for
    more than a quarter of the window is not counted as running."""
    fleet = PodFleet([{}, {}, {}], workdir=str(tmp_path))
    t0, t1 = 100.0, 112.0
    steady = [99.0 + 0.1 * k for k in range(140)]                    # through t1
    bursty = [t for t in steady if (t - 99.0) % 2.0 < 1.0]           # 1 s on / 1 s off, idle at t1
    stopped = [t for t in steady if t < 106.0]                        # silent for the last 6 s
    fleet.results = {0: {"times": steady}, 1: {"times": bursty}, 2: {"times": stopped}}
    w = fleet.window(t0, t1)
    assert [p.running for p in w.pods] == [True, True, False]
    assert w.concurrent == 2


def _alive(pid: int) -> bool:
    """Running (not gone, not a zombie nobody reaped yet)."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except FileNotFoundError:
        return False


def _wait_gone(pids, timeout_s=30.0) -> list[int]:
    deadline = time.monotonic() + timeout_s
    while time.monotonic() < deadline:
        left = [p for p in pids if _alive(p)]
        if not left:
            return []
        time.sleep(0.1)
    return [p for p in pids if _alive(p)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("how", ["orchestrator_exits", "launcher_killed"])
def test_pods_do_not_outlive_the_orchestrator(tmp_path, how):
    """A bench killed at its time limit must not leave pods running kernels on
    the GPU: the launcher kills its pods when its stdin closes, and a pod whose
    launcher dies gets SIGTERM (PR_SET_PDEATHSIG) / sees its parent change."""
    import signal

    launcher = PodLauncher()
    fleet = PodFleet([{}, {}], dtype="fp32", workdir=str(tmp_path), device="cpu", launcher=launcher,
                     extra_env={"OMP_NUM_THREADS": "1"})
    try:
        fleet.start()
        fleet.wait_ready(timeout_s=240)
        pids = [int(fleet.board.row(i)[3]) for i in range(2)]
        assert all(_alive(p) for p in pids)
        if how == "orchestrator_exits":
            launcher.p.stdin.close()  # what the orchestrator's death looks like to the launcher
        else:
            launcher.p.send_signal(signal.SIGKILL)
        launcher.p.wait(timeout=30)
        assert _wait_gone(pids) == []
    finally:
        for p in [int(fleet.board.row(i)[3]) for i in range(2)] if fleet.board is not None else []:
            if p and _alive(p):
                os.kill(p, signal.SIGKILL)


def test_pod_kernel_config_follows_the_slice():
    from nos_amd.models.pod import kernel_config

    whole = kernel_config(None, {})
    assert whole == {"gemm_bf16": "latency", "gemm_f32": "latency", "attention_f32": "h3", "f32_math": "h3",
                     "gemm_f32x6_tile": "policy", "ln_handoff": "on", "h3_epilogue": "lds", "h3_layout": "2x2", "h3_hot_ring": "2", "h3_hot_bn": "128", "h3_lna_wide": "off"}
    assert kernel_config(1.0, {}) == whole
    frac = kernel_config(36 / 288, {})
    assert frac == {"gemm_bf16": "throughput", "gemm_f32": "small", "attention_f32": "h3n", "f32_math": "h3",
                    "gemm_f32x6_tile": "128x128", "ln_handoff": "on",
                                                         "h3_epilogue": "lds", "h3_layout": "2x2", "h3_hot_ring": "2", "h3_hot_bn": "128", "h3_lna_wide": "off"}
    # an exclusive CU-mask slice plans for its own CUs (budget-aware tiles)
    assert kernel_config(36 / 288, {}, cu_budget=32) == {"gemm_bf16": "throughput", "gemm_f32": "latency",
                                                         "attention_f32": "h3n", "f32_math": "h3",
                                                         "gemm_f32x6_tile": "128x128", "ln_handoff": "on",
                                                         "h3_epilogue": "lds", "h3_layout": "2x2", "h3_hot_ring": "2", "h3_hot_bn": "128", "h3_lna_wide": "off"}
    assert kernel_config(None, {}, cu_budget=32) == whole
    # A/B overrides win over the slice rule: the exact-f32 MFMA kernels stay selectable
    assert kernel_config(0.125, {"NOS_AMD_ATTN_F32_VARIANT": "w4k64"})["attention_f32"] == "w4k64"
    assert kernel_config(0.125, {"NOS_AMD_F32_MATH": "exact"})["f32_math"] == "exact"
    # every name is one the native library accepts
    from nos_amd import ops
    import inspect

    src = (inspect.getsource(ops.set_attention_f32_variant) + inspect.getsource(ops.set_gemm_f32_policy)
           + inspect.getsource(ops.set_f32_math) + inspect.getsource(ops.set_gemm_f32x6_tile) + inspect.getsource(ops.set_gemm_f32h3_layout))
    for v in (*whole.values(), *frac.values()):
        assert f'"{v}"' in src or v in ("latency", "throughput", "on", "off", "lds", "reg", "2", "128")
