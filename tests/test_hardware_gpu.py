"""The real device path on an MI355X (weakness 3: "nothing
exercises the real device path" in the reference).

* libnos_amdsmi against the real amd-smi: read-only queries a partition agent
  and the device plugin depend on (mode, XCDs/CUs, VRAM, activity, processes);
* the device plugin on the real GPU: a CU-mask slice allocation's
  ``ROC_GLOBAL_CU_MASK`` is handed to a child process (as the kubelet hands it
  to a container) and the gfx950 placement probe, run inside that process,
  must see exactly the slice's CUs on every XCD.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest
import torch

from nos_amd.api import constants as C

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _smi():
    from nos_amd.gpu.amdsmi import AmdSmi

    return AmdSmi.real()


def _local_gpu(smi):
    """The amd-smi GPU that is HIP device 0 of this process."""
    gpus = smi.gpus()
    for g in gpus:
        if g.hip_id == 0:
            return g
    return gpus[0]


def test_amdsmi_real_partitions_map_to_physical_gpus():
    """Physical GPUs vs logical devices: every amd-smi processor handle is a
    partition of exactly one physical GPU, HIP ids are unique, and (SPX) each
    GPU's single partition is the GPU itself with its whole memory/CUs."""
    smi = _smi()
    try:
        gpus = smi.gpus()
        hip_ids = []
        for g in gpus:
            parts = smi.partitions(g.index)
            assert len(parts) == g.num_partitions, (g, parts)
            assert sum(p.num_cus for p in parts) == g.num_cus, parts
            assert all(p.gpu_index == g.index for p in parts)
            if len(parts) == 1:
                assert parts[0].hip_id == g.hip_id and parts[0].memory_gb == g.memory_gb, (g, parts[0])
            hip_ids += [p.hip_id for p in parts]
        assert len(set(hip_ids)) == len(hip_ids)
        visible = torch.cuda.device_count()
        assert set(range(visible)) <= set(hip_ids) or len(hip_ids) >= visible, (hip_ids, visible)
    finally:
        smi.close()


def test_amdsmi_real_rescan_keeps_the_handle_to_hip_id_mapping():
    """nos_smi_rescan (the device plugin's poll) shuts the amd-smi session down
    and enumerates again: the same physical GPUs, partitions and HIP ids /
    render nodes must come back (no mode changed in between)."""
    smi = _smi()
    try:
        def snapshot():
            return [(g.index, g.uuid, g.bdf, g.hip_id, g.drm_render, g.compute_mode,
                     tuple((p.partition, p.hip_id, p.drm_render) for p in smi.partitions(g.index)))
                    for g in smi.gpus()]

        before = snapshot()
        smi.rescan()
        after = snapshot()
        assert before == after
        assert all(not g.switching for g in smi.gpus())
    finally:
        smi.close()


def test_amdsmi_real_readonly_queries():
    smi = _smi()
    try:
        assert smi.count() >= 1
        g = _local_gpu(smi)
        assert g.num_xcds == 8 and g.num_cus == 256, g
        assert g.compute_mode in ("SPX", "DPX", "QPX", "CPX"), g
        assert g.memory_mode.startswith("NPS"), g
        assert 250 <= g.memory_gb <= 300, g   # 288 GB HBM3E
        assert g.uuid and g.bdf, g
        act = smi.activity(g.index)
        assert 0 <= act["gfx"] <= 100 and 0 <= act["umc"] <= 100, act
        torch.ones(1, device="cuda").sum().item()  # this process now holds a GPU context
        procs = smi.processes(g.index)
        assert isinstance(procs, list)
    finally:
        smi.close()


def test_device_plugin_slice_mask_is_enforced_in_a_child_process():
    from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin

    smi = _smi()
    try:
        g = _local_gpu(smi)
        plugin = NosAmdDevicePlugin("node", smi, mode=C.PARTITIONING_CUMASK, cu_policy="even")
        plugin.set_config("node-1", {"cuPolicy": "even", "allocation": "pack", "gpus": [
            {"index": g.index, "slices": [{"profile": "10gb", "memoryGB": 10, "replicas": 4}]}]})
        res = "amd.com/gpu-10gb"
        devs = [d.id for d in plugin.list_devices(res)]
        assert len(devs) == 4
        pick = plugin.preferred_allocation(res, devs, [], 1)
        alloc = plugin.allocate(res, pick, owner="pod-a")
        mask = alloc.envs[C.ENV_CU_MASK]
        assert alloc.envs[C.ENV_VISIBLE_DEVICES] == str(g.index)
        expect = set(plugin.cus_of(pick[0]))
        assert len(expect) == 64   # 4 slices of a 256-CU GPU, 8 CUs on each XCD
    finally:
        smi.close()
    # the mask is process-wide (HIP runtime): the default stream, a stream the
    # tenant creates later and a high-priority one (as RCCL's internal streams
    # are) must all stay on the slice's CUs
    code = (
        "import json, sys, torch; sys.path.insert(0, %r)\n"
        "from nos_amd.ops import probes\n"
        "out = [probes.placement_summary(probes.placement(nwg=4096))]\n"
        "for s in (torch.cuda.Stream(), torch.cuda.Stream(priority=-1)):\n"
        "    out.append(probes.placement_summary(probes.placement(stream=s.cuda_stream, nwg=4096)))\n"
        "print(json.dumps(out))\n" % REPO)
    env = dict(os.environ)
    env[C.ENV_CU_MASK] = mask   # what the kubelet puts in the container's environment
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    for summary in json.loads(out.stdout.strip().splitlines()[-1]):
        assert summary["distinct_cus"] == 64, summary
        assert summary["cus_per_xcc"] == {str(x): 8 for x in range(8)} or \
            summary["cus_per_xcc"] == {x: 8 for x in range(8)}, summary


def test_trainer_pod_step_on_gpu_overlaps_bucket_launches_with_backward():
    """The DP trainer pod on the GPU (world 1): forward + backward with the
    gradient hooks driving the bucketed collective path on a side stream, then
    SGD; the loss falls and every bucket was started from inside backward."""
    from nos_amd.models.tenants import CollectiveTenant

    t = CollectiveTenant(dim=512, bucket_mb=1, device=0, layers=4, batch=256)
    assert len(t.bucketer.buckets) >= 2
    w0 = [m.weight.detach().clone() for m in t.model]
    losses = []
    for _ in range(3):
        with torch.no_grad():
            losses.append(t.model(t.x).float().square().mean().item())
        t.step()
    torch.cuda.synchronize()
    assert t.bucketer.launched_in_backward == 3 * len(t.bucketer.buckets)
    assert all(not torch.equal(a, m.weight) for a, m in zip(w0, t.model))
    assert losses[-1] < losses[0]
    assert t.flops_per_step() == 6.0 * 256 * 512 * 512 * 4


def test_slice_prober_prices_slices_on_their_cu_slots():
    """The gpuagent's slice probe on the real GPU: a 36 GB slice (4 CUs per XCD)
    against the whole GPU, idle and (for the slice) under co-tenant load on the
    complement CUs.  More CUs must price higher; the loaded numbers exist."""
    from nos_amd.agents.probe import METRICS, SliceProber

    smi = _smi()
    prober = SliceProber(smi, iters=2000, loaded=True)
    small = prober(0, "36gb")
    whole = SliceProber(smi, iters=2000, loaded=False)(0, "288gb")
    assert small["cus"] == 32 and whole["cus"] == 256
    for k in ("tflops", "gemmtflops", "gbps"):
        assert small[k] > 0 and whole[k] > 0, k
    assert whole["gemmtflops"] > 3 * small["gemmtflops"]
    assert whole["tflops"] > 3 * small["tflops"]
    assert small["loadedgbps"] > 0 and small["loadedgemmtflops"] > 0
    assert set(small) >= set(METRICS)
