"""Logical partitions vs physical GPUs (libnos_amdsmi + device plugin + labeler).

In DPX/QPX/CPX amd-smi enumerates one processor handle per partition; the
library groups them back into physical GPUs (the reference resolves MIG
devices to their parent GPU: pkg/gpu/nvml/client.go:59-146)."""
from __future__ import annotations

import pytest

from nos_amd.agents.devices import node_labels
from nos_amd.api import constants as C
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu import amdpart
from nos_amd.gpu.amdsmi import AmdSmi
from nos_amd.gpu.fakesmi import FakeSmi


@pytest.fixture(params=["native", "python"])
def cpx_node(request):
    if request.param == "native":
        smi = AmdSmi.fake(gpus=8, compute="CPX")
        yield smi
        smi.close()
    else:
        yield FakeSmi(gpus=8, compute="CPX", node="n")


def test_cpx_node_counts_physical_gpus(cpx_node):
    smi = cpx_node
    assert smi.count() == 8
    labels = node_labels(smi)
    assert labels[C.LABEL_AMD_COUNT] == "8" and labels[C.LABEL_AMD_COMPUTE_MODE] == "CPX"
    hip = []
    for g in smi.gpus():
        parts = smi.partitions(g.index)
        assert len(parts) == 8 and g.num_partitions == 8
        assert [p.partition for p in parts] == list(range(8))
        assert all(p.num_xcds == 1 and p.num_cus == 32 and p.memory_gb == 36 and p.memory_shared for p in parts)
        assert parts[0].hip_id == g.hip_id  # a GPU's HIP id is its first logical device's
        hip += [p.hip_id for p in parts]
    assert hip == list(range(64))  # GPU-major enumeration


def test_device_plugin_exposes_one_device_per_partition(cpx_node):
    plugin = NosAmdDevicePlugin("n", cpx_node, mode=C.PARTITIONING_AMDPART)
    devs = plugin.list_devices("amd.com/partition-1xcd.36gb")
    assert len(devs) == 64
    d = next(x for x in devs if x.gpu_index == 2 and x.partition == 3)
    alloc = plugin.allocate("amd.com/partition-1xcd.36gb", [d.id], owner="pod")
    assert alloc.envs[C.ENV_VISIBLE_DEVICES] == "19"
    assert "/dev/dri/renderD147" in alloc.devices and alloc.envs[C.ENV_MEMORY_LIMIT_GB] == "36"


def test_static_cpx_partitions_as_amd_gpu(cpx_node):
    """BASELINE config 2: static CPX, every partition is an amd.com/gpu."""
    plugin = NosAmdDevicePlugin("n", cpx_node, mode=C.PARTITIONING_AMDPART, expose_partitions_as_gpu=True)
    assert len(plugin.list_devices(C.RESOURCE_AMD_GPU)) == 64


def test_mixed_modes_enumerate_gpu_major():
    smi = FakeSmi(gpus=3, node="n")
    smi.compute = ["CPX", "DPX", "SPX"]
    parts = [smi.partitions(i) for i in range(3)]
    assert [p.hip_id for p in parts[1]] == [8, 9] and parts[2][0].hip_id == 10
    assert [p.memory_gb for p in parts[1]] == [144, 144]
    plugin = NosAmdDevicePlugin("n", smi, mode=C.PARTITIONING_AMDPART)
    res = plugin.resources()
    assert {k: len(v) for k, v in res.items()} == {"amd.com/partition-1xcd.36gb": 8,
                                                 "amd.com/partition-4xcd.144gb": 2,
                                                 "amd.com/partition-8xcd.288gb": 1}


def test_native_fake_matches_python_fake():
    smi = AmdSmi.fake(gpus=3, compute="QPX")
    try:
        py = FakeSmi(gpus=3, compute="QPX", node="x")
        for i in range(3):
            a = [(p.hip_id, p.num_cus, p.num_xcds, p.vram_mb, p.memory_shared) for p in smi.partitions(i)]
            b = [(p.hip_id, p.num_cus, p.num_xcds, p.vram_mb, p.memory_shared) for p in py.partitions(i)]
            assert a == b
    finally:
        smi.close()


def test_geometries_follow_reported_memory():
    """No hard-coded 288 GB: a GPU reporting 256 GB yields 32 GB CPX partitions,
    and the device plugin names them the same way."""
    gs = amdpart.get_allowed_geometries("AMD Instinct MI355X", memory_mb=262144, xcds=8)
    profs = {str(p) for g in gs for p in g.geometry}
    assert profs == {"8xcd.256gb", "4xcd.128gb", "2xcd.64gb", "1xcd.32gb"}
    smi = FakeSmi(gpus=1, compute="CPX", vram_mb=262144, node="n")
    plugin = NosAmdDevicePlugin("n", smi, mode=C.PARTITIONING_AMDPART)
    assert set(plugin.resources()) == {"amd.com/partition-1xcd.32gb"}
    assert amdpart.get_allowed_geometries("unknown-gpu") is None
