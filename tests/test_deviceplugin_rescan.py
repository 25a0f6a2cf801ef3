"""Device plugin on a real cluster:

* ``device_env="container"``: the runtime mounts only the allocated render
  nodes, so HIP inside the container numbers them from 0 -- host HIP ids
  would hide the GPU;
* a mode switched by ANOTHER process (the partition agent) is invisible to the
  plugin's own amd-smi session until it re-enumerates (``nos_smi_rescan``);
* the plugin follows the node's partitioning label instead of reading it once.
Both fakes (native C++ and Python) model the amd-smi session semantics."""
from __future__ import annotations

import pytest

from nos_amd.api import constants as C
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu.amdsmi import ERR_SWITCHING, AmdSmi, AmdSmiError
from nos_amd.gpu.fakesmi import FakeSmi


@pytest.fixture(params=["native", "python"])
def smi8(request):
    if request.param == "native":
        s = AmdSmi.fake(gpus=8)
        yield s
        s.close()
    else:
        yield FakeSmi(gpus=8, node="n")


def test_container_env_renumbers_visible_devices(smi8):
    plugin = NosAmdDevicePlugin("n", smi8, device_env="container")
    devs = {d.gpu_index: d for d in plugin.list_devices(C.RESOURCE_AMD_GPU)}
    a = plugin.allocate(C.RESOURCE_AMD_GPU, [devs[5].id], owner="pod-a")
    render5 = smi8.gpu(5).drm_render
    assert a.envs[C.ENV_VISIBLE_DEVICES] == "0"
    assert a.devices == ["/dev/kfd", f"/dev/dri/renderD{render5}"]
    b = plugin.allocate(C.RESOURCE_AMD_GPU, [devs[6].id, devs[3].id], owner="pod-b")
    assert b.envs[C.ENV_VISIBLE_DEVICES] == "0,1" and len(b.devices) == 3
    # host numbering (bare metal / simulator) keeps the host HIP ids
    host = NosAmdDevicePlugin("n", smi8, device_env="host")
    h = host.allocate(C.RESOURCE_AMD_GPU, [devs[5].id], owner="pod-c")
    assert h.envs[C.ENV_VISIBLE_DEVICES] == str(smi8.gpu(5).hip_id)


def test_container_env_for_a_partition(smi8):
    smi8.set_compute_partition(2, "CPX")
    plugin = NosAmdDevicePlugin("n", smi8, mode=C.PARTITIONING_AMDPART, device_env="container")
    d = next(x for x in plugin.list_devices("amd.com/partition-1xcd.36gb") if x.partition == 3)
    a = plugin.allocate("amd.com/partition-1xcd.36gb", [d.id], owner="p")
    assert a.envs[C.ENV_VISIBLE_DEVICES] == "0"
    assert a.devices[1] == f"/dev/dri/renderD{smi8.partitions(2)[3].drm_render}"


def test_external_mode_switch_is_invisible_until_rescan(smi8):
    plugin = NosAmdDevicePlugin("n", smi8, mode=C.PARTITIONING_AMDPART)
    assert len(plugin.list_devices("amd.com/partition-8xcd.288gb")) == 8
    smi8.inject("external_switch=5:CPX")  # the partition agent's process switched GPU 5
    plugin.refresh()
    assert smi8.gpu(5).compute_mode == "SPX"  # this session still sees its enumeration
    assert not plugin.list_devices("amd.com/partition-1xcd.36gb")
    plugin.rescan()
    assert smi8.gpu(5).compute_mode == "CPX"
    assert len(plugin.list_devices("amd.com/partition-1xcd.36gb")) == 8
    assert len(plugin.list_devices("amd.com/partition-8xcd.288gb")) == 7
    # HIP ids are GPU-major after the re-enumeration: GPU 6 follows GPU 5's 8 partitions
    assert smi8.gpu(6).hip_id == 5 + 8


def test_plugin_follows_the_partitioning_label(smi8):
    plugin = NosAmdDevicePlugin("n", smi8, mode=None)
    assert set(plugin.resources()) == {C.RESOURCE_AMD_GPU}
    assert plugin.set_mode(C.PARTITIONING_AMDPART)
    assert set(plugin.resources()) == {"amd.com/partition-8xcd.288gb"}
    assert not plugin.set_mode(C.PARTITIONING_AMDPART)  # unchanged
    assert plugin.set_mode(C.PARTITIONING_CUMASK)
    plugin.set_config("n-1", {"gpus": [{"index": 0, "slices": [{"profile": "36gb", "replicas": 2}]}]})
    assert len(plugin.list_devices("amd.com/gpu-36gb")) == 2
    assert plugin.set_mode(None) and plugin.config is None


def test_switch_in_flight_does_not_block_other_gpus(smi8):
    """The slow part of a switch runs without the library lock: other GPUs keep
    answering, the switching GPU reports ERR_SWITCHING (gpus() serves its last
    known state flagged ``switching``), rescan is deferred."""
    import threading
    import time

    smi8.gpus()
    smi8.inject("switch_delay_ms=400")
    t = threading.Thread(target=smi8.set_compute_partition, args=(1, "DPX"))
    t.start()
    time.sleep(0.1)
    t0 = time.monotonic()
    assert smi8.gpu(2).compute_mode == "SPX" and time.monotonic() - t0 < 0.1
    with pytest.raises(AmdSmiError) as e:
        smi8.gpu(1)
    assert e.value.rc == ERR_SWITCHING
    g1 = next(g for g in smi8.gpus() if g.index == 1)
    assert g1.switching and g1.compute_mode == "SPX"
    with pytest.raises(AmdSmiError):
        smi8.rescan()
    plugin = NosAmdDevicePlugin("n", smi8, mode=C.PARTITIONING_AMDPART)  # keeps enumerating the others
    assert len(plugin.list_devices("amd.com/partition-8xcd.288gb")) == 7
    t.join()
    smi8.inject("clear")
    assert smi8.gpu(1).compute_mode == "DPX" and not smi8.gpus()[1].switching
