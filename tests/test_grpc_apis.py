"""Device-plugin v1beta1 and PodResources v1 over real gRPC unix sockets."""
from __future__ import annotations

import yaml

from nos_amd.api import constants as C
from nos_amd.deviceplugin.grpc_server import DevicePluginServers, endpoint_name
from nos_amd.deviceplugin.plugin import NosAmdDevicePlugin
from nos_amd.gpu.fakesmi import FakeSmi
from nos_amd.grpcapi.protos import deviceplugin as dp
from nos_amd.resource.client import ContainerDevices, ContainerResources, PodResources
from nos_amd.resource.podresources_grpc import GrpcLister, serve
from nos_amd.sim.kubelet_grpc import DeviceManager


def _slice_cfg(plan: str, slices: dict[int, int]) -> str:
    return yaml.safe_dump({"version": "v1", "planId": plan, "cuPolicy": "proportional", "allocation": "spread",
                           "gpus": [{"index": g, "slices": [{"profile": "10gb", "memoryGB": 10, "replicas": n}]}
                                    for g, n in slices.items()]})


def test_messages_roundtrip_on_the_wire():
    r = dp.ContainerAllocateResponse(envs={"ROC_GLOBAL_CU_MASK": "0xff"},
                                     devices=[dp.DeviceSpec(container_path="/dev/kfd", host_path="/dev/kfd")])
    back = dp.ContainerAllocateResponse.FromString(r.SerializeToString())
    assert back.envs["ROC_GLOBAL_CU_MASK"] == "0xff" and back.devices[0].host_path == "/dev/kfd"
    assert endpoint_name("amd.com/gpu-10gb") == "nos-amd-gpu-10gb.sock"


def test_device_plugin_lifecycle_against_kubelet(tmp_path):
    km = DeviceManager(tmp_path)
    plugin = NosAmdDevicePlugin("n1", FakeSmi(gpus=2, node="n1"), mode=C.PARTITIONING_CUMASK)
    servers = DevicePluginServers(plugin, tmp_path)
    try:
        plugin.set_config("n1-1", _slice_cfg("1", {0: 2, 1: 2}))
        servers.sync()
        res = "amd.com/gpu-10gb"
        assert km.wait_for(lambda: len(km.healthy(res)) == 4)
        a = km.allocate(res, 1)
        b = km.allocate(res, 1)
        # spread: the two pods land on different GPUs, each with its own CU mask
        assert {a["envs"][C.ENV_VISIBLE_DEVICES], b["envs"][C.ENV_VISIBLE_DEVICES]} == {"0", "1"}
        assert a["envs"][C.ENV_CU_MASK] and a["devices"][0] == "/dev/kfd"
        # a new plan re-advertises through ListAndWatch, no restart
        plugin.set_config("n1-2", _slice_cfg("2", {0: 4, 1: 4}))
        servers.sync()
        assert km.wait_for(lambda: len(km.healthy(res)) == 8)
        # a plan without slices: the two devices still in use stay, unhealthy, until released
        plugin.set_config("n1-3", yaml.safe_dump({"gpus": []}))
        servers.sync()
        assert km.wait_for(lambda: km.healthy(res) == [] and len(km.endpoints[res].devices) == 2)
        plugin.sync_allocated(set())  # PodResources: the pods are gone
        plugin.refresh()
        servers.sync()
        assert res not in servers.servers
    finally:
        servers.stop()
        km.stop()


def test_podresources_grpc_roundtrip(tmp_path):
    class L:
        def list(self):
            return [PodResources("p", "ns", [ContainerResources("c", [ContainerDevices("amd.com/gpu", ["g0"])])])]

        def get_allocatable_resources(self):
            return [ContainerDevices("amd.com/gpu", ["g0", "g1"])]

    srv = serve(L(), tmp_path / "kubelet.sock")
    try:
        cl = GrpcLister(tmp_path / "kubelet.sock")
        pr = cl.list()
        assert pr[0].name == "p" and pr[0].containers[0].devices[0].device_ids == ["g0"]
        assert cl.get_allocatable_resources()[0].device_ids == ["g0", "g1"]
        cl.close()
    finally:
        srv.stop(grace=0)
