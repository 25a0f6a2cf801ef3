"""Node actuation of a partitioning plan by the gpupartitioner's strategies
against the in-process API server -- the role of the reference's fake-client
tests (``internal/partitioning/{mig,mps}/partitioner_test.go``): which
annotations and ConfigMap keys a plan writes, which stale ones it removes, and
the enforced device-plugin propagation delay (on a fake clock)."""
from __future__ import annotations

import yaml

from nos_amd.api import constants as C
from nos_amd.kube import factory as kf
from nos_amd.partitioning.state import GPUPartitioning, NodePartitioning
from nos_amd.partitioning.strategies import AmdPartPartitioner, CuMaskPartitioner, DevicePluginConfigRef
from nos_amd.sim.apiserver import ApiServer
from nos_amd.utils.clock import FakeClock


def _node(api: ApiServer, name: str, ann: dict | None = None) -> dict:
    n = kf.build_node(name).with_labels({C.LABEL_GPU_PARTITIONING: "cumask", "amd.com/gpu.count": "2"}) \
        .with_annotations(ann or {}).get()
    return api.create(n)


def test_cumask_partitioner_writes_config_map_key_annotations_and_label_after_the_delay():
    clock = FakeClock()
    api = ApiServer(clock=clock)
    ref = DevicePluginConfigRef()
    node = _node(api, "n1", {"nos.nebuly.com/spec-gpu-0-10gb": "3", "nos.nebuly.com/spec-gpu-1-20gb": "1",
                             "unrelated": "keep"})
    _node(api, "n2")
    # another node's key and this node's previous plan already in the ConfigMap
    api.create({"kind": "Namespace", "metadata": {"name": ref.namespace}})
    api.create({"kind": "ConfigMap", "metadata": {"name": ref.name, "namespace": ref.namespace},
                "data": {"n2-100": "x", "n1-050": "old"}})
    part = NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-36gb": 2}),
                             GPUPartitioning.of(1, {"amd.com/gpu-72gb": 1, "amd.com/gpu-36gb": 1})])
    t0 = clock.now()
    CuMaskPartitioner(api, ref, delay_s=5.0, clock=clock).apply_partitioning(node, "101", part)
    assert clock.now() - t0 == 5.0  # the enforced ConfigMap propagation delay
    cmap = api.get("ConfigMap", ref.name, ref.namespace)
    assert set(cmap["data"]) == {"n2-100", "n1-101"}  # the node's stale key removed, other nodes kept
    cfg = yaml.safe_load(cmap["data"]["n1-101"])
    assert cfg  # the device plugin's per-plan config for this node
    n1 = api.get("Node", "n1")
    ann = n1["metadata"]["annotations"]
    assert ann[C.ANNOTATION_PARTITIONING_PLAN] == "101"
    assert ann["nos.nebuly.com/spec-gpu-0-36gb"] == "2"
    assert ann["nos.nebuly.com/spec-gpu-1-72gb"] == "1" and ann["nos.nebuly.com/spec-gpu-1-36gb"] == "1"
    assert "nos.nebuly.com/spec-gpu-0-10gb" not in ann and "nos.nebuly.com/spec-gpu-1-20gb" not in ann
    assert ann["unrelated"] == "keep"
    assert n1["metadata"]["labels"][C.LABEL_DEVICE_PLUGIN_CONFIG] == "n1-101"
    # the other node is untouched
    assert C.ANNOTATION_PARTITIONING_PLAN not in (api.get("Node", "n2")["metadata"].get("annotations") or {})


def test_cumask_partitioner_creates_the_namespace_and_config_map_when_missing():
    clock = FakeClock()
    api = ApiServer(clock=clock)
    node = _node(api, "n1")
    ref = DevicePluginConfigRef(name="dp-cfg", namespace="nos-dp")
    CuMaskPartitioner(api, ref, delay_s=0, clock=clock).apply_partitioning(
        node, "7", NodePartitioning([GPUPartitioning.of(0, {"amd.com/gpu-36gb": 8})]))
    assert api.try_get("Namespace", "nos-dp") is not None
    assert set(api.get("ConfigMap", "dp-cfg", "nos-dp")["data"]) == {"n1-7"}


def test_amdpart_partitioner_writes_geometry_and_mode_annotations_only():
    api = ApiServer(clock=FakeClock())
    node = _node(api, "n1", {"nos.nebuly.com/spec-gpu-0-1xcd.36gb": "8", C.ANNOTATION_SPEC_MODE_FORMAT.format(index=1):
                             "CPX/NPS1"})
    part = NodePartitioning([GPUPartitioning.of(0, {"amd.com/partition-2xcd.72gb": 4}, "DPX/NPS1"),
                             GPUPartitioning.of(1, {"amd.com/partition-8xcd.288gb": 1}, "")])
    AmdPartPartitioner(api).apply_partitioning(node, "55", part)
    ann = api.get("Node", "n1")["metadata"]["annotations"]
    assert ann[C.ANNOTATION_PARTITIONING_PLAN] == "55"
    assert ann["nos.nebuly.com/spec-gpu-0-2xcd.72gb"] == "4" and ann["nos.nebuly.com/spec-gpu-1-8xcd.288gb"] == "1"
    assert ann[C.ANNOTATION_SPEC_MODE_FORMAT.format(index=0)] == "DPX/NPS1"
    # the stale spec and the mode of a GPU whose plan names none are removed
    assert "nos.nebuly.com/spec-gpu-0-1xcd.36gb" not in ann
    assert C.ANNOTATION_SPEC_MODE_FORMAT.format(index=1) not in ann
    assert api.try_get("ConfigMap", C.DEFAULT_DEVICE_PLUGIN_CM_NAME, C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE) is None
