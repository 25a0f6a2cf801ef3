"""The generated deployment manifests are fresh, parse, and their embedded
component configs load with the same loaders the binaries use."""
from __future__ import annotations

from pathlib import Path

import yaml

from nos_amd.api import config as cfgmod
from nos_amd.cmd import manifests
from nos_amd.gpu import amdpart
from nos_amd.scheduler import config as schedcfg

REPO = Path(__file__).resolve().parent.parent


def test_config_tree_is_fresh():
    assert manifests.main(["--out", str(REPO / "config"), "--check"]) == 0, \
        "run `python -m nos_amd.cmd.manifests --out config`"


def _objs():
    for f in sorted((REPO / "config").rglob("*.yaml")):
        yield from (o for o in yaml.safe_load_all(f.read_text()) if o)


def test_embedded_configs_load(tmp_path):
    kinds = set()
    for o in _objs():
        if o["kind"] != "ConfigMap":
            continue
        for name, text in (o.get("data") or {}).items():
            p = tmp_path / name
            p.write_text(text)
            if name == "scheduler_config.yaml":
                c = schedcfg.load(p)
                assert c.profiles[0].scheduler_name == "nos-scheduler"
                kinds.add("KubeSchedulerConfiguration")
            elif name == "known_partition_geometries.yaml":
                t = amdpart.load_known_geometries(p)
                assert len(t["MI355X"]) == 6
                kinds.add("geometries")
            else:
                c = cfgmod.load(p)
                kinds.add(c.kind)
    assert {"OperatorConfig", "GpuPartitionerConfig", "PartitionAgentConfig", "GpuAgentConfig",
            "DevicePluginConfig", "KubeSchedulerConfiguration", "geometries"} <= kinds


def test_daemonsets_are_privileged_and_node_selected():
    dss = [o for o in _objs() if o["kind"] == "DaemonSet"]
    assert len(dss) == 4
    for ds in dss:
        spec = ds["spec"]["template"]["spec"]
        assert spec["nodeSelector"]["nos.nebuly.com/gpu-partitioning"] in ("partition", "cumask")
        c = spec["containers"][0]
        assert c["securityContext"]["privileged"] is True
        assert any(m["mountPath"] == "/var/lib/kubelet/pod-resources" for m in c["volumeMounts"])
        assert c["env"][0]["name"] == "NODE_NAME"
