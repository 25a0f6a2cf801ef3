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
    for f in sorted(p for p in (REPO / "config").rglob("*.yaml") if p.name != "values.yaml"):
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
            "DevicePluginConfig", "KubeSchedulerConfiguration"} <= kinds
    # no fixed geometry table by default: the planner derives geometries from each node's amd-smi memory
    assert "geometries" not in kinds


def test_known_geometries_override_is_rendered(tmp_path):
    table = [{"models": ["MI355X"], "allowedGeometries": [{"compute": "CPX", "memory": "NPS1",
                                                          "profiles": {"1xcd.36gb": 8}}]}]
    out = manifests.render({"gpuPartitioner": {"knownPartitionGeometries": table}})
    cms = {k: t for o in yaml.safe_load_all(out["gpupartitioner/manager.yaml"]) if o and o["kind"] == "ConfigMap"
           for k, t in (o.get("data") or {}).items()}
    p = tmp_path / "g.yaml"
    p.write_text(cms["known_partition_geometries.yaml"])
    assert len(amdpart.load_known_geometries(p)["MI355X"]) == 1
    assert yaml.safe_load(cms["gpu_partitioner_config.yaml"])["knownPartitionGeometriesFile"]


def test_every_referenced_secret_certificate_and_service_is_rendered():
    """Nothing a workload, webhook or monitor points at is left for the user to create."""
    objs = [o for o in _objs() if "metadata" in o]
    by_kind: dict = {}
    for o in objs:
        by_kind.setdefault(o["kind"], {})[o["metadata"]["name"]] = o
    certs = by_kind.get("Certificate", {})
    secrets_made = {c["spec"]["secretName"] for c in certs.values()} | set(by_kind.get("Secret", {}))
    pods = [w["spec"]["template"] for k in ("Deployment", "DaemonSet") for w in by_kind.get(k, {}).values()]
    for t in pods:
        for v in t["spec"].get("volumes", []):
            if "secret" in v:
                assert v["secret"]["secretName"] in secrets_made, v
    for vwc in by_kind.get("ValidatingWebhookConfiguration", {}).values():
        ns_name = vwc["metadata"]["annotations"]["cert-manager.io/inject-ca-from"]
        assert ns_name.split("/")[1] in certs
        for h in vwc["webhooks"]:
            assert h["clientConfig"]["service"]["name"] in by_kind["Service"]
    for c in certs.values():
        assert c["spec"]["issuerRef"]["name"] in by_kind["Issuer"]
        assert any(d.startswith("nos-amd-webhook-service.") for d in c["spec"]["dnsNames"])
    # every Service selects some workload's pods; every ServiceMonitor selects a Service with its port
    for svc in by_kind["Service"].values():
        sel = svc["spec"]["selector"]
        assert any(all(t["metadata"]["labels"].get(k) == v for k, v in sel.items()) for t in pods), svc
    monitors = by_kind.get("ServiceMonitor", {})
    assert {m.split("-metrics-monitor")[0] for m in monitors} >= {"nos-amd-operator", "nos-amd-gpupartitioner",
                                                                  "nos-amd-partagent", "nos-amd-gpuagent"}
    for m in monitors.values():
        want = m["spec"]["selector"]["matchLabels"]
        svcs = [s for s in by_kind["Service"].values()
                if all(s["metadata"].get("labels", {}).get(k) == v for k, v in want.items())]
        assert svcs and all(any(p["name"] == m["spec"]["endpoints"][0]["port"] for p in s["spec"]["ports"])
                            for s in svcs)
    # the auth proxy can review tokens, and Prometheus has a reader role to bind
    assert "nos-amd-metrics-reader" in by_kind["ClusterRole"]


def test_daemonsets_are_privileged_and_node_selected():
    dss = [o for o in _objs() if o["kind"] == "DaemonSet"]
    assert len(dss) == 5  # partagent, gpuagent, device plugin x (cumask, partition, hybrid)
    for ds in dss:
        spec = ds["spec"]["template"]["spec"]
        if "nodeSelector" in spec:
            kinds = [spec["nodeSelector"]["nos.nebuly.com/gpu-partitioning"]]
        else:  # the partition agent serves partition AND hybrid nodes
            (expr,) = spec["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][
                "nodeSelectorTerms"][0]["matchExpressions"]
            assert expr["key"] == "nos.nebuly.com/gpu-partitioning" and expr["operator"] == "In"
            kinds = expr["values"]
        assert set(kinds) <= {"partition", "cumask", "hybrid"}
        c = spec["containers"][0]
        assert c["securityContext"]["privileged"] is True
        assert any(m["mountPath"] == "/var/lib/kubelet/pod-resources" for m in c["volumeMounts"])
        assert c["env"][0]["name"] == "NODE_NAME"


def test_values_overrides_render_and_validate(tmp_path):
    """Helm-values equivalent: overrides reach the embedded configs, disabled
    components disappear, the default namespace is refused, telemetry is opt-in."""
    base = manifests.render()
    assert "telemetry/job.yaml" not in base
    v = manifests.apply_set({}, "gpuPartitioner.cuPolicy=shared")
    v = manifests.apply_set(v, "gpuPartitioner.batchWindowIdleSeconds=3")
    v = manifests.merge_values(v, {"namespace": "gpu-sharing", "amdGpuResourceMemoryGB": 144,
                                   "shareTelemetry": True,
                                   "gpuPartitioner": {"gpuAgent": {"enabled": False}}})
    out = manifests.render(v)
    assert "gpuagent/daemonset.yaml" not in out and "partagent/daemonset.yaml" in out
    docs = [o for rel, text in out.items() if not rel.startswith("samples/") and rel != "values.yaml"
            for o in yaml.safe_load_all(text) if o]
    assert all(o["metadata"].get("namespace", "gpu-sharing") == "gpu-sharing" for o in docs
               if o["kind"] not in ("ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition",
                                    "ValidatingWebhookConfiguration", "Namespace", "Kustomization"))
    cms = {k: t for o in docs if o["kind"] == "ConfigMap" for k, t in (o.get("data") or {}).items()}
    p = tmp_path / "gp.yaml"
    p.write_text(cms["gpu_partitioner_config.yaml"])
    gp = cfgmod.load(p)
    assert gp.batch_window_idle_seconds == 3 and gp.amd_gpu_resource_memory_gb == 144
    assert yaml.safe_load(cms["scheduler_config.yaml"])["profiles"][0]["pluginConfig"][0]["args"][
        "amdGpuResourceMemoryGB"] == 144
    assert yaml.safe_load(cms["metrics.yaml"])["components"]["nosGpuPartitioner"] is True
    import pytest
    with pytest.raises(ValueError):
        manifests.render({"namespace": "default"})
    with pytest.raises(ValueError):
        manifests.render(manifests.apply_set({}, "gpuPartitioner.slicePlacement=diagonal"))
    # --stdout renders one stream; --dump-values round-trips through --values
    vals = tmp_path / "values.yaml"
    vals.write_text(yaml.safe_dump(manifests.DEFAULT_VALUES))
    assert manifests.main(["--values", str(vals), "--out", str(tmp_path / "cfg")]) == 0
    assert (tmp_path / "cfg" / "gpupartitioner" / "manager.yaml").read_text() == \
        (REPO / "config" / "gpupartitioner" / "manager.yaml").read_text()
