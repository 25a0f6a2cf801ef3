"""Render the deployment manifests under ``config/`` (the reference's
kustomize tree, ``config/**``, and Helm chart values).

Components: CRDs + samples, the operator (Deployment, webhook Service and
ValidatingWebhookConfiguration), the scheduler (Deployment +
KubeSchedulerConfiguration), the gpupartitioner (Deployment + config +
known MI355X partition geometries), and the node DaemonSets (partition
agent on ``gpu-partitioning=partition`` nodes, gpuagent and device plugin on
``cumask`` nodes) -- privileged, mounting ``/dev/kfd``, ``/dev/dri``, the
PodResources socket and the device-plugin directory.  RBAC follows the
controller-gen markers of the reference controllers.

python -m nos_amd.cmd.manifests --out config      (check: --check)
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import yaml

from ..api import constants as C
from ..api import v1alpha1

NS = "nos-system"


class _Dumper(yaml.SafeDumper):
    """Multi-line strings (embedded config files) as literal blocks."""


_Dumper.add_representer(str, lambda d, s: d.represent_scalar("tag:yaml.org,2002:str", s,
                                                             style="|" if "\n" in s else None))


def _dump(o) -> str:
    return yaml.dump(o, Dumper=_Dumper, sort_keys=False)


IMAGE = "ghcr.io/nos-amd/nos-amd:0.1.0"
IMAGE_ROCM = "ghcr.io/nos-amd/nos-amd-rocm:0.1.0"  # rocm/pytorch base for the GPU-side DaemonSets


def _sa(name: str) -> dict:
    return {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": name, "namespace": NS}}


def _cluster_role(name: str, rules: list[dict]) -> list[dict]:
    return [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": name},
             "rules": rules},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding", "metadata": {"name": name},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": name},
             "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": NS}]}]


def _rule(groups, resources, verbs) -> dict:
    return {"apiGroups": groups, "resources": resources, "verbs": verbs}


RW = ["get", "list", "watch", "create", "update", "patch", "delete"]
RO = ["get", "list", "watch"]
LEASES = _rule(["coordination.k8s.io"], ["leases"], RW)
EVENTS = _rule([""], ["events"], ["create", "patch"])


def _config_map(name: str, files: dict[str, str]) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": NS}, "data": files}


def _probes() -> dict:
    return {"livenessProbe": {"httpGet": {"path": "/healthz", "port": 8081}, "initialDelaySeconds": 15,
                              "periodSeconds": 20},
            "readinessProbe": {"httpGet": {"path": "/readyz", "port": 8081}, "initialDelaySeconds": 5,
                               "periodSeconds": 10}}


def _container(name: str, module: str, args: list[str], image: str = IMAGE, env: dict | None = None,
               mounts: list[dict] | None = None, privileged: bool = False, probes: bool = True) -> dict:
    c = {"name": name, "image": image, "command": ["python", "-m", module], "args": args,
         "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}, "limits": {"memory": "1Gi"}},
         "volumeMounts": mounts or []}
    if env:
        c["env"] = [{"name": k, **v} if isinstance(v, dict) else {"name": k, "value": v} for k, v in env.items()]
    if privileged:
        c["securityContext"] = {"privileged": True}
    else:
        c["securityContext"] = {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}}
    if probes:
        c.update(_probes())
    return c


def _deployment(name: str, container: dict, volumes: list[dict]) -> dict:
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": NS, "labels": {"app": name}},
            "spec": {"replicas": 1, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}},
                                  "spec": {"serviceAccountName": name, "containers": [container],
                                           "volumes": volumes, "securityContext": {"runAsNonRoot": True},
                                           "terminationGracePeriodSeconds": 10}}}}


NODE_ENV = {C.ENV_NODE_NAME: {"valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}}}
HOST_VOLUMES = [
    {"name": "kfd", "hostPath": {"path": "/dev/kfd"}},
    {"name": "dri", "hostPath": {"path": "/dev/dri"}},
    {"name": "pod-resources", "hostPath": {"path": "/var/lib/kubelet/pod-resources"}},
    {"name": "device-plugins", "hostPath": {"path": C.DEVICE_PLUGIN_DIR}},
]
HOST_MOUNTS = [
    {"name": "kfd", "mountPath": "/dev/kfd"},
    {"name": "dri", "mountPath": "/dev/dri"},
    {"name": "pod-resources", "mountPath": "/var/lib/kubelet/pod-resources"},
]


def _daemonset(name: str, container: dict, kind: str, volumes: list[dict]) -> dict:
    return {"apiVersion": "apps/v1", "kind": "DaemonSet",
            "metadata": {"name": name, "namespace": NS, "labels": {"app": name}},
            "spec": {"selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}},
                                  "spec": {"serviceAccountName": name, "containers": [container],
                                           "nodeSelector": {C.LABEL_GPU_PARTITIONING: kind},
                                           "priorityClassName": "system-node-critical",
                                           "tolerations": [{"key": "amd.com/gpu", "operator": "Exists",
                                                            "effect": "NoSchedule"}],
                                           "volumes": volumes}}}}


def _cfg_mount(name: str) -> tuple[dict, dict]:
    return ({"name": "config", "configMap": {"name": name}}, {"name": "config", "mountPath": "/etc/nos-amd"})


# ------------------------------------------------------------------ components
def crds() -> dict[str, list[dict]]:
    samples = [v1alpha1.build_eq("team-a", "quota-a").with_min({"cpu": "2", "memory": "8Gi",
                                                                C.RESOURCE_GPU_MEMORY: 36})
               .with_max({"cpu": "16", "memory": "64Gi", C.RESOURCE_GPU_MEMORY: 144}).get(),
               v1alpha1.build_composite_eq("team-b", "quota-b").with_namespaces("team-b", "team-c")
               .with_min({"cpu": "4", "memory": "16Gi", C.RESOURCE_GPU_MEMORY: 72})
               .with_max({"cpu": "32", "memory": "128Gi", C.RESOURCE_GPU_MEMORY: 288}).get()]
    for s in samples:
        s.pop("status", None)
    return {"crd/bases.yaml": [v1alpha1.crd(v1alpha1.KIND_EQ), v1alpha1.crd(v1alpha1.KIND_CEQ)],
            "samples/quotas.yaml": samples}


def operator() -> dict[str, list[dict]]:
    name = "nos-amd-operator"
    vol, mnt = _cfg_mount(name + "-config")
    certs = {"name": "cert", "secret": {"secretName": "nos-amd-webhook-server-cert"}}
    c = _container("manager", "nos_amd.cmd.operator",
                   ["--config", "/etc/nos-amd/operator_config.yaml", "--webhook-port", "9443",
                    "--webhook-cert-dir", "/tmp/k8s-webhook-server/serving-certs"],
                   mounts=[mnt, {"name": "cert", "mountPath": "/tmp/k8s-webhook-server/serving-certs",
                                 "readOnly": True}])
    c["ports"] = [{"containerPort": 9443, "name": "webhook-server"}]
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "OperatorConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "metrics": {"bindAddress": "127.0.0.1:8080"},
           "leaderElection": {"leaderElect": True, "resourceName": "nos-amd-operator"},
           "amdGpuResourceMemoryGB": C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "nos-amd-webhook-service", "namespace": NS},
           "spec": {"selector": {"app": name}, "ports": [{"port": 443, "targetPort": 9443}]}}

    def hook(kind: str, path: str, ops: list[str]) -> dict:
        plural = kind.lower() + "s"
        return {"name": f"v{kind.lower()}.kb.io", "admissionReviewVersions": ["v1"], "sideEffects": "None",
                "failurePolicy": "Fail",
                "clientConfig": {"service": {"name": "nos-amd-webhook-service", "namespace": NS, "path": path}},
                "rules": [{"apiGroups": [C.GROUP], "apiVersions": [C.VERSION], "operations": ops,
                           "resources": [plural]}]}

    from ..api.webhook_server import CEQ_PATH, EQ_PATH

    vwc = {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
           "metadata": {"name": "nos-amd-validating-webhook-configuration",
                        "annotations": {"cert-manager.io/inject-ca-from": f"{NS}/nos-amd-serving-cert"}},
           "webhooks": [hook("ElasticQuota", EQ_PATH, ["CREATE", "UPDATE"]),
                        hook("CompositeElasticQuota", CEQ_PATH, ["CREATE", "UPDATE"])]}
    rules = [_rule([C.GROUP], ["elasticquotas", "compositeelasticquotas"], RW),
             _rule([C.GROUP], ["elasticquotas/status", "compositeelasticquotas/status"], ["get", "update", "patch"]),
             _rule([""], ["pods"], ["get", "list", "watch", "patch", "update"]), LEASES, EVENTS]
    return {"operator/manager.yaml": [_sa(name), _config_map(name + "-config",
                                                             {"operator_config.yaml": yaml.safe_dump(cfg)}),
                                      _deployment(name, c, [vol, certs])],
            "operator/rbac.yaml": _cluster_role(name, rules),
            "operator/webhook.yaml": [svc, vwc]}


def scheduler() -> dict[str, list[dict]]:
    name = "nos-amd-scheduler"
    vol, mnt = _cfg_mount(name + "-config")
    sched_cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1", "kind": "KubeSchedulerConfiguration",
                 "leaderElection": {"leaderElect": False},
                 "profiles": [{"schedulerName": "nos-scheduler",
                               "plugins": {"preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
                                           "postFilter": {"enabled": [{"name": "CapacityScheduling"}],
                                                          "disabled": [{"name": "*"}]},
                                           "reserve": {"enabled": [{"name": "CapacityScheduling"}]}},
                               "pluginConfig": [{"name": "CapacityScheduling", "args": {
                                   "amdGpuResourceMemoryGB": C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB}}]}]}
    c = _container("scheduler", "nos_amd.cmd.scheduler", ["--config", "/etc/nos-amd/scheduler_config.yaml",
                                                          "--health-probe-bind-address", ":8081"], mounts=[mnt])
    rules = [_rule([""], ["pods"], RO + ["patch", "update", "delete"]), _rule([""], ["pods/binding"], ["create"]),
             _rule([""], ["pods/status"], ["patch", "update"]), _rule([""], ["nodes", "namespaces"], RO),
             _rule(["policy"], ["poddisruptionbudgets"], RO), _rule([C.GROUP], ["elasticquotas",
                                                                                 "compositeelasticquotas"], RO),
             LEASES, EVENTS]
    return {"scheduler/deployment.yaml": [_sa(name), _config_map(name + "-config", {
        "scheduler_config.yaml": yaml.safe_dump(sched_cfg)}), _deployment(name, c, [vol])],
        "scheduler/rbac.yaml": _cluster_role(name, rules)}


def known_geometries_yaml() -> str:
    from ..gpu.amdpart import mi355x_geometries

    gs = [{"compute": g.compute, "memory": g.memory, "profiles": {str(p): n for p, n in g.geometry.items()}}
          for g in mi355x_geometries()]
    return yaml.safe_dump([{"models": ["AMD-Instinct-MI355X", "AMD Instinct MI355X", "MI355X"],
                            "allowedGeometries": gs}], sort_keys=False)


def gpupartitioner() -> dict[str, list[dict]]:
    name = "nos-amd-gpupartitioner"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "GpuPartitionerConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "metrics": {"bindAddress": "127.0.0.1:8080"},
           "leaderElection": {"leaderElect": True, "resourceName": "nos-amd-gpupartitioner"},
           "schedulerConfigFile": "/etc/nos-amd/scheduler_config.yaml",
           "knownPartitionGeometriesFile": "/etc/nos-amd/known_partition_geometries.yaml",
           "batchWindowTimeoutSeconds": 60, "batchWindowIdleSeconds": 10,
           "devicePluginConfigMap": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME, "namespace": NS},
           "devicePluginDelaySeconds": 5, "planReportTimeoutSeconds": 300,
           "amdGpuResourceMemoryGB": C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB,
           "slicePlacement": "pack", "cuPolicy": "even"}
    sched = scheduler()["scheduler/deployment.yaml"][1]["data"]["scheduler_config.yaml"]
    c = _container("manager", "nos_amd.cmd.gpupartitioner", ["--config", "/etc/nos-amd/gpu_partitioner_config.yaml"],
                   mounts=[mnt])
    rules = [_rule([""], ["pods"], RO), _rule([""], ["nodes"], RO + ["patch", "update"]),
             _rule([""], ["configmaps"], RW), _rule([C.GROUP], ["elasticquotas", "compositeelasticquotas"], RO),
             _rule(["policy"], ["poddisruptionbudgets"], RO), LEASES, EVENTS]
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME,
                                                                  "namespace": NS}, "data": {}}
    return {"gpupartitioner/manager.yaml": [
        _sa(name), _config_map(name + "-config", {"gpu_partitioner_config.yaml": yaml.safe_dump(cfg),
                                                  "scheduler_config.yaml": sched,
                                                  "known_partition_geometries.yaml": known_geometries_yaml()}),
        cm, _deployment(name, c, [vol])],
        "gpupartitioner/rbac.yaml": _cluster_role(name, rules)}


def node_agents() -> dict[str, list[dict]]:
    out: dict[str, list[dict]] = {}
    node_rules = [_rule([""], ["nodes"], RO + ["patch", "update"]), _rule([""], ["pods"], RO + ["delete"]),
                  _rule([""], ["configmaps"], RO), EVENTS]
    # partition agent (migagent analogue)
    name = "nos-amd-partagent"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "PartitionAgentConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "reportConfigIntervalSeconds": 10,
           "allowModeChanges": True, "defaultComputeMode": "SPX", "defaultMemoryMode": "NPS1"}
    c = _container("partagent", "nos_amd.cmd.partagent", ["--config", "/etc/nos-amd/partition_agent_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV, mounts=HOST_MOUNTS + [mnt], privileged=True)
    out["partagent/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
        "partition_agent_config.yaml": yaml.safe_dump(cfg)}),
        _daemonset(name, c, C.PARTITIONING_AMDPART, HOST_VOLUMES + [vol])]
    out["partagent/rbac.yaml"] = _cluster_role(name, node_rules)
    # gpuagent (CU-mask reporter + probes)
    name = "nos-amd-gpuagent"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "GpuAgentConfig", "health": {"healthProbeBindAddress": ":8081"},
           "reportConfigIntervalSeconds": 10, "probeEnabled": True}
    c = _container("gpuagent", "nos_amd.cmd.gpuagent", ["--config", "/etc/nos-amd/gpu_agent_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV, mounts=HOST_MOUNTS + [mnt], privileged=True)
    out["gpuagent/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
        "gpu_agent_config.yaml": yaml.safe_dump(cfg)}), _daemonset(name, c, C.PARTITIONING_CUMASK, HOST_VOLUMES + [vol])]
    out["gpuagent/rbac.yaml"] = _cluster_role(name, node_rules)
    # device plugin (one DaemonSet per partitioning kind + plain GPU nodes could reuse it)
    name = "nos-amd-device-plugin"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "DevicePluginConfig",
           "health": {"healthProbeBindAddress": ":8081"},
           "configMap": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME, "namespace": NS},
           "socketDir": C.DEVICE_PLUGIN_DIR, "cuPolicy": "even"}
    c = _container("device-plugin", "nos_amd.cmd.deviceplugin", ["--config", "/etc/nos-amd/device_plugin_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV,
                   mounts=HOST_MOUNTS + [{"name": "device-plugins", "mountPath": C.DEVICE_PLUGIN_DIR}, mnt],
                   privileged=True)
    dss = []
    for kind in (C.PARTITIONING_CUMASK, C.PARTITIONING_AMDPART):
        ds = _daemonset(f"{name}-{kind}", c, kind, HOST_VOLUMES + [vol])
        ds["spec"]["template"]["metadata"]["labels"] = {"app": name}
        ds["spec"]["selector"]["matchLabels"] = {"app": name, "nos.nebuly.com/kind": kind}
        ds["spec"]["template"]["metadata"]["labels"]["nos.nebuly.com/kind"] = kind
        ds["spec"]["template"]["spec"]["serviceAccountName"] = name
        dss.append(ds)
    out["deviceplugin/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
        "device_plugin_config.yaml": yaml.safe_dump(cfg)})] + dss
    out["deviceplugin/rbac.yaml"] = _cluster_role(name, node_rules)
    return out


def render() -> dict[str, str]:
    files: dict[str, list[dict]] = {"namespace.yaml": [{"apiVersion": "v1", "kind": "Namespace",
                                                        "metadata": {"name": NS}}]}
    for part in (crds(), operator(), scheduler(), gpupartitioner(), node_agents()):
        files.update(part)
    out = {k: "---\n".join(_dump(o) for o in v) for k, v in files.items()}
    out["kustomization.yaml"] = yaml.safe_dump({"apiVersion": "kustomize.config.k8s.io/v1beta1",
                                                "kind": "Kustomization", "namespace": NS,
                                                "resources": sorted(k for k in files if not k.startswith("samples/"))},
                                               sort_keys=False)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", default="config")
    ap.add_argument("--check", action="store_true", help="fail if the files on disk are stale")
    a = ap.parse_args(argv)
    root = Path(a.out)
    stale = []
    for rel, text in render().items():
        p = root / rel
        header = "# generated by `python -m nos_amd.cmd.manifests`; do not edit\n"
        if a.check:
            if not p.exists() or p.read_text() != header + text:
                stale.append(rel)
            continue
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(header + text)
    if stale:
        print("stale manifests:", ", ".join(stale), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
