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

Deployment knobs come from a Helm-style values tree (``DEFAULT_VALUES``;
the reference's ``helm-charts/nos/values.yaml`` keys with AMD names), so a
user can render a customised install without Helm:

    python -m nos_amd.cmd.manifests --out config                 (defaults; --check)
    python -m nos_amd.cmd.manifests --values my.yaml --set gpuPartitioner.cuPolicy=shared --stdout
    python -m nos_amd.cmd.manifests --dump-values > values.yaml

Like the chart's ``templates/validation.yaml`` the ``default`` namespace is
refused; ``shareTelemetry: true`` adds the metrics-exporter post-install Job
(``templates/pod_metrics-exporter.yaml``), off by default.
"""
from __future__ import annotations

import argparse
import copy
import sys
from pathlib import Path

import yaml

from ..api import constants as C
from ..api import v1alpha1

NS = "nos-system"

DEFAULT_VALUES: dict = {
    "namespace": NS,
    "amdGpuResourceMemoryGB": C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB,
    "leaderElection": True,
    "logLevel": "info",
    "shareTelemetry": False,
    "telemetryEndpoint": "",
    "image": {"repository": "ghcr.io/nos-amd/nos-amd", "tag": "0.1.0"},
    "rocmImage": {"repository": "ghcr.io/nos-amd/nos-amd-rocm", "tag": "0.1.0"},
    "operator": {"enabled": True, "webhook": {"enabled": True}},
    # webhook serving certificate: cert-manager Issuer + Certificate (config/operator/certificate.yaml);
    # disabled -> provide the TLS secret "nos-amd-webhook-server-cert" yourself
    "certManager": {"enabled": True},
    # /metrics behind a kube-rbac-proxy sidecar (https :8443) + a Service per component,
    # and Prometheus-operator ServiceMonitors for them
    "metrics": {"authProxy": True, "serviceMonitor": True,
                "authProxyImage": {"repository": "quay.io/brancz/kube-rbac-proxy", "tag": "v0.18.0"}},
    "scheduler": {"enabled": True, "schedulerName": "nos-scheduler"},
    "gpuPartitioner": {
        "enabled": True,
        "batchWindowTimeoutSeconds": 60,
        "batchWindowIdleSeconds": 10,
        "devicePluginDelaySeconds": 5,
        "planReportTimeoutSeconds": 300,
        "slicePlacement": "pack",
        # auto: "shared" with the pod server (its tenants share every CU, MPS's
        # default), "proportional" CU masks for process pods otherwise
        "cuPolicy": "auto",
        "reserveWholeGpus": 0,
        "preferredMemoryMode": "NPS1",
        "knownPartitionGeometries": None,  # list override; default: derived from each node's amd-smi memory/XCDs
        "partitionAgent": {"enabled": True, "reportConfigIntervalSeconds": 10, "allowModeChanges": True,
                           "defaultComputeMode": "SPX", "defaultMemoryMode": "NPS1"},
        "gpuAgent": {"enabled": True, "reportConfigIntervalSeconds": 10, "probeEnabled": True},
        "devicePlugin": {"enabled": True},
        # pod server on cumask nodes (nos_amd/podserver, the MPS analogue): one
        # server process per GPU hosts every slice pod's inferences, so slices
        # per GPU are bounded by memory and tenantsPerGpu, not by the 8 HWS
        # process slots
        "podServer": {"enabled": False, "tenantsPerGpu": 48, "lanes": 16,
                      "socketDir": C.DEFAULT_POD_SERVER_SOCKET_DIR},
    },
}

_V: dict = DEFAULT_VALUES  # values of the render in progress (set by render())


def _ns() -> str:
    return _V["namespace"]


def _img(key: str) -> str:
    return f"{_V[key]['repository']}:{_V[key]['tag']}"


def merge_values(base: dict, override: dict) -> dict:
    """Deep merge (Helm semantics: maps merge, everything else replaces)."""
    out = copy.deepcopy(base)
    for k, v in (override or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge_values(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def apply_set(values: dict, expr: str) -> dict:
    """``--set a.b.c=value`` (value parsed as YAML: numbers, booleans, lists)."""
    path, _, raw = expr.partition("=")
    if not path or not _:
        raise ValueError(f"--set expects key=value, got {expr!r}")
    node: dict = {}
    cur = node
    keys = path.split(".")
    for k in keys[:-1]:
        cur = cur.setdefault(k, {})
    cur[keys[-1]] = yaml.safe_load(raw) if raw != "" else ""
    return merge_values(values, node)


def resolve_values(v: dict) -> dict:
    """Defaults that depend on other values: ``cuPolicy: auto`` is ``shared``
    when the pod server is enabled -- its tenants then share every CU and the
    lanes' HIP graphs (an explicit even/proportional policy gives pod-server
    tenants CU-masked streams, captured under slice-budgeted kernel configs)
    -- and ``proportional`` otherwise."""
    gp = v["gpuPartitioner"]
    if gp.get("cuPolicy") == "auto":
        gp["cuPolicy"] = "shared" if gp["podServer"]["enabled"] else "proportional"
    return v


def validate_values(v: dict) -> None:
    if v["namespace"] in ("", "default"):
        raise ValueError("nos-amd must not be installed in the 'default' namespace")
    gp = v["gpuPartitioner"]
    if gp["batchWindowTimeoutSeconds"] <= 0 or gp["batchWindowIdleSeconds"] <= 0:
        raise ValueError("gpuPartitioner batch windows must be > 0")
    if gp["slicePlacement"] not in ("pack", "spread", "measured"):
        raise ValueError("gpuPartitioner.slicePlacement must be pack|spread|measured")
    if gp["cuPolicy"] not in ("auto", "even", "proportional", "shared"):
        raise ValueError("gpuPartitioner.cuPolicy must be auto|even|proportional|shared")
    ps = gp["podServer"]
    if ps["enabled"] and not (1 <= int(ps["lanes"]) <= 32 and int(ps["tenantsPerGpu"]) >= 1):
        raise ValueError("gpuPartitioner.podServer: lanes must be 1..32 (one HW queue each), tenantsPerGpu >= 1")
    if int(v["amdGpuResourceMemoryGB"]) <= 0:
        raise ValueError("amdGpuResourceMemoryGB must be > 0")
    if v["metrics"]["serviceMonitor"] and not v["metrics"]["authProxy"]:
        raise ValueError("metrics.serviceMonitor scrapes the auth proxy: enable metrics.authProxy")


class _Dumper(yaml.SafeDumper):
    """Multi-line strings (embedded config files) as literal blocks."""


_Dumper.add_representer(str, lambda d, s: d.represent_scalar("tag:yaml.org,2002:str", s,
                                                             style="|" if "\n" in s else None))


def _dump(o) -> str:
    return yaml.dump(o, Dumper=_Dumper, sort_keys=False)


IMAGE, IMAGE_ROCM = "image", "rocmImage"  # value keys; rocm/pytorch base for the GPU-side DaemonSets


def _sa(name: str) -> dict:
    return {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": name, "namespace": _ns()}}


def _cluster_role(name: str, rules: list[dict]) -> list[dict]:
    return [{"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": name},
             "rules": rules},
            {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding", "metadata": {"name": name},
             "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": name},
             "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": _ns()}]}]


def _rule(groups, resources, verbs) -> dict:
    return {"apiGroups": groups, "resources": resources, "verbs": verbs}


RW = ["get", "list", "watch", "create", "update", "patch", "delete"]
RO = ["get", "list", "watch"]
LEASES = _rule(["coordination.k8s.io"], ["leases"], RW)
EVENTS = _rule([""], ["events"], ["create", "patch"])


def _config_map(name: str, files: dict[str, str]) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": _ns()}, "data": files}


def _probes() -> dict:
    return {"livenessProbe": {"httpGet": {"path": "/healthz", "port": 8081}, "initialDelaySeconds": 15,
                              "periodSeconds": 20},
            "readinessProbe": {"httpGet": {"path": "/readyz", "port": 8081}, "initialDelaySeconds": 5,
                               "periodSeconds": 10}}


def _container(name: str, module: str, args: list[str], image: str = IMAGE, env: dict | None = None,
               mounts: list[dict] | None = None, privileged: bool = False, probes: bool = True) -> dict:
    c = {"name": name, "image": _img(image), "command": ["python", "-m", module],
         "args": args + ["--log-level", _V["logLevel"]],
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
            "metadata": {"name": name, "namespace": _ns(), "labels": {"app": name}},
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


def _daemonset(name: str, container: dict, kind: str | tuple[str, ...], volumes: list[dict]) -> dict:
    if not isinstance(kind, str):  # several partitioning kinds: node affinity instead of a selector
        ds = _daemonset(name, container, kind[0], volumes)
        spec = ds["spec"]["template"]["spec"]
        del spec["nodeSelector"]
        spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": C.LABEL_GPU_PARTITIONING, "operator": "In", "values": list(kind)}]}]}}}
        return ds
    return {"apiVersion": "apps/v1", "kind": "DaemonSet",
            "metadata": {"name": name, "namespace": _ns(), "labels": {"app": name}},
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


WEBHOOK_SECRET = "nos-amd-webhook-server-cert"
SERVING_CERT = "nos-amd-serving-cert"
WEBHOOK_SERVICE = "nos-amd-webhook-service"
METRICS_READER = "nos-amd-metrics-reader"


def _with_metrics(name: str, workload: dict, upstream_port: int = 8080) -> list[dict]:
    """Expose a component's /metrics (bound to 127.0.0.1:<upstream_port>)
    through a kube-rbac-proxy sidecar on https :8443 (authn/z by token review,
    the reference's operator_auth_proxy_patch.yaml), a Service, and a
    ServiceMonitor (config/*/prometheus/monitor.yaml).  Returns the extra objects."""
    m = _V["metrics"]
    if not m["authProxy"]:
        return []
    img = m["authProxyImage"]
    proxy = {"name": "kube-rbac-proxy", "image": f"{img['repository']}:{img['tag']}",
             "args": ["--secure-listen-address=0.0.0.0:8443", f"--upstream=http://127.0.0.1:{upstream_port}/",
                      "--logtostderr=true", "--v=0"],
             "ports": [{"containerPort": 8443, "name": "https", "protocol": "TCP"}],
             "resources": {"requests": {"cpu": "5m", "memory": "64Mi"}, "limits": {"memory": "128Mi"}},
             "securityContext": {"allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}}}
    workload["spec"]["template"]["spec"]["containers"].append(proxy)
    labels = dict(workload["spec"]["selector"]["matchLabels"])
    svc = {"apiVersion": "v1", "kind": "Service",
           "metadata": {"name": f"{name}-metrics", "namespace": _ns(), "labels": {"app": name, "metrics": "nos-amd"}},
           "spec": {"selector": {"app": labels["app"]},
                    "ports": [{"name": "https", "port": 8443, "targetPort": "https", "protocol": "TCP"}]}}
    out = [svc]
    if m["serviceMonitor"]:
        out.append({"apiVersion": "monitoring.coreos.com/v1", "kind": "ServiceMonitor",
                    "metadata": {"name": f"{name}-metrics-monitor", "namespace": _ns(), "labels": {"app": name}},
                    "spec": {"selector": {"matchLabels": {"app": name, "metrics": "nos-amd"}},
                             "endpoints": [{"path": "/metrics", "port": "https", "scheme": "https",
                                            "bearerTokenFile": "/var/run/secrets/kubernetes.io/serviceaccount/token",
                                            "tlsConfig": {"insecureSkipVerify": True}}]}})
    return out


def _auth_proxy_rules() -> list[dict]:
    """What the kube-rbac-proxy sidecar needs to authenticate/authorise scrapers."""
    return [_rule(["authentication.k8s.io"], ["tokenreviews"], ["create"]),
            _rule(["authorization.k8s.io"], ["subjectaccessreviews"], ["create"])]


def monitoring() -> dict[str, list[dict]]:
    """ClusterRole a Prometheus service account is bound to for scraping."""
    if not _V["metrics"]["authProxy"]:
        return {}
    return {"monitoring/metrics-reader.yaml": [
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": METRICS_READER},
         "rules": [{"nonResourceURLs": ["/metrics"], "verbs": ["get"]}]}]}


def certificates() -> list[dict]:
    """cert-manager self-signed Issuer + the webhook serving Certificate whose
    secret the operator Deployment mounts and whose CA cert-manager injects into
    the ValidatingWebhookConfiguration (config/operator/certmanager/certificate.yaml)."""
    svc = f"{WEBHOOK_SERVICE}.{_ns()}.svc"
    return [{"apiVersion": "cert-manager.io/v1", "kind": "Issuer",
             "metadata": {"name": "nos-amd-selfsigned-issuer", "namespace": _ns()}, "spec": {"selfSigned": {}}},
            {"apiVersion": "cert-manager.io/v1", "kind": "Certificate",
             "metadata": {"name": SERVING_CERT, "namespace": _ns()},
             "spec": {"dnsNames": [svc, svc + ".cluster.local"], "secretName": WEBHOOK_SECRET,
                      "issuerRef": {"kind": "Issuer", "name": "nos-amd-selfsigned-issuer"},
                      "privateKey": {"rotationPolicy": "Always"}}}]


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
    certs = {"name": "cert", "secret": {"secretName": WEBHOOK_SECRET}}
    c = _container("manager", "nos_amd.cmd.operator",
                   ["--config", "/etc/nos-amd/operator_config.yaml"] +
                   (["--webhook-port", "9443", "--webhook-cert-dir", "/tmp/k8s-webhook-server/serving-certs"]
                    if _V["operator"]["webhook"]["enabled"] else []),
                   mounts=[mnt, {"name": "cert", "mountPath": "/tmp/k8s-webhook-server/serving-certs",
                                 "readOnly": True}])
    c["ports"] = [{"containerPort": 9443, "name": "webhook-server"}]
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "OperatorConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "metrics": {"bindAddress": "127.0.0.1:8080"},
           "leaderElection": {"leaderElect": _V["leaderElection"], "resourceName": "nos-amd-operator"},
           "amdGpuResourceMemoryGB": _V["amdGpuResourceMemoryGB"]}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": WEBHOOK_SERVICE, "namespace": _ns()},
           "spec": {"selector": {"app": name}, "ports": [{"port": 443, "targetPort": 9443}]}}

    def hook(kind: str, path: str, ops: list[str]) -> dict:
        plural = kind.lower() + "s"
        return {"name": f"v{kind.lower()}.kb.io", "admissionReviewVersions": ["v1"], "sideEffects": "None",
                "failurePolicy": "Fail",
                "clientConfig": {"service": {"name": WEBHOOK_SERVICE, "namespace": _ns(), "path": path}},
                "rules": [{"apiGroups": [C.GROUP], "apiVersions": [C.VERSION], "operations": ops,
                           "resources": [plural]}]}

    from ..api.webhook_server import CEQ_PATH, EQ_PATH

    vwc = {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
           "metadata": {"name": "nos-amd-validating-webhook-configuration",
                        "annotations": {"cert-manager.io/inject-ca-from": f"{_ns()}/{SERVING_CERT}"}},
           "webhooks": [hook("ElasticQuota", EQ_PATH, ["CREATE", "UPDATE"]),
                        hook("CompositeElasticQuota", CEQ_PATH, ["CREATE", "UPDATE"])]}
    rules = [_rule([C.GROUP], ["elasticquotas", "compositeelasticquotas"], RW),
             _rule([C.GROUP], ["elasticquotas/status", "compositeelasticquotas/status"], ["get", "update", "patch"]),
             _rule([""], ["pods"], ["get", "list", "watch", "patch", "update"]), LEASES, EVENTS] + _auth_proxy_rules()
    dep = _deployment(name, c, [vol, certs])
    out = {"operator/manager.yaml": [_sa(name), _config_map(name + "-config",
                                                            {"operator_config.yaml": yaml.safe_dump(cfg)}), dep],
           "operator/rbac.yaml": _cluster_role(name, rules)}
    out["operator/metrics.yaml"] = _with_metrics(name, dep)
    if _V["operator"]["webhook"]["enabled"]:
        out["operator/webhook.yaml"] = [svc, vwc]
        if _V["certManager"]["enabled"]:
            out["operator/certificate.yaml"] = certificates()
    return {k: v for k, v in out.items() if v}


def scheduler() -> dict[str, list[dict]]:
    name = "nos-amd-scheduler"
    vol, mnt = _cfg_mount(name + "-config")
    sched_cfg = {"apiVersion": "kubescheduler.config.k8s.io/v1", "kind": "KubeSchedulerConfiguration",
                 "leaderElection": {"leaderElect": False},
                 "profiles": [{"schedulerName": _V["scheduler"]["schedulerName"],
                               "plugins": {"preFilter": {"enabled": [{"name": "CapacityScheduling"}]},
                                           "postFilter": {"enabled": [{"name": "CapacityScheduling"}],
                                                          "disabled": [{"name": "*"}]},
                                           "reserve": {"enabled": [{"name": "CapacityScheduling"}]}},
                               "pluginConfig": [{"name": "CapacityScheduling", "args": {
                                   "amdGpuResourceMemoryGB": _V["amdGpuResourceMemoryGB"]}}]}]}
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

    if _V["gpuPartitioner"].get("knownPartitionGeometries"):
        return yaml.safe_dump(_V["gpuPartitioner"]["knownPartitionGeometries"], sort_keys=False)
    gs = [{"compute": g.compute, "memory": g.memory, "profiles": {str(p): n for p, n in g.geometry.items()}}
          for g in mi355x_geometries()]
    return yaml.safe_dump([{"models": ["AMD-Instinct-MI355X", "AMD Instinct MI355X", "MI355X"],
                            "allowedGeometries": gs}], sort_keys=False)


def gpupartitioner() -> dict[str, list[dict]]:
    name = "nos-amd-gpupartitioner"
    gp = _V["gpuPartitioner"]
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "GpuPartitionerConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "metrics": {"bindAddress": "127.0.0.1:8080"},
           "leaderElection": {"leaderElect": _V["leaderElection"], "resourceName": "nos-amd-gpupartitioner"},
           "schedulerConfigFile": "/etc/nos-amd/scheduler_config.yaml",
           "knownPartitionGeometriesFile": ("/etc/nos-amd/known_partition_geometries.yaml"
                                            if gp.get("knownPartitionGeometries") else ""),
           "reserveWholeGpus": gp["reserveWholeGpus"], "preferredMemoryMode": gp["preferredMemoryMode"],
           "batchWindowTimeoutSeconds": gp["batchWindowTimeoutSeconds"],
           "batchWindowIdleSeconds": gp["batchWindowIdleSeconds"],
           "devicePluginConfigMap": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME, "namespace": _ns()},
           "devicePluginDelaySeconds": gp["devicePluginDelaySeconds"],
           "planReportTimeoutSeconds": gp["planReportTimeoutSeconds"],
           "amdGpuResourceMemoryGB": _V["amdGpuResourceMemoryGB"],
           "slicePlacement": gp["slicePlacement"], "cuPolicy": gp["cuPolicy"]}
    sched = scheduler()["scheduler/deployment.yaml"][1]["data"]["scheduler_config.yaml"]
    c = _container("manager", "nos_amd.cmd.gpupartitioner", ["--config", "/etc/nos-amd/gpu_partitioner_config.yaml"],
                   mounts=[mnt])
    rules = [_rule([""], ["pods"], RO), _rule([""], ["nodes"], RO + ["patch", "update"]),
             _rule([""], ["configmaps"], RW), _rule([C.GROUP], ["elasticquotas", "compositeelasticquotas"], RO),
             _rule(["policy"], ["poddisruptionbudgets"], RO), LEASES, EVENTS] + _auth_proxy_rules()
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME,
                                                                  "namespace": _ns()}, "data": {}}
    dep = _deployment(name, c, [vol])
    files = {"gpu_partitioner_config.yaml": yaml.safe_dump(cfg), "scheduler_config.yaml": sched}
    if gp.get("knownPartitionGeometries"):  # else geometries follow each node's amd-smi memory/XCDs
        files["known_partition_geometries.yaml"] = known_geometries_yaml()
    out = {"gpupartitioner/manager.yaml": [_sa(name), _config_map(name + "-config", files), cm, dep],
           "gpupartitioner/rbac.yaml": _cluster_role(name, rules),
           "gpupartitioner/metrics.yaml": _with_metrics(name, dep)}
    return {k: v for k, v in out.items() if v}


def node_agents() -> dict[str, list[dict]]:
    out: dict[str, list[dict]] = {}
    gp = _V["gpuPartitioner"]
    pa, ga, ps = gp["partitionAgent"], gp["gpuAgent"], gp["podServer"]
    node_rules = [_rule([""], ["nodes"], RO + ["patch", "update"]), _rule([""], ["pods"], RO + ["delete"]),
                  _rule([""], ["configmaps"], RO), EVENTS]
    # partition agent (migagent analogue)
    name = "nos-amd-partagent"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "PartitionAgentConfig",
           "health": {"healthProbeBindAddress": ":8081"}, "metrics": {"bindAddress": "127.0.0.1:8080"},
           "reportConfigIntervalSeconds": pa["reportConfigIntervalSeconds"],
           "allowModeChanges": pa["allowModeChanges"], "defaultComputeMode": pa["defaultComputeMode"],
           "defaultMemoryMode": pa["defaultMemoryMode"]}
    c = _container("partagent", "nos_amd.cmd.partagent", ["--config", "/etc/nos-amd/partition_agent_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV, mounts=HOST_MOUNTS + [mnt], privileged=True)
    if pa["enabled"]:
        # hybrid nodes run it too: it switches their modes, its hybrid reporter reports slices
        ds = _daemonset(name, c, (C.PARTITIONING_AMDPART, C.PARTITIONING_HYBRID), HOST_VOLUMES + [vol])
        out["partagent/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
            "partition_agent_config.yaml": yaml.safe_dump(cfg)}), ds]
        out["partagent/rbac.yaml"] = _cluster_role(name, node_rules + _auth_proxy_rules())
        if extra := _with_metrics(name, ds):
            out["partagent/metrics.yaml"] = extra
    # gpuagent (CU-mask reporter + probes)
    name = "nos-amd-gpuagent"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "GpuAgentConfig", "health": {"healthProbeBindAddress": ":8081"},
           "metrics": {"bindAddress": "127.0.0.1:8080"},
           "reportConfigIntervalSeconds": ga["reportConfigIntervalSeconds"], "probeEnabled": ga["probeEnabled"],
           "podServerTenants": ps["tenantsPerGpu"] if ps["enabled"] else 0}
    c = _container("gpuagent", "nos_amd.cmd.gpuagent", ["--config", "/etc/nos-amd/gpu_agent_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV, mounts=HOST_MOUNTS + [mnt], privileged=True)
    if ga["enabled"]:
        ds = _daemonset(name, c, C.PARTITIONING_CUMASK, HOST_VOLUMES + [vol])
        out["gpuagent/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
            "gpu_agent_config.yaml": yaml.safe_dump(cfg)}), ds]
        out["gpuagent/rbac.yaml"] = _cluster_role(name, node_rules + _auth_proxy_rules())
        if extra := _with_metrics(name, ds):
            out["gpuagent/metrics.yaml"] = extra
    # device plugin (one DaemonSet per partitioning kind + plain GPU nodes could reuse it)
    name = "nos-amd-device-plugin"
    vol, mnt = _cfg_mount(name + "-config")
    cfg = {"apiVersion": C.CONFIG_API_VERSION, "kind": "DevicePluginConfig",
           "health": {"healthProbeBindAddress": ":8081"},
           "configMap": {"name": C.DEFAULT_DEVICE_PLUGIN_CM_NAME, "namespace": _ns()},
           "socketDir": C.DEVICE_PLUGIN_DIR, "cuPolicy": gp["cuPolicy"], "deviceEnv": "container",
           "rescanSeconds": 5, "podServerSocketDir": ps["socketDir"] if ps["enabled"] else ""}
    c = _container("device-plugin", "nos_amd.cmd.deviceplugin", ["--config", "/etc/nos-amd/device_plugin_config.yaml"],
                   image=IMAGE_ROCM, env=NODE_ENV,
                   mounts=HOST_MOUNTS + [{"name": "device-plugins", "mountPath": C.DEVICE_PLUGIN_DIR}, mnt],
                   privileged=True)
    dss = []
    for kind in (C.PARTITIONING_CUMASK, C.PARTITIONING_AMDPART, C.PARTITIONING_HYBRID):
        ds = _daemonset(f"{name}-{kind}", c, kind, HOST_VOLUMES + [vol])
        ds["spec"]["template"]["metadata"]["labels"] = {"app": name}
        ds["spec"]["selector"]["matchLabels"] = {"app": name, "nos.nebuly.com/kind": kind}
        ds["spec"]["template"]["metadata"]["labels"]["nos.nebuly.com/kind"] = kind
        ds["spec"]["template"]["spec"]["serviceAccountName"] = name
        dss.append(ds)
    if gp["devicePlugin"]["enabled"]:
        out["deviceplugin/daemonset.yaml"] = [_sa(name), _config_map(name + "-config", {
            "device_plugin_config.yaml": yaml.safe_dump(cfg)})] + dss
        out["deviceplugin/rbac.yaml"] = _cluster_role(name, node_rules)
    # pod server (MPS-daemon analogue): one process per GPU, sockets in a host
    # directory the device plugin mounts into every pod-server slice pod
    if ps["enabled"]:
        name = "nos-amd-podserver"
        c = _container("podserver", "nos_amd.cmd.podserver",
                       ["--gpus", "all", "--socket-dir", ps["socketDir"], "--lanes", str(ps["lanes"]),
                        "--max-tenants", str(ps["tenantsPerGpu"]),
                        # evict tenants whose devices no pod holds (kubelet PodResources)
                        "--pod-resources-socket", C.KUBELET_PODRESOURCES_SOCKET],
                       image=IMAGE_ROCM, env=NODE_ENV,
                       mounts=HOST_MOUNTS + [{"name": "podserver-sockets", "mountPath": ps["socketDir"]}],
                       privileged=True, probes=False)
        c["resources"] = {"requests": {"cpu": "2", "memory": "4Gi"}, "limits": {"memory": "64Gi"}}
        ds = _daemonset(name, c, C.PARTITIONING_CUMASK, HOST_VOLUMES[:3] + [
            {"name": "podserver-sockets", "hostPath": {"path": ps["socketDir"], "type": "DirectoryOrCreate"}}])
        out["podserver/daemonset.yaml"] = [_sa(name), ds]
    return out


def telemetry() -> dict[str, list[dict]]:
    """Post-install metrics export (``templates/configmap_metrics.yaml`` +
    ``pod_metrics-exporter.yaml``): component toggles + chart values, POSTed to
    ``telemetryEndpoint`` (or only logged when it is empty)."""
    name = "nos-amd-metrics-exporter"
    gp = _V["gpuPartitioner"]
    metrics = {"installationUUID": "", "components": {
        "nosOperator": _V["operator"]["enabled"], "nosScheduler": _V["scheduler"]["enabled"],
        "nosGpuPartitioner": gp["enabled"]}, "chartValues": _V}
    vol, mnt = _cfg_mount(name + "-config")
    args = ["--metrics-file", "/etc/nos-amd/metrics.yaml"]
    if _V["telemetryEndpoint"]:
        args += ["--metrics-endpoint", _V["telemetryEndpoint"]]
    c = _container("exporter", "nos_amd.cmd.metricsexporter", args, mounts=[mnt], probes=False)
    job = {"apiVersion": "batch/v1", "kind": "Job",
           "metadata": {"name": name, "namespace": _ns(),
                        "annotations": {"helm.sh/hook": "post-install", "helm.sh/hook-delete-policy": "hook-succeeded"}},
           "spec": {"backoffLimit": 0, "template": {"spec": {"restartPolicy": "Never", "containers": [c],
                                                             "volumes": [vol]}}}}
    return {"telemetry/job.yaml": [_config_map(name + "-config", {"metrics.yaml": yaml.safe_dump(metrics)}), job]}


def render(values: dict | None = None) -> dict[str, str]:
    """Render every manifest file for ``values`` (merged over DEFAULT_VALUES)."""
    global _V
    v = resolve_values(merge_values(DEFAULT_VALUES, values or {}))
    validate_values(v)
    prev, _V = _V, v
    try:
        files: dict[str, list[dict]] = {"namespace.yaml": [{"apiVersion": "v1", "kind": "Namespace",
                                                            "metadata": {"name": _ns()}}]}
        parts = [crds()]
        if v["operator"]["enabled"]:
            parts.append(operator())
        if v["scheduler"]["enabled"]:
            parts.append(scheduler())
        if v["gpuPartitioner"]["enabled"]:
            parts.append(gpupartitioner())
        parts.append(node_agents())
        parts.append(monitoring())
        if v["shareTelemetry"]:
            parts.append(telemetry())
        for part in parts:
            files.update(part)
    finally:
        _V = prev
    out = {k: "---\n".join(_dump(o) for o in docs) for k, docs in files.items()}
    out["values.yaml"] = "# the values this tree was rendered with (--values / --set to customise)\n" + \
        yaml.safe_dump(v, sort_keys=False)
    out["kustomization.yaml"] = yaml.safe_dump({"apiVersion": "kustomize.config.k8s.io/v1beta1",
                                                "kind": "Kustomization", "namespace": v["namespace"],
                                                "resources": sorted(k for k in files if not k.startswith("samples/"))},
                                               sort_keys=False)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--out", default="config")
    ap.add_argument("--check", action="store_true", help="fail if the files on disk are stale")
    ap.add_argument("--values", action="append", default=[], help="values YAML file(s), merged in order")
    ap.add_argument("--set", action="append", default=[], help="key.path=value override (YAML value)")
    ap.add_argument("--stdout", action="store_true", help="print one multi-document stream (helm template)")
    ap.add_argument("--dump-values", action="store_true", help="print the default values and exit")
    a = ap.parse_args(argv)
    if a.dump_values:
        sys.stdout.write(yaml.safe_dump(DEFAULT_VALUES, sort_keys=False))
        return 0
    values: dict = {}
    for f in a.values:
        values = merge_values(values, yaml.safe_load(Path(f).read_text()) or {})
    for expr in a.set:
        values = apply_set(values, expr)
    rendered = render(values)
    if a.stdout:
        docs = [text for rel, text in sorted(rendered.items()) if rel not in ("kustomization.yaml", "values.yaml")]
        sys.stdout.write("---\n".join(docs))
        return 0
    root = Path(a.out)
    stale = []
    for rel, text in rendered.items():
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
