"""Component configuration kinds (``config.nos.nebuly.com/v1alpha1``).

Accept the same YAML as the reference (``pkg/api/nos.nebuly.com/config/v1alpha1/*.go``,
defaults in ``config/*/manager/*_config.yaml``) plus AMD fields.  NVIDIA-named
keys are accepted as aliases of the AMD ones so existing files keep working:

* ``nvidiaGpuResourceMemoryGB``  -> ``amdGpuResourceMemoryGB`` (default 288: one MI355X)
* ``knownMigGeometriesFile``     -> ``knownPartitionGeometriesFile``
* ``MigAgentConfig`` kind        -> ``PartitionAgentConfig``

Durations are plain seconds (the reference stores raw integers in
``time.Duration`` fields and multiplies by ``time.Second`` at use,
``cmd/gpupartitioner/gpupartitioner.go:194-195,240``).
"""
from __future__ import annotations

from pathlib import Path
from typing import Any

import yaml
from pydantic import BaseModel, ConfigDict, Field, field_validator, model_validator

from . import constants as C


class _M(BaseModel):
    model_config = ConfigDict(populate_by_name=True, extra="allow")


class HealthSpec(_M):
    health_probe_bind_address: str = Field(":8081", alias="healthProbeBindAddress")


class MetricsSpec(_M):
    bind_address: str = Field("127.0.0.1:8080", alias="bindAddress")


class WebhookSpec(_M):
    port: int = 9443


class LeaderElectionSpec(_M):
    leader_elect: bool = Field(False, alias="leaderElect")
    resource_name: str = Field("", alias="resourceName")
    resource_namespace: str = Field("nos-system", alias="resourceNamespace")
    release_on_cancel: bool = Field(False, alias="leaderElectionReleaseOnCancel")
    lease_duration_seconds: float = Field(15.0, alias="leaseDurationSeconds")


class ControllerManagerSpec(_M):
    api_version: str = Field(C.CONFIG_API_VERSION, alias="apiVersion")
    kind: str = ""
    health: HealthSpec = Field(default_factory=HealthSpec)
    metrics: MetricsSpec = Field(default_factory=MetricsSpec)
    webhook: WebhookSpec = Field(default_factory=WebhookSpec)
    leader_election: LeaderElectionSpec = Field(default_factory=LeaderElectionSpec, alias="leaderElection")
    log_level: str = Field("info", alias="logLevel")


class NamespacedObject(_M):
    name: str = ""
    namespace: str = ""


def _alias(data: Any, old: str, new: str) -> Any:
    if isinstance(data, dict) and old in data and new not in data:
        data = dict(data)
        data[new] = data.pop(old)
    return data


class OperatorConfig(ControllerManagerSpec):
    kind: str = "OperatorConfig"
    amd_gpu_resource_memory_gb: int = Field(C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB, alias="amdGpuResourceMemoryGB")

    @model_validator(mode="before")
    @classmethod
    def _aliases(cls, d):
        return _alias(d, "nvidiaGpuResourceMemoryGB", "amdGpuResourceMemoryGB")


class GpuPartitionerConfig(ControllerManagerSpec):
    kind: str = "GpuPartitionerConfig"
    scheduler_config_file: str = Field("", alias="schedulerConfigFile")
    known_partition_geometries_file: str = Field("", alias="knownPartitionGeometriesFile")
    batch_window_timeout_seconds: float = Field(60.0, alias="batchWindowTimeoutSeconds")
    batch_window_idle_seconds: float = Field(10.0, alias="batchWindowIdleSeconds")
    device_plugin_config_map: NamespacedObject = Field(
        default_factory=lambda: NamespacedObject(name=C.DEFAULT_DEVICE_PLUGIN_CM_NAME,
                                                 namespace=C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE),
        alias="devicePluginConfigMap")
    device_plugin_delay_seconds: float = Field(5.0, alias="devicePluginDelaySeconds")
    # new: repartition of a GPU-wide mode may take seconds; the plan handshake times out after this
    plan_report_timeout_seconds: float = Field(300.0, alias="planReportTimeoutSeconds")
    amd_gpu_resource_memory_gb: int = Field(C.DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB, alias="amdGpuResourceMemoryGB")
    # new: CU-mask slice placement over a node's GPUs ("pack" = reference first-fit, "spread")
    slice_placement: str = Field("pack", alias="slicePlacement")
    # new: CU-mask layout of a GPU's slices in the device plugin ("even" | "proportional" | "shared" |
    # "split": slices of ``isolatedProfiles`` get proportional masks inside ``isolatedCuSlots`` CU slots
    # per XCD reserved for them, every other slice shares the remaining slots -- an isolated pool and a
    # shared pool on one GPU)
    cu_policy: str = Field("proportional", alias="cuPolicy")
    isolated_profiles: list[str] = Field(default_factory=list, alias="isolatedProfiles")
    isolated_cu_slots: int = Field(0, alias="isolatedCuSlots")
    # amdpart anti-starvation: whole (SPX) GPUs per node never split for fractional pods
    reserve_whole_gpus: int = Field(0, alias="reserveWholeGpus")
    # NPS mode the planner asks for when a geometry exists in several memory modes
    preferred_memory_mode: str = Field("NPS1", alias="preferredMemoryMode")

    @model_validator(mode="before")
    @classmethod
    def _aliases(cls, d):
        d = _alias(d, "knownMigGeometriesFile", "knownPartitionGeometriesFile")
        return _alias(d, "nvidiaGpuResourceMemoryGB", "amdGpuResourceMemoryGB")

    def validate_config(self) -> None:
        """``GpuPartitionerConfig.Validate`` (gpu_partitioner_config.go:39-50)."""
        if self.batch_window_timeout_seconds <= 0:
            raise ValueError("batchWindowTimeoutSeconds must be greater than 0")
        if self.batch_window_idle_seconds <= 0:
            raise ValueError("batchWindowIdleSeconds must be greater than 0")
        if self.device_plugin_delay_seconds <= 0:
            raise ValueError("devicePluginDelaySeconds must be greater than 0")
        if self.slice_placement not in ("pack", "spread", "measured"):
            raise ValueError("slicePlacement must be 'pack', 'spread' or 'measured'")
        if self.cu_policy not in ("even", "proportional", "shared", "split"):
            raise ValueError("cuPolicy must be 'even', 'proportional', 'shared' or 'split'")
        if self.cu_policy == "split" and not (self.isolated_profiles and 0 < self.isolated_cu_slots < 32):
            raise ValueError("cuPolicy split needs isolatedProfiles and 0 < isolatedCuSlots < 32")

    def with_defaults(self) -> "GpuPartitionerConfig":
        """Default the device-plugin ConfigMap name/namespace when missing
        (``cmd/gpupartitioner/gpupartitioner.go:102-121``)."""
        if not self.device_plugin_config_map.name:
            self.device_plugin_config_map.name = C.DEFAULT_DEVICE_PLUGIN_CM_NAME
        if not self.device_plugin_config_map.namespace:
            self.device_plugin_config_map.namespace = C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE
        return self


class PartitionAgentConfig(ControllerManagerSpec):
    """MigAgentConfig analogue (mig_agent_config.go:27-31)."""

    kind: str = "PartitionAgentConfig"
    report_config_interval_seconds: float = Field(10.0, alias="reportConfigIntervalSeconds")
    allow_mode_changes: bool = Field(False, alias="allowModeChanges")
    mode_switch_timeout_seconds: float = Field(120.0, alias="modeSwitchTimeoutSeconds")
    default_compute_mode: str = Field("SPX", alias="defaultComputeMode")
    default_memory_mode: str = Field("NPS1", alias="defaultMemoryMode")

    @field_validator("report_config_interval_seconds")
    @classmethod
    def _pos(cls, v):
        if v <= 0:
            raise ValueError("reportConfigIntervalSeconds must be > 0")
        return v


class GpuAgentConfig(ControllerManagerSpec):
    """GpuAgentConfig (gpu_agent_config.go:27-31) + probe settings."""

    kind: str = "GpuAgentConfig"
    report_config_interval_seconds: float = Field(10.0, alias="reportConfigIntervalSeconds")
    probe_enabled: bool = Field(True, alias="probeEnabled")
    probe_interval_seconds: float = Field(300.0, alias="probeIntervalSeconds")
    probe_gemm_size: int = Field(4096, alias="probeGemmSize")
    # > 0: the node runs the pod server (nos_amd/podserver) with this many
    # tenants per GPU; published as nos.nebuly.com/pod-server.tenants, it lifts
    # the HWS process bound on cumask slices per GPU
    pod_server_tenants: int = Field(0, alias="podServerTenants")


class DevicePluginConfig(ControllerManagerSpec):
    kind: str = "DevicePluginConfig"
    config_map: NamespacedObject = Field(
        default_factory=lambda: NamespacedObject(name=C.DEFAULT_DEVICE_PLUGIN_CM_NAME,
                                                 namespace=C.DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE),
        alias="configMap")
    socket_dir: str = Field(C.DEVICE_PLUGIN_DIR, alias="socketDir")
    # how CU masks are assigned to cumask slices: "even" (split the GPU's CUs
    # evenly among the slices of its geometry), "proportional" (to memory),
    # "shared" (no mask; MPS-without-limits semantics)
    cu_policy: str = Field("proportional", alias="cuPolicy")
    # HIP_VISIBLE_DEVICES of an allocation: "container" (0..k-1 over the render
    # nodes mounted into the container) or "host" (host HIP ids, bare metal)
    device_env: str = Field("container", alias="deviceEnv")
    # seconds between amd-smi rescans (modes switched by the partition agent) and
    # reads of the node's partitioning label
    rescan_seconds: float = Field(5.0, alias="rescanSeconds")
    # pod-server slices (nos_amd/podserver, the MPS analogue): slices of a cumask
    # node are served by the node's pod server, one per GPU at
    # <podServerSocketDir>/gpu-<index>.sock; pods get that socket (mounted) and
    # their slice, never a device node.  "" = pods run as GPU processes.
    pod_server_socket_dir: str = Field("", alias="podServerSocketDir")


class MetricsExporterConfig(_M):
    endpoint: str = ""
    enabled: bool = False


KINDS: dict[str, type[ControllerManagerSpec]] = {
    "OperatorConfig": OperatorConfig,
    "GpuPartitionerConfig": GpuPartitionerConfig,
    "PartitionAgentConfig": PartitionAgentConfig,
    "MigAgentConfig": PartitionAgentConfig,
    "GpuAgentConfig": GpuAgentConfig,
    "DevicePluginConfig": DevicePluginConfig,
}


def load(path: str | Path, expected_kind: str | None = None) -> ControllerManagerSpec:
    """``ctrl.ConfigFile().AtPath(file).OfKind(&cfg)`` equivalent."""
    data = yaml.safe_load(Path(path).read_text()) or {}
    return parse(data, expected_kind)


def parse(data: dict, expected_kind: str | None = None) -> ControllerManagerSpec:
    kind = data.get("kind") or expected_kind
    if kind not in KINDS:
        raise ValueError(f"unknown config kind {kind!r}")
    cls = KINDS[kind]
    if expected_kind and KINDS.get(expected_kind) is not cls:
        raise ValueError(f"expected config kind {expected_kind}, got {kind}")
    cfg = cls.model_validate(data)
    if isinstance(cfg, GpuPartitionerConfig):
        cfg.with_defaults().validate_config()
    return cfg
