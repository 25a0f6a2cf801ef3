"""Names shared by every component: labels, annotations, resources, defaults.

Kept API-compatible with the reference where the reference's names are not
NVIDIA-specific (``pkg/api/nos.nebuly.com/v1alpha1/{labels,annotations,constants}.go``,
``pkg/constant/constants.go``); NVIDIA names are replaced by AMD ones.
"""
from __future__ import annotations

# --------------------------------------------------------------- API group
GROUP = "nos.nebuly.com"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"
CONFIG_API_VERSION = "config.nos.nebuly.com/v1alpha1"

# --------------------------------------------------------------- labels
# v1alpha1/labels.go:19-24
LABEL_CAPACITY_INFO = "nos.nebuly.com/capacity"
LABEL_GPU_PARTITIONING = "nos.nebuly.com/gpu-partitioning"

CAPACITY_IN_QUOTA = "in-quota"      # pkg/constant/constants.go:24-29
CAPACITY_OVER_QUOTA = "over-quota"

# PartitioningKind values (pkg/gpu/partitioning.go:87-91 had mig|mps|hybrid)
PARTITIONING_AMDPART = "partition"  # compute/memory partition modes (MIG analogue)
PARTITIONING_CUMASK = "cumask"      # CU-mask slices (MPS analogue)
PARTITIONING_HYBRID = "hybrid"      # partition modes + memory slices per partition (gpu/hybrid.py)
PARTITIONING_KINDS = (PARTITIONING_AMDPART, PARTITIONING_CUMASK, PARTITIONING_HYBRID)

# --------------------------------------------------------------- annotations
# v1alpha1/annotations.go:21-58 -- kept exactly
ANNOTATION_GPU_SPEC_PREFIX = "nos.nebuly.com/spec-gpu"
ANNOTATION_GPU_STATUS_PREFIX = "nos.nebuly.com/status-gpu"
ANNOTATION_PARTITIONING_PLAN = "nos.nebuly.com/spec-partitioning-plan"
ANNOTATION_REPORTED_PARTITIONING_PLAN = "nos.nebuly.com/status-partitioning-plan"
ANNOTATION_GPU_STATUS_FORMAT = ANNOTATION_GPU_STATUS_PREFIX + "-{index}-{profile}-{status}"
ANNOTATION_GPU_SPEC_FORMAT = ANNOTATION_GPU_SPEC_PREFIX + "-{index}-{profile}"
# new: measured per-slice throughput published by the gpuagent probe
ANNOTATION_SLICE_TFLOPS_FORMAT = "nos.nebuly.com/probe-gpu-{index}-{profile}-tflops"
ANNOTATION_SLICE_GBPS_FORMAT = "nos.nebuly.com/probe-gpu-{index}-{profile}-gbps"
ANNOTATION_PROBE_PREFIX = "nos.nebuly.com/probe-gpu"
# new: desired/current partition modes written by the amdpart strategy / agent
ANNOTATION_SPEC_MODE_FORMAT = "nos.nebuly.com/spec-mode-gpu-{index}"
ANNOTATION_STATUS_MODE_FORMAT = "nos.nebuly.com/status-mode-gpu-{index}"
# set by the partition agent while a GPU's last mode switch failed or is still
# running past its deadline (value: the reason); removed once the GPU is healthy
ANNOTATION_STATUS_ERROR_FORMAT = "nos.nebuly.com/status-error-gpu-{index}"
ANNOTATION_STATUS_ERROR_PREFIX = "nos.nebuly.com/status-error-gpu-"
MODE_SWITCHING = "SWITCHING"

# --------------------------------------------------------------- resources
RESOURCE_GPU_MEMORY = "nos.nebuly.com/gpu-memory"  # v1alpha1/constants.go:24-27 (GB)
RESOURCE_AMD_GPU = "amd.com/gpu"
AMD_RESOURCE_PREFIX = "amd.com/"
AMD_PARTITION_RESOURCE_PREFIX = "amd.com/partition-"
AMD_SLICE_RESOURCE_PREFIX = "amd.com/gpu-"
REGEX_AMD_PARTITION_RESOURCE = r"^amd\.com/partition-(\d+xcd\.\d+gb)$"
REGEX_AMD_PARTITION_PROFILE = r"^(\d+)xcd\.(\d+)gb$"
REGEX_AMD_SLICE_RESOURCE = r"^amd\.com/gpu-(\d+gb)$"
REGEX_AMD_SLICE_PROFILE = r"^(\d+)gb$"
REGEX_MEMORY_GB = r"(\d+)gb"

# --------------------------------------------------------------- node labels
# written by the nos-amd partition agent / gpuagent from amd-smi (the role of
# the NVIDIA GPU operator's gpu.product/count/memory labels, constants.go:78-87)
LABEL_AMD_PRODUCT = "amd.com/gpu.product"
LABEL_AMD_COUNT = "amd.com/gpu.count"
LABEL_AMD_MEMORY = "amd.com/gpu.memory"          # MB, like the NVIDIA label
LABEL_AMD_XCDS = "amd.com/gpu.xcds"
LABEL_AMD_CUS = "amd.com/gpu.cus"
LABEL_AMD_COMPUTE_MODE = "amd.com/gpu.compute-partition"
LABEL_AMD_MEMORY_MODE = "amd.com/gpu.memory-partition"
# processes the amdgpu HWS runs concurrently per logical GPU (hws_max_conc_proc, gpu/kfd.py)
LABEL_AMD_MAX_PROCS = "amd.com/gpu.max-concurrent-processes"
LABEL_DEVICE_PLUGIN_CONFIG = "nos.nebuly.com/device-plugin.config"
# tenants the node's pod server (nos_amd/podserver, MPS analogue) hosts per GPU:
# present = slices are served by the pod server, and this replaces the HWS
# process bound on slices per GPU (the server is ONE GPU process)
LABEL_POD_SERVER_TENANTS = "nos.nebuly.com/pod-server.tenants"

# --------------------------------------------------------------- env
ENV_NODE_NAME = "NODE_NAME"
ENV_CU_MASK = "ROC_GLOBAL_CU_MASK"
ENV_VISIBLE_DEVICES = "HIP_VISIBLE_DEVICES"
ENV_MEMORY_LIMIT_GB = "NOS_AMD_MEMORY_LIMIT_GB"
ENV_POD_SERVER = "NOS_AMD_POD_SERVER"        # pod-server socket of the slice's GPU
ENV_POD_CU_MASK = "NOS_AMD_POD_CU_MASK"      # CU mask the pod server applies to the tenant's stream
ENV_POD_TOKEN = "NOS_AMD_POD_TOKEN"          # per-allocation token: the pod server's key to the slice record
DEFAULT_POD_SERVER_SOCKET_DIR = "/run/nos-amd/podserver"

# --------------------------------------------------------------- defaults
DEFAULT_AMD_GPU_RESOURCE_MEMORY_GB = 288   # one MI355X (HBM3E)
DEFAULT_PODRESOURCES_TIMEOUT_S = 10.0
DEFAULT_PODRESOURCES_MAX_MSG = 16 * 1024 * 1024
DEFAULT_DEVICE_PLUGIN_CM_NAME = "nos-amd-device-plugin-configs"
DEFAULT_DEVICE_PLUGIN_CM_NAMESPACE = "nos-system"
DEFAULT_DEVICE_PLUGIN_DS_LABEL = ("app", "nos-amd-device-plugin")
KUBELET_PODRESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
DEVICE_PLUGIN_DIR = "/var/lib/kubelet/device-plugins/"

# --------------------------------------------------------------- controller names
ELASTIC_QUOTA_CONTROLLER = "eq-controller"
COMPOSITE_ELASTIC_QUOTA_CONTROLLER = "ceq-controller"
CLUSTER_STATE_NODE_CONTROLLER = "clusterstate-node-controller"
CLUSTER_STATE_POD_CONTROLLER = "clusterstate-pod-controller"
AMDPART_PARTITIONER_CONTROLLER = "amdpart-partitioner-controller"
CUMASK_PARTITIONER_CONTROLLER = "cumask-partitioner-controller"

INTERNAL_ERROR_MSG = "internal error"

# --------------------------------------------------------------- field indexes
POD_PHASE_KEY = "status.phase"
POD_NODE_NAME_KEY = "spec.nodeName"
