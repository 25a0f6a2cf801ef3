"""nos_amd -- an MI355X-native Kubernetes GPU-sharing stack with the capabilities of nos.

Subpackages (see SURVEY.md section 1 for the layer map):

* ``api``           CRDs, labels, annotations, component configs (L2)
* ``resource``/``gpu``  resource math, device model, AMD partition + CU-mask slicing models (L1)
* ``sim``           in-process API server + kubelet simulator (replaces envtest/kind)
* ``runtime``       controller runtime (work queues, manager, leader election)
* ``scheduler``     scheduler framework + CapacityScheduling elastic-quota plugin
* ``partitioning``  planner / snapshot / actuator + amdpart and cumask strategies (L3)
* ``controllers``   operator, gpupartitioner, partition agent, gpuagent (L4)
* ``deviceplugin``  nos-amd device plugin (partitions and CU-mask slices)
* ``ops``           gfx950 HIP kernels (attention, GEMM, LayerNorm, probes, CU-mask streams)
* ``models``        tenant workloads (YOLOS detector, GEMM + RCCL all-reduce trainer)
* ``parallel``      torch.distributed / RCCL helpers for tenants
* ``cmd``           component entry points (operator, scheduler, gpupartitioner, ...)
"""
__version__ = "0.1.0"
