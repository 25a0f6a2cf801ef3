"""Prometheus metrics of the nos-amd components.

The reference exposes only controller-runtime defaults; these are the
metrics the north-star measurement needs (plan latency, repartition time,
pending fractional pods, schedulable fractional pods per node, GPU
utilisation, probe-measured slice throughput, tenant step time / all-reduce
bandwidth).  All live in one registry so an in-process simulator can expose
or scrape them without a server.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

REGISTRY = CollectorRegistry(auto_describe=True)

PLAN_DURATION = Histogram("nos_plan_duration_seconds", "gpupartitioner planning time", ["kind"],
                          registry=REGISTRY, buckets=(0.001, 0.005, 0.01, 0.05, 0.1, 0.5, 1, 5, 10))
PLANS_APPLIED = Counter("nos_plans_applied_total", "partitioning plans applied", ["kind"], registry=REGISTRY)
REPARTITION_DURATION = Histogram("nos_repartition_duration_seconds", "GPU mode switch time", ["mode"],
                                 registry=REGISTRY, buckets=(0.01, 0.1, 0.5, 1, 2, 5, 10, 30, 60, 120))
PENDING_FRACTIONAL_PODS = Gauge("nos_pending_fractional_pods", "pending pods requesting GPU fractions",
                                registry=REGISTRY)
SCHEDULABLE_PODS_PER_NODE = Gauge("nos_schedulable_fractional_pods_per_node",
                                  "fractional pods a node can host", ["node", "profile"], registry=REGISTRY)
GPU_UTIL = Gauge("nos_gpu_util_percent", "GPU gfx activity", ["node", "gpu"], registry=REGISTRY)
SLICE_TFLOPS = Gauge("nos_slice_tflops", "probe-measured bf16 MFMA TFLOP/s of a slice",
                     ["node", "gpu", "profile"], registry=REGISTRY)
SLICE_GBPS = Gauge("nos_slice_hbm_gbps", "probe-measured HBM GB/s of a slice", ["node", "gpu", "profile"],
                   registry=REGISTRY)
TENANT_STEP = Histogram("nos_tenant_step_time_seconds", "tenant step time", ["tenant"], registry=REGISTRY)
ALLREDUCE_BUSBW = Gauge("nos_allreduce_busbw_gbps", "tenant all-reduce bus bandwidth", ["tenant"],
                        registry=REGISTRY)
RECONCILES = Counter("nos_reconciles_total", "reconcile calls", ["controller", "result"], registry=REGISTRY)
INFERENCE_TIME = Histogram("inference_time_seconds", "Time required for running a single inference",
                           registry=REGISTRY)  # same name as the reference demo client
# pod server (nos_amd/podserver): tenants hosted, requests waiting for a lane,
# completed inferences per pod, request latency (queue + replay)
PODSERVER_TENANTS = Gauge("nos_podserver_tenants", "pods hosted by the GPU's pod server", ["gpu"],
                          registry=REGISTRY)
PODSERVER_QUEUED = Gauge("nos_podserver_queued_requests", "requests waiting for a lane", ["gpu"], registry=REGISTRY)
PODSERVER_INFERENCES = Counter("nos_podserver_inferences_total", "inferences run for a pod", ["gpu", "pod"],
                               registry=REGISTRY)
PODSERVER_REQUEST_TIME = Histogram("nos_podserver_request_seconds", "pod-server request time (queue + replay)",
                                   ["gpu"], registry=REGISTRY,
                                   buckets=(0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1))


def exposition() -> bytes:
    return generate_latest(REGISTRY)


def serve(port: int) -> None:  # pragma: no cover - network side effect
    from prometheus_client import start_http_server

    start_http_server(port, registry=REGISTRY)
