"""nos-amd headline benchmark: fractional-GPU pods on MI355X.

The reference's one published benchmark (demos/gpu-sharing-comparison,
BASELINE.md) runs YOLOS-small inference pods that each request a 10 GB GPU
slice and reports per-pod latency / aggregate throughput for time-slicing,
MPS and MIG on one A100-80GB.  This bench runs the same workload MI355X-first:

1. control plane (untimed): the nos-amd scheduler + cumask partitioner +
   device plugin (in-process simulator) place fractional pods requesting
   ``amd.com/gpu-<slice>gb`` slices on an N-GPU node; the device plugin's
   allocations (XCD-symmetric CU masks) are what the tenants run with.  The
   number of such pods the node can hold is reported as
   ``schedulable_fractional_pods_per_node``;
2. data plane (timed): on every GPU (one rank per GPU), ``--pods-per-gpu``
   YOLOS-small pods (random-init weights, synthetic 800x1066 images, bf16),
   each on its own CU-masked HIP stream replaying its own HIP graph of the
   gfx950 kernels (MFMA GEMMs with fused epilogues, flash attention,
   LayerNorm).  A step = one inference by every pod.  Optionally a
   collective tenant per GPU runs GEMM + RCCL all-reduce over xGMI.

value = aggregate images/s over all pods of all GPUs (whole job).
vs_baseline = value / (21.89 img/s x n_gpus): 21.89 img/s is the reference's
best aggregate (MPS, 7 pods, 1x A100-80GB; BASELINE.md, derived from
README.md:70), scaled by the GPU count because the workload is weak-scaled.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

BASELINE_IMG_PER_S_PER_GPU = 21.89  # 7 / 0.3198 s, MPS, A100-80GB


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pods-per-gpu", type=int, default=8)
    ap.add_argument("--slice-gb", type=int, default=10, help="GPU memory per fractional pod (demo: 10)")
    ap.add_argument("--mode", choices=["cumask", "shared", "exclusive"], default="shared",
                    help="device-plugin CU policy of the 10 GB slices -- shared: memory-capped slices whose "
                         "kernels run concurrently on all CUs (the MPS behaviour of the reference demo); "
                         "cumask: each slice also gets exclusive XCD-symmetric CUs (compute isolation); "
                         "exclusive: one pod per GPU")
    ap.add_argument("--collective", action="store_true", help="add a GEMM + RCCL all-reduce tenant per GPU")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-control-plane", action="store_true")
    ap.add_argument("--gemm-impl", choices=["register", "lds"], default="register",
                    help="GEMM epilogue implementation (A/B switch; register is the default)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


def init_dist():
    """One rank per GPU over RCCL (backend "nccl").  NOS_AMD_BENCH_BACKEND=gloo
    rehearses the multi-rank path with several ranks sharing one GPU (RCCL
    refuses two ranks on one device): device = LOCAL_RANK mod device count."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("NOS_AMD_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def plan(args, world: int, num_cus: int) -> tuple[list[list[int] | None], dict]:
    """Per-pod CU masks for this GPU + control-plane facts."""
    from nos_amd.gpu.topology import split_even

    info: dict = {}
    if args.mode == "exclusive":
        return [None], info
    if not args.no_control_plane:
        from nos_amd.bench_support import control_plane_plan

        masks, info = control_plane_plan(n_gpus=world, pods_per_gpu=args.pods_per_gpu, slice_gb=args.slice_gb,
                                         num_cus=num_cus, local_gpu=int(os.environ.get("LOCAL_RANK", "0")),
                                         cu_policy="shared" if args.mode == "shared" else "even")
        return masks, info
    if args.mode == "shared":
        return [None] * args.pods_per_gpu, info
    return [s.cus() for s in split_even(args.pods_per_gpu)], info


def main(argv=None) -> int:
    args = parse_args(argv)
    world, rank, local = init_dist()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    from nos_amd.models.tenants import CollectiveTenant, InferenceTenants, TenantSpec
    from nos_amd.models.yolos import YolosConfig, demo_input_hw, flops_per_image, seq_len
    from nos_amd.ops import _lib
    from nos_amd.ops.streams import device_info

    _lib.require_native_on_gpu()
    dinfo = device_info(local)
    masks, cp = plan(args, world, dinfo["num_cus"])
    from nos_amd import ops

    # one pod owning the GPU wants latency-shaped GEMM tiles, co-running pods throughput-shaped ones
    ops.set_gemm_policy("latency" if len(masks) == 1 else "throughput")
    ops.set_gemm_impl(args.gemm_impl)
    cfg = YolosConfig.small()
    hw = demo_input_hw()
    specs = [TenantSpec(f"pod-{rank}-{i}", m) for i, m in enumerate(masks)]
    tenants = InferenceTenants(specs, dinfo["num_cus"], cfg, hw, use_graphs=not args.no_graphs)
    tenants.prepare()
    coll = CollectiveTenant(device=local) if args.collective else None

    smi = None
    try:
        from nos_amd.gpu.amdsmi import ActivitySampler, AmdSmi

        smi = AmdSmi.real()
    except Exception as e:  # amd-smi not usable on this box: util unreported
        print(f"[bench] amd-smi unavailable: {e}", file=sys.stderr)
        ActivitySampler = None  # type: ignore

    with torch.no_grad():
        for _ in range(args.warmup):
            tenants.launch_all()
            if coll:
                coll.step()
        tenants.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        sampler_gpu = [local]
        if smi is not None:
            try:
                # amd-smi enumerates physical GPUs; map by hip id when possible
                hip_ids = {g.hip_id: g.index for g in smi.gpus()}
                sampler_gpu = [hip_ids.get(local, local)]
            except Exception:
                pass
        sampler = ActivitySampler(smi, sampler_gpu, 0.02) if smi is not None else None
        if sampler:
            sampler.__enter__()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tenants.launch_all()
            if coll:
                coll.step()
        tenants.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if sampler:
            sampler.__exit__(None, None, None)

    util = sampler.mean() if sampler else None
    on_gpu = os.environ.get("NOS_AMD_BENCH_BACKEND", "nccl") == "nccl"
    t = torch.tensor([elapsed, util if util is not None else -1.0], dtype=torch.float64,
                     device="cuda" if on_gpu else "cpu")
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed = mx[0].item()
        util = t[1].item() / world if t[1].item() >= 0 else None
    n_pods_gpu = len(specs)
    images = args.steps * n_pods_gpu * world
    value = images / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    fl = flops_per_image(cfg, hw)
    result = {
        "metric": "fractional_pod_throughput_img_per_s",
        "value": round(value, 2),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (BASELINE_IMG_PER_S_PER_GPU * world), 2),
        "dtype": "bf16",
        "data": "synthetic (random-init YOLOS-small weights, random 800x1066 images)",
        "config": {
            "model": "YOLOS-small (hustvl/yolos-small architecture)",
            "global_batch": n_pods_gpu * world,
            "seq_len": seq_len(cfg, hw),
            "parallelism": f"{args.mode} x{n_pods_gpu} pods/GPU, {world} GPU(s)",
            "pods_per_gpu": n_pods_gpu,
            "slice_gb": args.slice_gb,
            "mode": args.mode,
            "collective_tenant": bool(args.collective),
            "graphs": not args.no_graphs,
        },
        "pod_latency_ms": round(ms_per_step, 3),
        "gpu_util_pct": None if util is None else round(util, 1),
        "achieved_tflops": round(value * fl / 1e12, 1),
        "schedulable_fractional_pods_per_node": cp.get("schedulable_fractional_pods_per_node"),
        "control_plane": cp,
        "baseline_img_per_s_per_gpu": BASELINE_IMG_PER_S_PER_GPU,
    }
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    tenants.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
