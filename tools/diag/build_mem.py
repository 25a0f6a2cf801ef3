"""Where a pod-server build's measured peak comes from (one tenant program):
device memory after compile, input, eager warm-up, graph capture."""
import sys

import torch

sys.path.insert(0, ".")
from nos_amd import ops  # noqa: E402
from nos_amd.models.yolos import GraphedTenant  # noqa: E402
from nos_amd.models.yolos_program import demo_tenant  # noqa: E402
from nos_amd.podserver import program as PG  # noqa: E402

ops.set_f32_math("h3")
ops.set_attention_f32_variant("h3n")
torch.cuda.set_device(0)
for small in (False, True):
    prog, w = demo_tenant("fp32", 0, small=small)
    p = PG.parse(prog, w, gpu=True)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    mb = lambda: (round((torch.cuda.memory_allocated() - base) / 2**20, 1), round((torch.cuda.max_memory_allocated() - base) / 2**20, 1))  # noqa: E731
    s = torch.cuda.Stream()
    with torch.no_grad(), torch.cuda.stream(s):
        m = p.compile("cuda")
        print("compiled", mb(), "est", round(p.bytes_estimate / 2**20, 1), "params", round(p.param_bytes / 2**20, 1))
        x = p.input_tensor("cuda")
        m(x)
        s.synchronize()
        print("eager", mb())
        gt = GraphedTenant(m, s, x)
        gt.capture(warmup=1, capture_error_mode="thread_local", light=True)
        s.synchronize()
        print("captured", mb())
    del m, gt, x
    torch.cuda.empty_cache()
