"""Property-based test of the program compiler on the CPU (hypothesis):
random validator-accepted programs (tests/program_fuzz.py: MLP chains,
attention, decoder sdpa, conv nets, matmul) compiled for the CPU -- every
lowering pass applied -- agree with their unfused eager fp32 reference.  The
GPU twin (tests/test_program_fuzz_gpu.py) runs the same programs on the pod
server's gfx950 kernels."""
from __future__ import annotations

import numpy as np
import torch
from hypothesis import HealthCheck, given, settings

from nos_amd.podserver import program as PG

from program_fuzz import programs, tolerance


@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(programs(gpu=False))
def test_compiled_programs_match_their_reference(case):
    prog, w, data, fam = case
    try:
        p = PG.parse(prog, w)
    except PG.ProgramError:
        return   # refused before anything was allocated: fine
    x = p.input_tensor("cpu", data)
    with torch.no_grad():
        ref = p.reference(x)
        got = p.compile("cpu")(x)
    dt = p.values[p.outputs[0]].dtype
    rel, ab = tolerance(dt)
    for g, r in zip(got, ref):
        g, r = g.float(), r.float()
        assert g.shape == r.shape, (fam, g.shape, r.shape)
        assert torch.equal(torch.isnan(g), torch.isnan(r)), fam
        err = float((g - r).nan_to_num().abs().max()) if r.numel() else 0.0
        assert err <= rel * float(r.nan_to_num().abs().max()) + ab, (fam, dt, err)
