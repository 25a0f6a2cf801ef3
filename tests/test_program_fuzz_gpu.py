"""Fuzzing the shared GPU pod server: hypothesis draws
random programs (tests/program_fuzz.py -- MLP chains with strided slices and
norms, fused-QKV attention, grouped-query / causal / rotary sdpa, conv nets
with grouped, depthwise, strided and dilated convs, activation x activation
matmul; dims around the tile edges 1, 31, 33, 127, 129; fp32 and bf16).  Every
program the validator accepts is registered on ONE pod server (HIP graphs
captured, as for any tenant), run once and compared with its eager fp32 CPU
reference; every program it refuses must be refused by the server too, before
anything is built.  A YOLOS co-tenant answers between examples and must keep
returning its first output bit for bit: a fuzzed tenant never disturbs it.
The tenants share one HIP context, so the validator plus the kernels' own
bounds are the only guard (docs/podserver.md)."""
from __future__ import annotations

import collections

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings

pytestmark = pytest.mark.gpu

from nos_amd import ops  # noqa: E402
from nos_amd.podserver import program as PG  # noqa: E402
from nos_amd.podserver.client import PodClient, PodServerError  # noqa: E402

from program_fuzz import programs, tolerance  # noqa: E402

STATS: collections.Counter = collections.Counter()


@pytest.fixture(scope="module")
def fleet(tmp_path_factory):
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver.server import PodServer

    ops.set_f32_math("h3")
    srv = PodServer(tmp_path_factory.mktemp("fz") / "s.sock", device="cuda", lanes=4, memory_gb=200).start()
    y = PodClient(srv.path, connect_timeout_s=60)
    y.register("yolos", *demo_tenant("fp32", 0, small=True), memory_limit_gb=4)
    first = y.infer(outputs=True)[0]
    yield srv, y, first
    y.close()
    srv.stop()


@settings(max_examples=400, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(case=programs(gpu=True))
def test_fuzzed_programs_run_correctly_beside_a_yolos_tenant(fleet, case):
    srv, yolos, first = fleet
    prog, w, data, fam = case
    try:
        p = PG.parse(prog, w, gpu=True)
    except PG.ProgramError:
        p = None
    c = PodClient(srv.path, connect_timeout_s=30)
    try:
        if p is None:
            with pytest.raises(PodServerError, match="ProgramError"):
                c.register("fz", prog, w, memory_limit_gb=4)
            STATS["refused"] += 1
            return
        c.register("fz", prog, w, memory_limit_gb=4)
        outs, _ = c.infer(data, outputs=True)
    finally:
        c.close()
    x = p.input_tensor("cpu", data)
    with torch.no_grad():
        ref = p.reference(x)
    rel, ab = tolerance(p.values[p.outputs[0]].dtype)
    for g, r in zip(outs, ref):
        g, r = torch.from_numpy(g).float(), r.float()
        assert g.shape == r.shape, (fam, g.shape, r.shape)
        assert torch.equal(torch.isnan(g), torch.isnan(r)), fam
        err = float((g - r).nan_to_num().abs().max()) if r.numel() else 0.0
        assert err <= rel * float(r.nan_to_num().abs().max()) + ab, (fam, err, prog["name"])
    STATS["ran"] += 1
    STATS[fam] += 1
    y = yolos.infer(outputs=True)[0]
    assert all(np.array_equal(a, b) for a, b in zip(y, first)), "the co-tenant's output changed"


def test_fuzz_covered_enough(fleet):
    """Runs after the property test (file order): at least 200 accepted
    programs ran, every family among them."""
    assert STATS["ran"] >= 200, dict(STATS)
    assert all(STATS[f] > 0 for f in ("mlp", "attn", "sdpa", "conv", "matmul", "decode")), dict(STATS)
