"""Correctness of a pod-server tenant's two HIP graphs (co-tenancy and solo),
alone and under a concurrent co-tenant, against eager runs of the same
program under the same kernel configs.

python tools/graph_check.py [--json out.json]

Prints one JSON object: max |diff| / max |ref| per check.  A co-tenancy graph
must match the eager co-tenancy-config run bit for bit, the solo graph the
eager whole-GPU-config run; "concurrent" replays the co-tenancy graph while
another tenant's graph replays on a second stream.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-solo", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch

    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.server import PodServer

    srv = PodServer("/tmp/nos_graph_check/gpu-0/server.sock", device="cuda", lanes=2, max_tenants=8,
                    solo_graphs=not a.no_solo)
    srv._init_device()
    out: dict = {"kernel_config": srv.kernel_config, "solo_config": srv.solo_config}

    def rel(x, r):
        x, r = x.float().cpu(), r.float().cpu()
        return float((x - r).abs().max() / (r.abs().max() + 1e-12))

    yolos = demo_tenant("fp32", 4)
    mlp = PG.mlp_program(dim=1024, layers=4, batch=256, dtype="bf16", seed=5)
    ta = srv._build(1, {"pod": "yolos"}, PG.parse(*yolos, gpu=True), 10.0, None)
    tb = srv._build(2, {"pod": "mlp"}, PG.parse(*mlp, gpu=True), 2.0, None)
    rng = np.random.default_rng(6)
    for t in (ta, tb):
        x = rng.standard_normal(tuple(t.x.shape)).astype(np.float32)
        t.x.copy_(torch.from_numpy(x).to(t.x.dtype).cuda())
    torch.cuda.synchronize()
    s1, s2 = srv._lanes
    res = {}
    with torch.no_grad():
        for name, t in (("yolos", ta), ("mlp", tb)):
            srv._apply_config(srv.kernel_config)
            eager_co = [o.clone() for o in t.model(t.x)]
            torch.cuda.synchronize()
            with torch.cuda.stream(s1):
                t.graph.replay()
            s1.synchronize()
            res[f"{name}_graph_vs_eager_co"] = [rel(o, r) for o, r in zip(t.outputs, eager_co)]
            if t.solo_graph is not None:
                srv._apply_config(srv.solo_config)
                eager_solo = [o.clone() for o in t.model(t.x)]
                srv._apply_config(srv.kernel_config)
                torch.cuda.synchronize()
                with torch.cuda.stream(s1):
                    t.solo_graph.replay()
                s1.synchronize()
                res[f"{name}_solo_vs_eager_solo"] = [rel(o, r) for o, r in zip(t.solo_outputs, eager_solo)]
                with torch.cuda.stream(s1):
                    t.graph.replay()
                s1.synchronize()
                res[f"{name}_graph_after_solo_vs_eager_co"] = [rel(o, r) for o, r in zip(t.outputs, eager_co)]
            res[f"{name}_eager_co_vs_reference"] = [
                rel(o, r) for o, r in zip(eager_co, PG.parse(*(yolos if name == "yolos" else mlp)).reference(
                    t.x.float().cpu()))]
            if name == "yolos":
                ref_co = eager_co
        # concurrent: A's co-tenancy graph while B's graph replays on the other lane
        bad = []
        stop = threading.Event()

        def hammer():
            while not stop.is_set():
                with torch.cuda.stream(s2):
                    tb.graph.replay()
                s2.synchronize()

        th = threading.Thread(target=hammer)
        th.start()
        try:
            for _ in range(8):
                with torch.cuda.stream(s1):
                    ta.graph.replay()
                s1.synchronize()
                bad.append([rel(o, r) for o, r in zip(ta.outputs, ref_co)])
        finally:
            stop.set()
            th.join()
        res["yolos_graph_concurrent_vs_eager_co"] = bad
        # the same two graphs of the built-in YolosDetector (round-3 server path)
        from nos_amd.models.yolos import GraphedTenant, YolosConfig, YolosDetector
        from nos_amd.models.yolos_program import yolos_weights

        m = YolosDetector(YolosConfig.small())
        m.load_numpy(yolos_weights(YolosConfig.small(), 4))
        m = m.cuda().eval()
        x = ta.x.clone()
        srv._apply_config(srv.kernel_config)
        g1 = GraphedTenant(m, srv._setup_stream, x)
        g1.capture(capture_error_mode="thread_local")
        if srv.solo_config is not None:
            g2 = GraphedTenant(m, srv._setup_stream, x)
            srv._apply_config(srv.solo_config)
            g2.capture(capture_error_mode="thread_local", pool=g1.graph.pool())
            srv._apply_config(srv.kernel_config)
        with torch.cuda.stream(s1):
            g1.graph.replay()
        s1.synchronize()
        res["detector_graph_vs_program_eager_co"] = [rel(o, r) for o, r in zip(g1.outputs, ref_co)]
    out["checks"] = res
    line = json.dumps(out)
    print(line)
    if a.json:
        Path(a.json).write_text(line + "\n")
    for t in (ta, tb):
        srv._free(t)
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
