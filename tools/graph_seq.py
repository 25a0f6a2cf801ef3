"""Replay-by-replay correctness of a freshly built pod-server tenant's graphs
(diagnostic for tools/graph_check.py): error of each replay against the
eager run of the same program and configs."""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    import numpy as np
    import torch

    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.server import PodServer

    out = {}
    for solo in (False, True):
        srv = PodServer("/tmp/nos_graph_seq/gpu-0/server.sock", device="cuda", lanes=2, solo_graphs=solo)
        srv._init_device()
        t = srv._build(1, {"pod": "y"}, PG.parse(*demo_tenant("fp32", 4), gpu=True), 10.0, None)
        x = np.random.default_rng(6).standard_normal(tuple(t.x.shape)).astype(np.float32)
        s1 = srv._lanes[0]
        seq = []

        def rel():
            return [float((o.float().cpu() - r.float().cpu()).abs().max() / r.float().cpu().abs().max())
                    for o, r in zip(t.outputs, ref)]

        with torch.no_grad():
            # replays BEFORE any eager run after the build, with the zero input the graph was captured on
            zin = [o.clone() for o in t.model(t.x)]
            ref = zin
            for _ in range(3):
                with torch.cuda.stream(s1):
                    t.graph.replay()
                s1.synchronize()
                seq.append(("zero_input", rel()))
            t.x.copy_(torch.from_numpy(x).cuda())
            torch.cuda.synchronize()
            ref = [o.clone() for o in t.model(t.x)]
            torch.cuda.synchronize()
            for _ in range(3):
                with torch.cuda.stream(s1):
                    t.graph.replay()
                s1.synchronize()
                seq.append(("new_input", rel()))
            # input copied on the lane stream right before the replay (the server's _run)
            x2 = np.random.default_rng(7).standard_normal(tuple(t.x.shape)).astype(np.float32)
            with torch.cuda.stream(s1):
                t.x.copy_(torch.from_numpy(x2).view(t.x.shape).to(t.x.dtype))
                t.graph.replay()
            s1.synchronize()
            ref = [o.clone() for o in t.model(t.x)]
            torch.cuda.synchronize()
            seq.append(("lane_copy_then_replay", rel()))
            with torch.cuda.stream(s1):
                t.graph.replay()
            s1.synchronize()
            seq.append(("replay_again", rel()))
        out[f"solo={solo}"] = seq
        srv._free(t)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
