"""Which op of a program makes its captured HIP graph diverge from eager
execution after the input changes (diagnostic): truncate the YOLOS program
at several nodes, capture each prefix on a zero input, write a random input,
replay, compare with eager."""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> int:
    import copy

    import numpy as np
    import torch

    from nos_amd import ops
    from nos_amd.models.pod import kernel_config
    from nos_amd.models.yolos_program import demo_tenant
    from nos_amd.podserver import program as PG
    from nos_amd.podserver.server import PodServer

    PodServer._apply_config(kernel_config(0.5, {}, 0))
    prog, w = demo_tenant("fp32", 4)
    names = [n["output"] for n in prog["nodes"]]
    picks = list(range(0, 12)) + [16, 20, 24, 30, 40, len(names) - 1]
    out = {}
    rng = np.random.default_rng(0)
    s = torch.cuda.Stream()
    for k in picks:
        p = copy.deepcopy(prog)
        p["nodes"] = p["nodes"][:k + 1]
        p["outputs"] = [names[k]]
        P = PG.parse(p, w, gpu=True)
        with torch.no_grad():
            m = P.compile("cuda")
            x = P.input_tensor("cuda")
            with torch.cuda.stream(s):
                for _ in range(2):
                    m(x)
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                y = m(x)
            x.copy_(torch.from_numpy(rng.standard_normal(tuple(x.shape)).astype(np.float32)).cuda())
            torch.cuda.synchronize()
            ref = m(x)[0].clone()
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                g.replay()
            s.synchronize()
            d = float((y[0].float() - ref.float()).abs().max() / (ref.float().abs().max() + 1e-12))
        out[f"{k}:{prog['nodes'][k]['op']}:{[st.kind for st in m.steps][-1] if m.steps else 'const'}"] = d
        del g
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
