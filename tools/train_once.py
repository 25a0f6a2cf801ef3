"""One training tenant stepping in this process, for rocprofv3 kernel stats
(no hipBLASLt GEMM, no at::native softmax in a step).

python tools/train_once.py --seq 2048 --steps 6
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--small", type=int, default=1)
    a = ap.parse_args()
    import numpy as np

    from nos_amd.models.llama_program import llama_config, llama_model, llama_program
    from nos_amd.podserver.client import PodClient
    from nos_amd.podserver.server import PodServer

    prog, w = llama_program(llama_model(llama_config(bool(a.small)), 0), a.seq)
    path = Path(tempfile.mkdtemp(prefix="nos_tr_", dir="/tmp")) / "s.sock"
    srv = PodServer(path, device="cuda", lanes=2, memory_gb=64).start()
    try:
        c = PodClient(srv.path, connect_timeout_s=60)
        rep = c.register("ft", prog, w, memory_limit_gb=10,
                         train={"loss": "cross_entropy", "optimizer": "adamw", "lr": 1e-4})
        ids = np.random.default_rng(0).integers(0, 32000 if a.small else 512, (1, a.seq + 1)).astype(np.int32)
        c.train_step(ids[:, :-1], ids[:, 1:])
        t0 = time.monotonic()
        losses = [c.train_step(ids[:, :-1], ids[:, 1:])["loss"] for _ in range(a.steps)]
        dt = (time.monotonic() - t0) / a.steps
        print(json.dumps({"seq": a.seq, "footprint_gb": rep["footprint_gb"], "step_s": round(dt, 4),
                          "tokens_per_s": round(a.seq / dt, 1), "losses": [round(x, 4) for x in losses]}), flush=True)
        c.close()
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
