"""Instruction mix per basic block of a gfx950 kernel, from the compiler's asm.

  python tools/asm_mix.py csrc/hip/attention_f32x.hip --kernel attn_fwd_f32x6_d64_kernelILb0

Compiles the source device-only (hipcc -S, gfx950), finds the kernel whose
mangled name contains ``--kernel``, and prints, per basic block, the count of
MFMA / VALU / transcendental / LDS / VMEM / SALU / waitcnt / nop instructions
-- the quick check of what a hot loop issues per MFMA before a PMC run.
"""
from __future__ import annotations

import argparse
import collections
import re
import subprocess
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks(asm: str, kernel: str) -> list[tuple[str, dict]]:
    m = re.search(r"^(_Z\S*" + re.escape(kernel) + r"\S*):", asm, re.M)
    if not m:
        raise SystemExit(f"kernel containing {kernel!r} not found")
    body = asm[m.end():asm.index(".Lfunc_end", m.end())]
    out, name, cnt = [], "entry", collections.Counter()
    for line in body.split("\n"):
        s = line.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            out.append((name, dict(cnt)))
            name, cnt = s.rstrip(":"), collections.Counter()
            continue
        if not s or s.startswith((".", ";", "//")):
            continue
        cnt[classify(s.split()[0])] += 1
    out.append((name, dict(cnt)))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--kernel", required=True, help="substring of the mangled kernel name")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", f"-I{REPO / 'csrc' / 'hip'}", a.source, "-o", str(out)], check=True,
                       stderr=subprocess.DEVNULL)
        asm = out.read_text()
    for name, c in blocks(asm, a.kernel):
        if c:
            print(f"{name:14s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
