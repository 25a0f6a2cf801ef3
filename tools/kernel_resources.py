"""Per-kernel register / LDS / occupancy report of the gfx950 kernels, from the
compiler's own resource-usage remarks (no GPU needed).

python tools/kernel_resources.py [csrc/hip/gemm_f32.hip ...] [--json out.json]

One row per kernel instantiation: VGPRs, AGPRs, SGPRs, VGPR/SGPR spills,
scratch bytes per lane, LDS bytes and the compiler's waves-per-SIMD occupancy.
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "SGPRs": "sgpr", "VGPRs Spill": "vgpr_spill", "SGPRs Spill": "sgpr_spill",
          "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occupancy", "LDS Size [bytes/block]": "lds"}


def demangle(names: list[str]) -> list[str]:
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.strip().splitlines()
    except Exception:
        return names


def analyse(src: Path, arch: str = "gfx950") -> list[dict]:
    # the per-source options of the real build (no-NaN / no-SLP attention and
    # GEMM sources), so the report describes the kernels that actually ship
    sys.path.insert(0, str(REPO))
    from nos_amd._native.build import HIP_EXTRA_FLAGS

    r = subprocess.run(["/opt/rocm/bin/hipcc", f"--offload-arch={arch}", "-O3", "-std=c++17", "--cuda-device-only",
                        *HIP_EXTRA_FLAGS.get(src.name, []), "-I", str(REPO / "csrc" / "hip"), "-c", str(src), "-o",
                        "/dev/null", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    rows: list[dict] = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (?:\S+ )?Function Name: (\S+)", line)
        if m:
            rows.append({"kernel": m.group(1), "file": src.name})
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*?): (-?\d+)", line)
        if m and rows and m.group(1).strip() in FIELDS:
            rows[-1][FIELDS[m.group(1).strip()]] = int(m.group(2))
    for row, name in zip(rows, demangle([x["kernel"] for x in rows])):
        row["kernel"] = name.replace("(anonymous namespace)::", "")
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    srcs = [Path(s) for s in a.sources] or sorted((REPO / "csrc" / "hip").glob("*.hip"))
    rows = [r for s in srcs for r in analyse(s)]
    for r in rows:
        print(f"{r['file']:<18} vgpr {r.get('vgpr', '?'):>3} agpr {r.get('agpr', '?'):>3} "
              f"spill v{r.get('vgpr_spill', '?')}/s{r.get('sgpr_spill', '?')} scratch {r.get('scratch', '?'):>3} "
              f"lds {r.get('lds', '?'):>6} occ {r.get('occupancy', '?')}  {r['kernel'][:110]}")
    if a.json:
        Path(a.json).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    sys.exit(main())
