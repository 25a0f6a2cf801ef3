"""Build an experimental variant of the gfx950 kernels for A/B measurements.

python tools/build_variant.py NAME PATCH.py   -> build/variants/NAME/libnos_hip.so
PATCH.py is run with the variant's source directory as argv[1] and edits the
copied sources in place; load the variant with NOS_AMD_HIP_LIB=<path>.
Extra arguments FILE.hip=FLAG add per-source compiler flags to the variant
(on top of nos_amd/_native/build.py:HIP_EXTRA_FLAGS).
"""
from __future__ import annotations

import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from nos_amd._native import build as nb  # noqa: E402


def main() -> int:
    name, patch = sys.argv[1], sys.argv[2]
    for spec in sys.argv[3:]:
        f, flag = spec.split("=", 1)
        nb.HIP_EXTRA_FLAGS = {**nb.HIP_EXTRA_FLAGS, f: [*nb.HIP_EXTRA_FLAGS.get(f, []), flag]}
    root = REPO / "build" / "variants" / name
    src = root / "src"
    if root.exists():
        shutil.rmtree(root)
    shutil.copytree(REPO / "csrc" / "hip", src)
    subprocess.run([sys.executable, patch, str(src)], check=True)
    out = nb.build_hip(force=True, src_dir=src, out=root / "libnos_hip.so", build_dir=root / "obj")
    print(out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
