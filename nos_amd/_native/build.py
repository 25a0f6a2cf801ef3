"""In-tree build of the native libraries of nos_amd.

* ``libnos_hip.so``     -- gfx950 HIP kernels (attention, GEMM, LayerNorm,
  probes) + CU-mask stream helpers.  Compiled with ``hipcc
  --offload-arch=gfx950`` and linked against the HIP runtime that PyTorch
  itself loads (``torch/lib/libamdhip64.so``) so that streams, pointers and
  graphs are shared with torch (two HIP runtimes in one process would not
  share a context).
* ``libnos_amdsmi.so``  -- amd-smi partition / telemetry access with an
  in-memory fake backend (C++17, ``dlopen``s ``libamd_smi`` lazily).

The outputs are written next to this file so they travel with the repo
snapshot to GPU boxes.  Objects are cached by mtime under ``build/native``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("NOS_AMD_ARCH", "gfx950")

HIP_SOURCES = ["attention.hip", "attention_f32.hip", "attention_f32x.hip", "gemm_f32.hip", "gemm_f32x.hip", "gemm_f32h.hip", "gemm.hip", "layernorm.hip", "probes.hip", "runtime.hip", "tenant_ops.hip", "attention_h3g.hip", "decode.hip"]
# per-source compiler flags, {file: [flags]} (CMakeLists.txt sets the same:
# tests/test_build_config.py); tools/build_variant.py adds to it for A/B builds.
# The bf16x6 kernels split fp32 into bf16 pieces and run the softmax with
# scalar f32 ops: without SLP re-packing them into v_pk_*_f32 next to the
# MFMAs, x6 attention is 3-5 % faster and the 28-pod fleet +2 %
# (profiles/r03_x6_scalar_split_ab.json)
# attention_f32x: -fno-honor-nans drops the canonicalising v_max_f32 the score
# row maximum got around every fmaxf (21 -> 17 VALU per QK tile); scores are
# never NaN for finite inputs
HIP_EXTRA_FLAGS: dict[str, list[str]] = {"attention_f32x.hip": ["-fno-slp-vectorize", "-fno-honor-nans"],
                                         "gemm_f32x.hip": ["-fno-slp-vectorize"],
                                         "attention.hip": ["-fno-slp-vectorize", "-fno-honor-nans"]}
HIP_LIB = HERE / "libnos_hip.so"
SMI_LIB = HERE / "libnos_amdsmi.so"


def _torch_lib_dir() -> Path | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = Path(spec.origin).parent / "lib"
            if (d / "libamdhip64.so").exists():
                return d
    except Exception:
        pass
    return None


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    if p.exists():
        return str(p)
    found = shutil.which("hipcc")
    if not found:
        raise RuntimeError("hipcc not found (ROCm required to build libnos_hip.so)")
    return found


def build_hip(force: bool = False, jobs: int = 8, verbose: bool = False, src_dir: Path | None = None,
              out: Path | None = None, build_dir: Path | None = None) -> Path:
    """``src_dir``/``out``/``build_dir`` build an experimental variant of the
    kernels (tools/build_variant.py) without touching the in-tree library."""
    src_dir = Path(src_dir) if src_dir else CSRC / "hip"
    out_lib = Path(out) if out else HIP_LIB
    bdir = Path(build_dir) if build_dir else BUILD
    bdir.mkdir(parents=True, exist_ok=True)
    hdr = sorted(src_dir.glob("*.h"))  # every kernel source may include any of them
    objs: list[Path] = []
    todo: list[tuple[Path, Path]] = []
    for s in HIP_SOURCES:
        src = src_dir / s
        obj = bdir / (s + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *hdr]):
            todo.append((src, obj))

    def compile_one(pair: tuple[Path, Path]) -> None:
        src, obj = pair
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
              "-Wno-unused-result", "-Wno-inline-asm", *HIP_EXTRA_FLAGS.get(src.name, []), "-I", str(src_dir), "-c",
              str(src), "-o", str(obj)], verbose)

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(compile_one, todo))
    if force or todo or _stale(out_lib, objs):
        tl = _torch_lib_dir()
        link = ["g++", "-shared", "-fPIC", "-o", str(out_lib), *map(str, objs)]
        if tl is not None:
            # bind to torch's own HIP runtime (same process-wide context)
            link += [f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"]
        else:
            link += [f"-L{ROCM / 'lib'}", "-lamdhip64", f"-Wl,-rpath,{ROCM / 'lib'}"]
        _run(link, verbose)
    return out_lib


def build_amdsmi(force: bool = False, verbose: bool = False, sanitize: str | None = None) -> Path:
    src = CSRC / "amdsmi" / "nos_amdsmi.cpp"
    out = SMI_LIB if sanitize is None else BUILD / f"libnos_amdsmi_{sanitize}.so"
    BUILD.mkdir(parents=True, exist_ok=True)
    if force or sanitize or _stale(out, [src]):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{ROCM / 'include'}",
               str(src), "-o", str(out), "-ldl", "-lpthread"]
        if sanitize:
            cmd[1:1] = [f"-fsanitize={sanitize}", "-g", "-fno-omit-frame-pointer"]
        _run(cmd, verbose)
    return out


def build_all(force: bool = False, jobs: int = 8, verbose: bool = False) -> dict[str, Path]:
    return {"amdsmi": build_amdsmi(force, verbose), "hip": build_hip(force, jobs, verbose)}


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="build nos_amd native libraries (gfx950)")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--only", choices=["hip", "amdsmi"], default=None)
    a = ap.parse_args(argv)
    if a.only == "hip":
        print(build_hip(a.force, a.jobs, a.verbose))
    elif a.only == "amdsmi":
        print(build_amdsmi(a.force, a.verbose))
    else:
        for k, v in build_all(a.force, a.jobs, a.verbose).items():
            print(k, v)
    return 0


if __name__ == "__main__":
    sys.exit(main())
