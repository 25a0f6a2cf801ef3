"""The two build paths (python -m nos_amd._native.build and CMake) compile the
same kernel sources, and every source under csrc/hip is built."""
from __future__ import annotations

import re
from pathlib import Path

from nos_amd._native import build

REPO = Path(__file__).resolve().parent.parent


def test_cmake_and_python_build_list_the_same_hip_sources():
    cmake = (REPO / "CMakeLists.txt").read_text()
    block = re.search(r"add_library\(nos_hip SHARED(.*?)\)", cmake, re.S).group(1)
    in_cmake = sorted(Path(p).name for p in block.split())
    assert in_cmake == sorted(build.HIP_SOURCES)
    on_disk = sorted(p.name for p in (REPO / "csrc" / "hip").glob("*.hip"))
    assert on_disk == sorted(build.HIP_SOURCES)


def test_cmake_sets_the_same_per_source_flags():
    cmake = (REPO / "CMakeLists.txt").read_text()
    props = dict(re.findall(r'set_source_files_properties\(csrc/hip/(\S+) PROPERTIES COMPILE_OPTIONS "([^"]*)"\)', cmake))
    assert {k: v.split(";") for k, v in props.items()} == build.HIP_EXTRA_FLAGS
