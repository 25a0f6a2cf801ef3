"""The bf16 GEMM's tile choice (csrc/hip/gemm_tiles.h), compiled for the host
with g++ and checked on the shapes it was measured on
(profiles/r02_gemm_bf16_tiles.json): the YOLOS-small projections at batch 1
(3401 rows) and 8 (27208 rows), and 4096^3."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
HARNESS = r'''
#include <cstdio>
#include "gemm_tiles.h"
int main() {
  const char* nm[] = {"base", "narrow", "wide", "big"};
  int M, N, pol, cus;
  while (std::scanf("%d %d %d %d", &M, &N, &pol, &cus) == 4) std::printf("%s\n", nm[nos_gemm::pick_tile(M, N, pol, cus)]);
}
'''
THROUGHPUT, LATENCY = 0, 1
B1, B8 = 3401, 8 * 3401


@pytest.fixture(scope="module")
def pick(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("tiles")
    (d / "h.cpp").write_text(HARNESS)
    subprocess.run([cxx, "-std=c++17", "-O1", "-I", str(REPO / "csrc" / "hip"), str(d / "h.cpp"), "-o", str(d / "h")],
                   check=True)

    def run(cases):
        inp = "".join(f"{m} {n} {p} {c}\n" for m, n, p, c in cases)
        out = subprocess.run([str(d / "h")], input=inp, capture_output=True, text=True, check=True).stdout
        return out.split()
    return run


def test_batch8_projections_use_the_8_wave_tiles(pick):
    # qkv (N 1152), proj/fc2 (N 384): 256x192, one round of 214 tiles for N 384; fc1 (N 1536): 256x256
    got = pick([(B8, 1152, THROUGHPUT, 256), (B8, 384, THROUGHPUT, 256), (B8, 1536, THROUGHPUT, 256),
                (B8, 384, LATENCY, 256)])
    assert got == ["wide", "wide", "big", "wide"]


def test_batch1_keeps_small_tiles(pick):
    # 3401 rows: too few 256-row tiles to occupy half the CUs; latency policy narrows N = 384 / 1536
    got = pick([(B1, 1152, THROUGHPUT, 256), (B1, 384, THROUGHPUT, 256), (B1, 384, LATENCY, 256),
                (B1, 1536, LATENCY, 256), (B1, 1152, LATENCY, 256)])
    assert got == ["base", "base", "narrow", "narrow", "base"]


def test_square_and_forced_policies(pick):
    got = pick([(4096, 4096, THROUGHPUT, 256), (4096, 4096, LATENCY, 256), (64, 64, 2, 256), (64, 64, 3, 256),
                (64, 64, 4, 256), (1, 8, THROUGHPUT, 256)])
    assert got == ["big", "big", "narrow", "big", "wide", "base"]


def test_fewer_cus_move_the_threshold(pick):
    # a 32-CU slice is filled by far fewer tiles: the 256-row tiles qualify at batch 1 on it
    assert pick([(B1, 1152, THROUGHPUT, 32)]) == ["wide"]
