"""libnos_amdsmi under ThreadSanitizer and AddressSanitizer/UBSan (host code
only; GPU sanitizers are not available on the pool): 8 threads race readers
against partition switches, process churn and fault injection on the fake
backend (``csrc/amdsmi/stress_fake.cpp``)."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
SRC = [REPO / "csrc/amdsmi/nos_amdsmi.cpp", REPO / "csrc/amdsmi/stress_fake.cpp"]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ required")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_amdsmi_fake_backend_is_sanitizer_clean(tmp_path, san):
    exe = tmp_path / "stress"
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           "-I/opt/rocm/include", *map(str, SRC), "-o", str(exe), "-ldl", "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=240)
    env = {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66", "ASAN_OPTIONS": "halt_on_error=1 detect_leaks=1",
           "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "ops=16000 bad=0" in r.stdout
