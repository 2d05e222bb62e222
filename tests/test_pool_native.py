"""CPU: the feature pipe's host parse pool (rf_io.cpp Pool) under ThreadSanitizer and AddressSanitizer.

tests/native/pool_stress.cpp includes rf_io.cpp and drives thousands of back-to-back Pool::run() calls with a
count that changes every call, each writing a vector on the caller's stack (FeaturePipe's parse pattern,
rf_io.cpp's pool_.run sites). Round 5's pool failed this: TSan reported the race on the shared count, and the
plain build hung (an index run twice drives the pending count past zero). GPU-free; host sanitizers only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "pool_stress.cpp")


@pytest.mark.parametrize("sanitizer,iters", [("thread", 4000), ("address", 20000)])
def test_pool_stress_sanitized(tmp_path, sanitizer, iters):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / f"pool_{sanitizer}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={sanitizer}", "-pthread", "-I", os.path.join(ROOT, "include"),
           SRC, "-o", exe, "-lz", "-ldl"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    if b.returncode != 0 and "cannot find" in b.stderr and "san" in b.stderr:
        pytest.skip(f"lib{sanitizer[0]}san not installed")
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, "8", str(iters)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "pool ok" in r.stdout
