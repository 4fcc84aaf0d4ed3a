"""The host analysis of solve(order="nd") (csrc/nd_order.cpp: the parallel
graph build, the bisection on a pool of workers, the parallel numbering and
symbolic pass) built with -fsanitize=thread and run on the CPU
(tests/cpp/nd_analysis_tsan.cpp): no data race reported, and the same plan
with 8 threads (twice) and with 1."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "basic_sparse_matrix_amd", "csrc")
SRC = os.path.join(ROOT, "tests", "cpp", "nd_analysis_tsan.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "nd_analysis_tsan")


def test_nd_analysis_thread_sanitizer():
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    cmd = [cxx, "-std=c++20", "-O1", "-g", "-fsanitize=thread", "-pthread", "-I", CSRC, SRC,
           os.path.join(CSRC, "nd_order.cpp"), "-o", EXE]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "tsan" in r.stderr.lower():
        pytest.skip("no ThreadSanitizer runtime: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "0 failed" in r.stdout
