"""The C++ host mirror (include/bsm.hpp) -- the reference is compiled Rust, so
its API is mirrored in C++ above the C-ABI -- driven by tests/cpp/test_mirror.cpp:
the reference's own unit tests restated in C++ plus seeded parity against the
C oracle. CPU: build, host-logic tests, and "no CPU fallback" (every hot-path
call raises bsm::DeviceError without a GPU). GPU: the whole program."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "basic_sparse_matrix_amd", "lib")
ORC = os.path.join(ROOT, "oracle", "build")
SRC = os.path.join(ROOT, "tests", "cpp", "test_mirror.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_mirror")


def _build():
    if not (os.path.exists(os.path.join(LIB, "libbsm_hip.so")) and os.path.exists(os.path.join(ORC, "libbsm_oracle.so"))):
        pytest.skip("libbsm_hip.so / libbsm_oracle.so not built (run __graft_entry__.build())")
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no C++ compiler")
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    cmd = [cxx, "-std=c++20", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
           "-L", LIB, "-lbsm_hip", "-L", ORC, "-lbsm_oracle", f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,{ORC}",
           "-Wl,-rpath-link,/opt/rocm/lib", "-o", EXE]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return EXE


def _run(*args, timeout=300):
    return subprocess.run([_build(), *args], capture_output=True, text=True, timeout=timeout)


def test_cpp_mirror_host_logic():
    r = _run("--host")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def test_cpp_mirror_no_cpu_fallback():
    """Without a GPU every hot-path call of the mirror throws DeviceError."""
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    r = _run("--expect-no-device")
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_on_gpu():
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout
