"""CPU checks of the C-ABI boundary: libbsm_hip.so loads without a GPU and
exports exactly the entry points include/bsm.h declares; the ctypes binding
declares every one of them; no-device behaviour fails loudly."""

import ctypes
import os
import re

import numpy as np
import pytest

from basic_sparse_matrix_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "bsm.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bsm_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/bsm.h but not exported"


def test_binding_covers_header():
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert bound == set(header_functions())


def test_api_version_and_errors():
    lib = _lib.load()
    assert lib.bsm_api_version() == 1
    # invalid argument path needs no device
    rc = lib.bsm_csr_shape(None, None, None, None, None)
    assert rc == _lib.BSM_ERR_INVALID
    assert "null" in _lib.last_error()


def test_no_cpu_fallback_without_device():
    """On a machine without a GPU every compute call must raise, not fall back."""
    lib = _lib.load()
    n = ctypes.c_int(0)
    lib.bsm_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    from basic_sparse_matrix_amd import Csr, Dense

    a = Csr.from_data([[1.0, 2.0], [0.0, 3.0]])
    with pytest.raises(_lib.DeviceUnavailable):
        a.mul_dense(Dense.from_data([[1.0, 1.0]]))


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "bsm.h"\nint main(void){ return bsm_api_version() == 1 ? 0 : 1; }\n')
    inc = os.path.join(ROOT, "include")
    libdir = os.path.join(ROOT, "basic_sparse_matrix_amd", "lib")
    for cc, name in (("gcc", "t.c"), ("g++", "t.cpp")):
        f = tmp_path / name
        f.write_text(src.read_text())
        exe = tmp_path / (name + ".out")
        r = os.system(f"{cc} -I{inc} {f} -L{libdir} -lbsm_hip -Wl,-rpath,{libdir} -o {exe} 2>/dev/null")
        assert r == 0, f"{cc} failed to compile against bsm.h"
        assert os.system(str(exe)) == 0
