"""Boundary tests: the C-ABI library loads, exports every function include/dpe_mvs.h declares,
and the ctypes mirror matches the reference struct layouts (main.h:50-59, :78-106)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from DPE_MVS import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dpe_mvs.h")
LIB = os.path.join(ROOT, "dpe-mvs_amd", "lib", "libdpe_mvs.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(dpe_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_api():
    fns = declared_functions()
    for must in ("dpe_create", "dpe_destroy", "dpe_pm_stage", "dpe_pm_execute", "dpe_pm_fetch", "dpe_pm_run", "dpe_last_error"):
        assert must in fns


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build with `make -C dpe-mvs_amd`"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing


def test_library_loads_without_gpu():
    lib = C.CDLL(LIB)
    p = _abi.DpePatchMatchParams()
    lib.dpe_params_default(C.byref(p))
    ref = _abi.default_params()
    for name, _ in _abi.DpePatchMatchParams._fields_:
        assert getattr(p, name) == pytest.approx(getattr(ref, name)), name


def test_struct_layouts():
    assert C.sizeof(_abi.DpeCamera) == 112
    offs = {n: getattr(_abi.DpePatchMatchParams, n).offset for n, _ in _abi.DpePatchMatchParams._fields_}
    # C layout of main.h:78-106 (bool = 1 byte, natural alignment)
    assert offs["geom_consistency"] == 28 and offs["strong_radius"] == 32
    assert offs["use_APD"] == 48 and offs["high_res_img"] == 53 and offs["max_scale_size"] == 56
    assert offs["state"] == 80 and C.sizeof(_abi.DpePatchMatchParams) == 84


def test_enum_values():
    assert (_abi.WEAK, _abi.STRONG, _abi.UNKNOWN) == (0, 1, 2)
    assert (_abi.FIRST_INIT, _abi.REFINE_INIT, _abi.REFINE_ITER) == (0, 1, 2)
