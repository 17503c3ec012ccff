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


def test_host_pin_refuses_gracefully_without_gpu():
    """dpe_host_pin / dpe_host_unpin (the host fusion's pinned candidate buffers): an argument error
    for a null buffer, and a runtime refusal -- not a crash -- where no device is present (here);
    callers then keep the buffer pageable."""
    import numpy as np
    lib = C.CDLL(LIB)
    lib.dpe_host_pin.argtypes = [C.c_void_p, C.c_size_t]
    lib.dpe_host_unpin.argtypes = [C.c_void_p]
    assert lib.dpe_host_pin(None, 16) == -1          # DPE_ERR_ARG
    a = np.zeros(1 << 16, np.uint8)
    rc = lib.dpe_host_pin(a.ctypes.data, a.nbytes)
    if rc == 0:                      # a GPU is present: pinning works and is undone
        assert lib.dpe_host_unpin(a.ctypes.data) == 0
    else:
        assert rc < 0


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


HOST_HEADER = os.path.join(ROOT, "include", "dpe_host.h")
HOST_LIB = os.path.join(ROOT, "dpe-mvs_amd", "lib", "libdpe_host.so")


def test_host_library_exports_every_declared_symbol():
    src = re.sub(r"/\*.*?\*/", "", open(HOST_HEADER).read(), flags=re.S)
    declared = sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(dpe_\w+)\s*\(", src, flags=re.M)))
    assert "dpe_run_pipeline" in declared
    out = subprocess.run(["nm", "-D", "--defined-only", HOST_LIB], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [f for f in declared if f not in exported]
    assert not missing, missing


def test_pipeline_options_layout_matches_header():
    # the ctypes mirror of DpePipelineOptions must agree with the C struct: probe the C defaults
    from DPE_MVS import pipeline
    o = pipeline.DpePipelineOptions()
    pipeline.lib().dpe_pipeline_default_options(C.byref(o))
    assert (o.verbose, o.fusion, o.depth, o.normal, o.world_size, o.base_seed) == (True, False, True, False, 1, 0x5EED)


def test_pybind_module_exposes_dpe_mvs():
    from DPE_MVS import _dpe
    assert "gpu_index" in _dpe.dpe_mvs.__doc__
