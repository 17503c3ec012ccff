"""TEST INFRASTRUCTURE — ctypes binding of the CPU restatement (oracle/dpe_oracle.cpp).

Parity checker only: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product path never imports this module.

Parity status: the reference (CUDA + cuRAND + textures + OpenCV, --use_fast_math) cannot be built
or run in this image and ships no tests or golden vectors, so the restatement
is pinned by per-function known-answer tests (tests/test_oracle_kat.py) and the committed golden
fixtures it produced (tests/golden/) rather than by reference outputs: PARITY VS THE CUDA BINARY IS
UNPINNED; parity of the HIP path is bit-exact against this restatement.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle_dpe.so")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "dpe-mvs_amd"))
from DPE_MVS import _abi  # noqa: E402  (the ABI structs are the boundary contract)


def build():
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def _load():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.oracle_pm_run.argtypes = [C.POINTER(_abi.DpePassInput), C.POINTER(_abi.DpePassState), C.c_int]
    lib.oracle_pm_run.restype = C.c_int
    lib.oracle_last_error.restype = C.c_char_p
    lib.oracle_ncc_old.argtypes = [C.POINTER(_abi.DpePassInput), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.oracle_ncc_old.restype = C.c_float
    lib.oracle_expf.argtypes = [C.c_float]
    lib.oracle_expf.restype = C.c_float
    lib.oracle_sinf.argtypes = [C.c_float]
    lib.oracle_sinf.restype = C.c_float
    lib.oracle_cosf.argtypes = [C.c_float]
    lib.oracle_cosf.restype = C.c_float
    lib.oracle_exp_d.argtypes = [C.c_double]
    lib.oracle_exp_d.restype = C.c_double
    lib.oracle_philox.argtypes = [C.c_uint32] * 6 + [C.POINTER(C.c_uint32)]
    lib.oracle_philox.restype = None
    lib.oracle_sample.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_float, C.c_float]
    lib.oracle_sample.restype = C.c_float
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def run_pass(pass_input: dict, state: dict, threads: int = 0) -> dict:
    """One PatchMatch pass on the CPU (same semantics as dpe_pm_run)."""
    if threads <= 0:
        threads = os.cpu_count() or 1
    b = _abi.PassBuffers(pass_input, state)
    rc = lib().oracle_pm_run(C.byref(b.inp), C.byref(b.st), int(threads))
    if rc != 0:
        raise RuntimeError("oracle_pm_run: " + lib().oracle_last_error().decode())
    return {k: v.copy() for k, v in b.outputs().items()}


def ncc_old(pass_input: dict, x: int, y: int, view: int, plane) -> float:
    b = _abi.PassBuffers(pass_input, {"planes": np.zeros((pass_input["images"][0].size, 4), np.float32),
                                      "weak": np.zeros(pass_input["images"][0].shape, np.uint8),
                                      "sel": np.zeros(pass_input["images"][0].shape, np.uint32)})
    pl = (C.c_float * 4)(*[float(v) for v in plane])
    return float(lib().oracle_ncc_old(C.byref(b.inp), x, y, view, pl))


def philox(ctr, key) -> list:
    out = (C.c_uint32 * 4)()
    lib().oracle_philox(*[int(c) & 0xFFFFFFFF for c in ctr], *[int(k) & 0xFFFFFFFF for k in key], out)
    return list(out)


def sample(img: np.ndarray, sx: float, sy: float) -> float:
    im = np.ascontiguousarray(img, np.float32)
    return float(lib().oracle_sample(im.ctypes.data_as(C.POINTER(C.c_float)), im.shape[1], im.shape[0], sx, sy))
