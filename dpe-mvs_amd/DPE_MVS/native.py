"""Python host binding of the HIP library (lib/libdpe_mvs.so) through its C-ABI.

There is no CPU fallback: if the library is missing this module raises at import.  The library
is built in-tree by `make -C dpe-mvs_amd` (or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPE_MVS_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdpe_mvs.so")

EXPORTED = [
    "dpe_params_default", "dpe_create", "dpe_destroy", "dpe_last_error", "dpe_pm_stage",
    "dpe_pm_execute", "dpe_pm_fetch", "dpe_pm_run", "dpe_pm_device_planes", "dpe_pm_export_depth",
    "dpe_pm_last_timings", "dpe_set_timing", "dpe_set_counting", "dpe_pm_last_counts",
    "dpe_fusion_stage", "dpe_fusion_candidates",
    "dpe_pm_stage_resident", "dpe_state_save", "dpe_state_snapshot", "dpe_state_fetch", "dpe_state_export_depth",
    "dpe_state_import_depth", "dpe_state_clear", "dpe_device_buffer", "dpe_device_copy",
    "dpe_resize_linear", "dpe_resize_u8", "dpe_canny", "dpe_roberts_threshold",
]

CLASSES = ["setup", "init", "strong", "ransac", "weak", "filter", "depth_to_weak", "local_refine"]


def load_library(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"HIP library not built: {path} (run `make -C dpe-mvs_amd`)")
    lib = C.CDLL(path)
    lib.dpe_params_default.argtypes = [C.POINTER(_abi.DpePatchMatchParams)]
    lib.dpe_params_default.restype = None
    lib.dpe_create.argtypes = [C.c_int]
    lib.dpe_create.restype = C.c_void_p
    lib.dpe_destroy.argtypes = [C.c_void_p]
    lib.dpe_destroy.restype = None
    lib.dpe_last_error.argtypes = []
    lib.dpe_last_error.restype = C.c_char_p
    for fn in ("dpe_pm_stage", "dpe_pm_run"):
        getattr(lib, fn).argtypes = [C.c_void_p, C.POINTER(_abi.DpePassInput), C.POINTER(_abi.DpePassState)]
        getattr(lib, fn).restype = C.c_int
    lib.dpe_pm_execute.argtypes = [C.c_void_p, C.c_void_p]
    lib.dpe_pm_execute.restype = C.c_int
    lib.dpe_pm_fetch.argtypes = [C.c_void_p, C.POINTER(_abi.DpePassState)]
    lib.dpe_pm_fetch.restype = C.c_int
    lib.dpe_pm_device_planes.argtypes = [C.c_void_p]
    lib.dpe_pm_device_planes.restype = C.c_void_p
    lib.dpe_pm_export_depth.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.dpe_pm_export_depth.restype = C.c_int
    lib.dpe_pm_last_timings.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int]
    lib.dpe_pm_last_timings.restype = C.c_int
    lib.dpe_set_timing.argtypes = [C.c_void_p, C.c_int]
    lib.dpe_set_timing.restype = None
    lib.dpe_set_counting.argtypes = [C.c_void_p, C.c_int]
    lib.dpe_set_counting.restype = None
    lib.dpe_pm_last_counts.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
    lib.dpe_pm_last_counts.restype = C.c_int
    lib.dpe_set_option.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.dpe_set_option.restype = C.c_int
    lib.dpe_pm_last_stat.argtypes = [C.c_void_p, C.c_int]
    lib.dpe_pm_last_stat.restype = C.c_longlong
    lib.dpe_fusion_stage.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.dpe_fusion_stage.restype = C.c_int
    lib.dpe_fusion_candidates.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.dpe_fusion_candidates.restype = C.c_int
    lib.dpe_resize_linear.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
    lib.dpe_resize_u8.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
    lib.dpe_canny.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p]
    lib.dpe_roberts_threshold.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    for fn in ("dpe_resize_linear", "dpe_resize_u8", "dpe_canny", "dpe_roberts_threshold"):
        getattr(lib, fn).restype = C.c_int
    return lib


def fusion_view_array(views):
    """[(depth f32 [H,W], normal f32 [H,W,3], DpeCamera)] -> (DpeFusionView array, arrays to keep alive)."""
    arr = (_abi.DpeFusionView * len(views))()
    keep = []
    for k, (d, n, cam) in enumerate(views):
        d = np.ascontiguousarray(d, np.float32)
        n = np.ascontiguousarray(n, np.float32)
        keep += [d, n]
        arr[k] = _abi.DpeFusionView(d.shape[1], d.shape[0], cam, d.ctypes.data, n.ctypes.data)
    return arr, keep


_LIB = load_library()


class DpeError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc != 0:
        msg = _LIB.dpe_last_error().decode(errors="replace")
        raise DpeError(f"{what} failed ({rc}): {msg}")


class PatchMatchContext:
    """One HIP device context (the reference's per-image `DPE` object minus the file I/O)."""

    def __init__(self, device: int = 0):
        self._ctx = _LIB.dpe_create(int(device))
        if not self._ctx:
            raise DpeError("dpe_create failed: " + _LIB.dpe_last_error().decode(errors="replace"))
        self._bufs = None

    def close(self):
        if self._ctx:
            _LIB.dpe_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # EdgeSegment's data-parallel stages (include/dpe_mvs.h; bit-identical to host/edges.cpp)
    def resize_linear(self, img: np.ndarray, nw: int, nh: int) -> np.ndarray:
        src = np.ascontiguousarray(img, np.float32)
        out = np.empty((nh, nw), np.float32)
        _check(_LIB.dpe_resize_linear(self._ctx, src.ctypes.data, src.shape[1], src.shape[0], out.ctypes.data, nw, nh),
               "dpe_resize_linear")
        return out

    def resize_u8(self, img: np.ndarray, nw: int, nh: int) -> np.ndarray:
        src = np.ascontiguousarray(img, np.uint8)
        out = np.empty((nh, nw), np.uint8)
        _check(_LIB.dpe_resize_u8(self._ctx, src.ctypes.data, src.shape[1], src.shape[0], out.ctypes.data, nw, nh),
               "dpe_resize_u8")
        return out

    def canny(self, img: np.ndarray, low: float, high: float) -> np.ndarray:
        src = np.ascontiguousarray(img, np.uint8)
        out = np.empty_like(src)
        _check(_LIB.dpe_canny(self._ctx, src.ctypes.data, src.shape[1], src.shape[0], float(low), float(high),
                              out.ctypes.data), "dpe_canny")
        return out

    def roberts_threshold(self, img: np.ndarray, thr: int) -> np.ndarray:
        src = np.ascontiguousarray(img, np.uint8)
        out = np.empty_like(src)
        _check(_LIB.dpe_roberts_threshold(self._ctx, src.ctypes.data, src.shape[1], src.shape[0], int(thr), out.ctypes.data),
               "dpe_roberts_threshold")
        return out

    def set_timing(self, on: bool):
        _LIB.dpe_set_timing(self._ctx, 1 if on else 0)

    def stage(self, pass_input: dict, state: dict):
        self._bufs = _abi.PassBuffers(pass_input, state)
        _check(_LIB.dpe_pm_stage(self._ctx, C.byref(self._bufs.inp), C.byref(self._bufs.st)), "dpe_pm_stage")

    def execute(self, stream: int | None = None):
        _check(_LIB.dpe_pm_execute(self._ctx, C.c_void_p(stream or 0)), "dpe_pm_execute")

    def fetch(self) -> dict:
        _check(_LIB.dpe_pm_fetch(self._ctx, C.byref(self._bufs.st)), "dpe_pm_fetch")
        return {k: v.copy() for k, v in self._bufs.outputs().items()}

    def run(self, pass_input: dict, state: dict) -> dict:
        self.stage(pass_input, state)
        self.execute()
        return self.fetch()

    def set_counting(self, on: bool):
        _LIB.dpe_set_counting(self._ctx, 1 if on else 0)

    def set_option(self, option: int, value: int):
        _check(_LIB.dpe_set_option(self._ctx, int(option), int(value)), "dpe_set_option")

    def last_stat(self, stat: int) -> int:
        return int(_LIB.dpe_pm_last_stat(self._ctx, int(stat)))

    def timings(self) -> dict:
        """{'total': ms, <class>: summed kernel ms} of the last execute (timing enabled)."""
        buf = (C.c_float * 9)()
        n = _LIB.dpe_pm_last_timings(self._ctx, buf, 9)
        out = {"total": float(buf[0])}
        for i, name in enumerate(CLASSES):
            if 1 + i < n:
                out[name] = float(buf[1 + i])
        return out

    def counts(self) -> dict:
        """{<class>: {'ncc', 'taps', 'geom', 'launches'}} of the last execute (counting enabled)."""
        buf = (C.c_ulonglong * 32)()
        _LIB.dpe_pm_last_counts(self._ctx, buf, 32)
        return {name: {"ncc": int(buf[4 * i]), "taps": int(buf[4 * i + 1]), "geom": int(buf[4 * i + 2]),
                       "launches": int(buf[4 * i + 3])} for i, name in enumerate(CLASSES)}

    def fusion_candidates(self, views, ref: int, src) -> tuple:
        """RunFusion's projection tests on the GPU (dpe_fusion_stage + dpe_fusion_candidates) for
        views = [(depth, normal, DpeCamera)]: (idx int32 [L*ns], val f32 [L*ns*3])."""
        arr, keep = fusion_view_array(views)
        _check(_LIB.dpe_fusion_stage(self._ctx, arr, len(views)), "dpe_fusion_stage")
        s = np.ascontiguousarray(src, np.int32)
        L = views[ref][0].size
        idx, val = np.empty(L * len(s), np.int32), np.empty(L * len(s) * 3, np.float32)
        _check(_LIB.dpe_fusion_candidates(self._ctx, int(ref), s.ctypes.data, len(s), idx.ctypes.data, val.ctypes.data),
               "dpe_fusion_candidates")
        return idx, val

    def device_planes(self) -> int:
        return int(_LIB.dpe_pm_device_planes(self._ctx) or 0)

    def export_depth(self, dev_ptr: int, stream: int | None = None):
        _check(_LIB.dpe_pm_export_depth(self._ctx, C.c_void_p(dev_ptr), C.c_void_p(stream or 0)), "dpe_pm_export_depth")


def run_pass(pass_input: dict, state: dict, device: int = 0) -> dict:
    ctx = PatchMatchContext(device)
    try:
        return ctx.run(pass_input, state)
    finally:
        ctx.close()


def param_struct(**overrides) -> _abi.DpePatchMatchParams:
    p = _abi.DpePatchMatchParams()
    _LIB.dpe_params_default(C.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


__all__ = ["PatchMatchContext", "run_pass", "param_struct", "DpeError", "LIB_PATH", "EXPORTED", "np"]
