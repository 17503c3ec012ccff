"""Python side of the C++ host pipeline (lib/libdpe_host.so, include/dpe_host.h).

The pipeline itself -- RunDPEPipeline / ProcessProblem / InuputInitialization, the dense_folder
I/O, the coarse-to-fine schedule, the epilogue and the .npy outputs -- is C++ (host/pipeline.cpp).
This module binds it with ctypes for what the pybind entry `DPE_MVS.dpe_mvs()` does not expose:

  * the one-process-per-GPU run from Python: `run_dpe_pipeline(..., dist=torch.distributed)` hands
    the C++ pipeline an all-gather callback (RCCL with the "nccl" backend, gloo on CPU);
  * a pass-runner hook (tests drive the C++ pipeline with the CPU oracle's runner);
  * the host helpers (grey decode, INTER_LINEAR resize, RescaleMatToTargetSize, camera reader).

It also holds writers for the dense_folder formats (.dmb, cams) used to build test datasets.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import struct

import numpy as np

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB = os.environ.get("DPE_HOST_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdpe_host.so")
OUT_NAME = "DPE"
SCHEDULE_REFERENCE, SCHEDULE_JACOBI = 0, 1

ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_float))


class DpePipelineOptions(C.Structure):
    _fields_ = [
        ("gpu_index", C.c_int),
        ("verbose", C.c_bool), ("fusion", C.c_bool), ("viz", C.c_bool), ("depth", C.c_bool),
        ("normal", C.c_bool), ("weak", C.c_bool), ("edge", C.c_bool),
        ("schedule", C.c_int),
        ("rank", C.c_int), ("world_size", C.c_int),
        ("allgather", ALLGATHER_FN), ("allgather_user", C.c_void_p),
        ("runner", C.c_void_p), ("runner_user", C.c_void_p),
        ("base_seed", C.c_uint64),
        ("keep_intermediate", C.c_bool),
        ("fusion_runner", C.c_void_p), ("fusion_user", C.c_void_p),
        ("max_iterations", C.c_int), ("photometric_only", C.c_bool),
        ("allgather_device", C.c_void_p), ("allgather_device_user", C.c_void_p),
        ("abort_collectives", C.c_void_p), ("abort_user", C.c_void_p),
    ]


class PipelineError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(HOST_LIB):
            raise RuntimeError(f"host library not built: {HOST_LIB} (run `make -C dpe-mvs_amd`)")
        L = C.CDLL(HOST_LIB)
        L.dpe_pipeline_default_options.argtypes = [C.POINTER(DpePipelineOptions)]
        L.dpe_run_pipeline.argtypes = [C.c_char_p, C.POINTER(DpePipelineOptions)]
        L.dpe_run_pipeline.restype = C.c_int
        L.dpe_pipeline_last_error.restype = C.c_char_p
        L.dpe_host_read_gray.argtypes = [C.c_char_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.dpe_host_read_camera.argtypes = [C.c_char_p, C.POINTER(_abi.DpeCamera)]
        L.dpe_host_resize_linear.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.dpe_host_rescale_nearest.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.dpe_host_read_bgr.argtypes = [C.c_char_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.dpe_host_edge_segment.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.dpe_host_canny.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p]
        L.dpe_host_resize_u8.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.dpe_host_connect.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.dpe_host_hough_lines_p.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, C.c_double,
                                             C.c_double, C.c_void_p, C.c_int]
        _lib = L
    return _lib


# ------------------------------------------------------------------------------ host helpers (C++)
def read_gray(path: str) -> np.ndarray:
    w, h = C.c_int(), C.c_int()
    if lib().dpe_host_read_gray(path.encode(), None, 0, C.byref(w), C.byref(h)) != 0:
        raise PipelineError(f"cannot decode {path}")
    out = np.empty((h.value, w.value), np.uint8)
    lib().dpe_host_read_gray(path.encode(), out.ctypes.data, out.nbytes, C.byref(w), C.byref(h))
    return out


def read_bgr(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_COLOR): uint8 [H, W, 3] BGR."""
    w, h = C.c_int(), C.c_int()
    if lib().dpe_host_read_bgr(path.encode(), None, 0, C.byref(w), C.byref(h)) != 0:
        raise PipelineError(f"cannot decode {path}")
    out = np.empty((h.value, w.value, 3), np.uint8)
    lib().dpe_host_read_bgr(path.encode(), out.ctypes.data, out.nbytes, C.byref(w), C.byref(h))
    return out


def read_camera(path: str) -> _abi.DpeCamera:
    cam = _abi.DpeCamera()
    if lib().dpe_host_read_camera(path.encode(), C.byref(cam)) != 0:
        raise PipelineError(f"cannot read camera {path}")
    return cam


def resize_linear(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    src = np.ascontiguousarray(img, dtype=np.float32)
    dst = np.empty((new_h, new_w), np.float32)
    lib().dpe_host_resize_linear(src.ctypes.data, src.shape[1], src.shape[0], dst.ctypes.data, new_w, new_h)
    return dst


def rescale_to(src: np.ndarray, W: int, H: int) -> np.ndarray:
    s = np.ascontiguousarray(src)
    dst = np.zeros((H, W) + s.shape[2:], s.dtype)
    elem = s.itemsize * int(np.prod(s.shape[2:], dtype=np.int64))
    lib().dpe_host_rescale_nearest(s.ctypes.data, s.shape[1], s.shape[0], dst.ctypes.data, W, H, elem)
    return dst


# ------------------------------------------------------------------------------ EdgeSegment (C++, edges.cpp)
def _u8(img: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(img)
    if a.dtype != np.uint8 or a.ndim != 2:
        raise ValueError("expected a 2-D uint8 image")
    return a


def edge_segment(scale: int, img: np.ndarray, mode: int, use_canny: bool, high_res: bool = True) -> np.ndarray:
    """EdgeSegment (DPE.cpp:129-291): mode 0 -> uint8 0/255 edges, mode 1 -> int32 labels."""
    a = _u8(img)
    ow, oh = C.c_int(), C.c_int()
    args = (scale, a.ctypes.data, a.shape[1], a.shape[0], mode, int(use_canny), int(high_res))
    if lib().dpe_host_edge_segment(*args, None, 0, C.byref(ow), C.byref(oh)) != 0:
        raise PipelineError("EdgeSegment failed")
    out = np.empty((oh.value, ow.value), np.uint8 if mode == 0 else np.int32)
    if lib().dpe_host_edge_segment(*args, out.ctypes.data, out.nbytes, C.byref(ow), C.byref(oh)) != 0:
        raise PipelineError("EdgeSegment failed")
    return out


def canny(img: np.ndarray, low: float, high: float) -> np.ndarray:
    """cv::Canny(img, low, high, 3, L2gradient=true) -> uint8 0/255."""
    a = _u8(img)
    out = np.empty_like(a)
    lib().dpe_host_canny(a.ctypes.data, a.shape[1], a.shape[0], low, high, out.ctypes.data)
    return out


def resize_u8(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv::resize(INTER_LINEAR) of an 8-bit image."""
    a = _u8(img)
    out = np.empty((new_h, new_w), np.uint8)
    lib().dpe_host_resize_u8(a.ctypes.data, a.shape[1], a.shape[0], out.ctypes.data, new_w, new_h)
    return out


def connect(img: np.ndarray):
    """Connect (DPE.cpp:27-127) -> (labels int32, counts per label)."""
    a = _u8(img)
    lab = np.empty(a.shape, np.int32)
    n = lib().dpe_host_connect(a.ctypes.data, a.shape[1], a.shape[0], lab.ctypes.data, None, 0)
    cnt = np.empty(max(n, 1), np.int32)
    lib().dpe_host_connect(a.ctypes.data, a.shape[1], a.shape[0], lab.ctypes.data, cnt.ctypes.data, n)
    return lab, cnt[:n]


def hough_lines_p(img: np.ndarray, rho: float, theta: float, threshold: int, min_len: float, max_gap: float) -> np.ndarray:
    """cv::HoughLinesP -> int32 [n, 4] segments (x0, y0, x1, y1)."""
    a = _u8(img)
    n = lib().dpe_host_hough_lines_p(a.ctypes.data, a.shape[1], a.shape[0], rho, theta, threshold, min_len, max_gap, None, 0)
    out = np.empty((max(n, 0), 4), np.int32)
    if n > 0:
        lib().dpe_host_hough_lines_p(a.ctypes.data, a.shape[1], a.shape[0], rho, theta, threshold, min_len, max_gap,
                                     out.ctypes.data, n)
    return out


# ------------------------------------------------------------------------------ dataset writers
CV_8UC1, CV_8SC1, CV_32SC1, CV_32FC1, CV_32FC3 = 0, 1, 4, 5, 21
_CV = {CV_8UC1: (np.uint8, 1), CV_8SC1: (np.int8, 1), CV_32SC1: (np.int32, 1), CV_32FC1: (np.float32, 1),
       CV_32FC3: (np.float32, 3)}


def read_bin_mat(path: str) -> np.ndarray:
    """ReadBinMat (DPE.cpp:293-318)."""
    with open(path, "rb") as f:
        version, rows, cols, typ = struct.unpack("<4i", f.read(16))
        if version != 1 or typ not in _CV:
            raise PipelineError(f"bad .dmb: {path}")
        dt, ch = _CV[typ]
        a = np.frombuffer(f.read(), dtype=dt)[: rows * cols * ch]
    return a.reshape((rows, cols, ch) if ch > 1 else (rows, cols)).copy()


def write_bin_mat(path: str, mat: np.ndarray) -> None:
    """WriteBinMat (DPE.cpp:320-339)."""
    mat = np.ascontiguousarray(mat)
    ch = mat.shape[2] if mat.ndim == 3 else 1
    typ = {("uint8", 1): CV_8UC1, ("int8", 1): CV_8SC1, ("int32", 1): CV_32SC1, ("uint32", 1): CV_32SC1,
           ("float32", 1): CV_32FC1, ("float32", 3): CV_32FC3}[(mat.dtype.name, ch)]
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", 1, mat.shape[0], mat.shape[1], typ))
        f.write(mat.tobytes())


def write_camera(path: str, K, R, t, dmin: float, dmax: float, depth_num: int = 192) -> None:
    """cams/%08d_cam.txt as ReadCamera parses it (4-number depth line)."""
    g = lambda v: repr(float(v))  # noqa: E731
    with open(path, "w") as f:
        f.write("extrinsic\n")
        for i in range(3):
            f.write(f"{g(R[i][0])} {g(R[i][1])} {g(R[i][2])} {g(t[i])}\n")
        f.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
        for i in range(3):
            f.write(f"{g(K[i][0])} {g(K[i][1])} {g(K[i][2])}\n")
        f.write(f"\n{g(dmin)} {g((dmax - dmin) / depth_num)} {depth_num} {g(dmax)}\n")


def std_round(v) -> int:
    """std::round (half away from zero) of a non-negative value."""
    f = math.floor(float(v))
    return int(f + 1) if float(v) - f >= 0.5 else int(f)


# ------------------------------------------------------------------------------ the pipeline
def _torch_allgather(dist):
    import torch
    world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")

    def cb(_user, send, count, recv):
        try:
            s = torch.from_numpy(np.ctypeslib.as_array(send, shape=(count,)).copy()).to(dev)
            out = torch.empty(world * count, dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(out, s)
            np.ctypeslib.as_array(recv, shape=(world * count,))[:] = out.cpu().numpy()
            return 0
        except Exception:   # noqa: BLE001 -- reported to the C++ side as a failed collective
            return -1
    return ALLGATHER_FN(cb)


ALLGATHER_DEV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class _DeviceArray:
    """A device buffer of the library as a torch tensor view (__cuda_array_interface__, no copy)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3}


def _torch_allgather_device(dist):
    """Device all-gather hook (dpe_allgather_dev_fn) over torch.distributed "nccl" (= RCCL): the
    depth maps go from the library's HBM buffers to the other ranks' without a host copy."""
    import torch
    world = dist.get_world_size()

    def cb(_user, send, count, recv):
        try:
            s = torch.as_tensor(_DeviceArray(send, count), device="cuda")
            r = torch.as_tensor(_DeviceArray(recv, world * count), device="cuda")
            dist.all_gather_into_tensor(r, s)
            torch.cuda.synchronize()
            return 0
        except Exception:   # noqa: BLE001 -- reported to the C++ side as a failed collective
            return -1
    return ALLGATHER_DEV_FN(cb)


def run_dpe_pipeline(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False,
                     viz: bool = False, depth: bool = True, normal: bool = False, weak: bool = False,
                     edge: bool = False, schedule: str = "reference", dist=None, runner=None,
                     base_seed: int = 0x5EED, keep_intermediate: bool = False, fusion_runner=None,
                     max_iterations: int = 0, photometric_only: bool = False, allgather_device=None) -> int:
    """RunDPEPipeline (main.cpp:474) through libdpe_host.  `dist`: an initialised torch.distributed
    (one process per GPU; problems split in contiguous blocks, depth maps all-gathered per pass).
    `runner`: (C function pointer, user pointer) of a dpe_pass_runner_fn; default the HIP library.
    `fusion_runner`: (C function pointer, user pointer) of a dpe_fusion_fn; default the HIP kernel.
    `max_iterations` (0 = the reference's 3) and `photometric_only` (no geometric passes) are the
    schedule knobs of BASELINE configs 1 and 2.  `allgather_device`: a Python callable
    (send_ptr, count, recv_ptr) -> int used as the device all-gather hook instead of the torch "nccl"
    one (tests drive the device exchange path through it on one GPU)."""
    o = DpePipelineOptions()
    lib().dpe_pipeline_default_options(C.byref(o))
    o.gpu_index = gpu_index
    o.verbose, o.fusion, o.viz, o.depth, o.normal, o.weak, o.edge = verbose, fusion, viz, depth, normal, weak, edge
    o.schedule = {"reference": SCHEDULE_REFERENCE, "jacobi": SCHEDULE_JACOBI}[schedule]
    o.base_seed = base_seed
    o.keep_intermediate = keep_intermediate
    o.max_iterations = max_iterations
    o.photometric_only = photometric_only
    keep = []
    if dist is not None and dist.get_world_size() > 1:
        o.rank, o.world_size = dist.get_rank(), dist.get_world_size()
        cb = _torch_allgather(dist)
        keep.append(cb)
        o.allgather = cb
        if allgather_device is not None:
            dcb = ALLGATHER_DEV_FN(lambda _user, send, count, recv: int(allgather_device(send, count, recv)))
            keep.append(dcb)
            o.allgather_device = C.cast(dcb, C.c_void_p)
        elif dist.get_backend() == "nccl" and runner is None:
            dcb = _torch_allgather_device(dist)
            keep.append(dcb)
            o.allgather_device = C.cast(dcb, C.c_void_p)
    if runner is not None:
        o.runner = C.cast(runner[0], C.c_void_p)
        o.runner_user = C.cast(runner[1], C.c_void_p) if runner[1] is not None else None
    if fusion_runner is not None:
        o.fusion_runner = C.cast(fusion_runner[0], C.c_void_p)
        o.fusion_user = C.cast(fusion_runner[1], C.c_void_p) if fusion_runner[1] is not None else None
    rc = lib().dpe_run_pipeline(dense_folder.encode(), C.byref(o))
    if rc != 0:
        raise PipelineError(lib().dpe_pipeline_last_error().decode(errors="replace"))
    return rc


def dpe_mvs(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False, viz: bool = False,
            depth: bool = True, normal: bool = False, weak: bool = False, edge: bool = False) -> int:
    """DPE_MVS.dpe_mvs through the pybind11 module (csrc/bindings.cpp:31-43 equivalent)."""
    from ._dpe import dpe_mvs as _native
    return _native(dense_folder, gpu_index, verbose, fusion, viz, depth, normal, weak, edge)
