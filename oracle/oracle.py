"""TEST INFRASTRUCTURE — ctypes binding of the CPU restatement (oracle/dpe_oracle.cpp).

Parity checker only: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product path never imports this module.

Parity status: the reference (CUDA + cuRAND + textures + OpenCV, --use_fast_math) cannot be built
or run in this image and ships no tests or golden vectors, so the restatement
is pinned by per-function known-answer tests (tests/test_oracle_kat.py, tests/test_oracle_functions.py) and the committed golden
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


def _load(path: str = LIB):
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    lib.oracle_pm_run.argtypes = [C.POINTER(_abi.DpePassInput), C.POINTER(_abi.DpePassState), C.c_int]
    lib.oracle_pm_run.restype = C.c_int
    lib.oracle_last_error.restype = C.c_char_p
    lib.oracle_ncc_old.argtypes = [C.POINTER(_abi.DpePassInput), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
    lib.oracle_ncc_old.restype = C.c_float
    lib.oracle_rcp_tap.argtypes = [C.c_void_p, C.c_void_p, C.c_long]
    lib.oracle_rcp_tap.restype = None
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
    P = C.POINTER
    inp = P(_abi.DpePassInput)
    lib.oracle_homography.argtypes = [inp, C.c_int, P(C.c_float), P(C.c_float)]
    lib.oracle_homography.restype = None
    lib.oracle_project.argtypes = [P(C.c_float), C.c_float, C.c_float, P(C.c_float)]
    lib.oracle_project.restype = None
    lib.oracle_ncc_new.argtypes = [inp, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                   P(C.c_float)]
    lib.oracle_ncc_new.restype = C.c_float
    lib.oracle_geom_cost.argtypes = [inp, C.c_int, C.c_int, C.c_int, P(C.c_float)]
    lib.oracle_geom_cost.restype = C.c_float
    lib.oracle_filter_strong.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    lib.oracle_filter_strong.restype = C.c_float
    lib.oracle_d2w_class.argtypes = [P(C.c_float), C.c_int]
    lib.oracle_d2w_class.restype = C.c_int
    lib.oracle_depth_normal.argtypes = [P(_abi.DpeCamera), P(C.c_float), C.c_int, C.c_int, P(C.c_float)]
    lib.oracle_depth_normal.restype = None
    lib.oracle_local_refine_select.argtypes = [P(C.c_float), P(C.c_int), P(C.c_float), C.c_float, C.c_float, P(C.c_float)]
    lib.oracle_local_refine_select.restype = C.c_int
    lib.oracle_topk_views.argtypes = [P(C.c_float), C.c_int, C.c_int, P(C.c_uint32)]
    lib.oracle_topk_views.restype = C.c_float
    lib.oracle_initial_cost.argtypes = [P(C.c_float), C.c_int, P(C.c_uint32)]
    lib.oracle_initial_cost.restype = C.c_float
    lib.oracle_view_select.argtypes = [P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_float), P(C.c_uint8),
                                       P(C.c_uint32), P(C.c_float)]
    lib.oracle_view_select.restype = None
    lib.oracle_ransac_fit.argtypes = [inp, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, P(C.c_float),
                                      P(C.c_int)]
    lib.oracle_ransac_fit.restype = None
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


_literal = {}


def literal_lib(mode: int):
    """The ORACLE_LITERAL build (dpe_oracle.cpp): 1 = ComputeHomography / ComputeCorrespondingPoint /
    tex2D(pt + 0.5f) as written with IEEE division, 2 = the same with a * (1 / b) divisions."""
    if mode not in _literal:
        _literal[mode] = _load(os.path.join(HERE, "build", f"liboracle_dpe_literal{mode}.so"))
    return _literal[mode]


_rcp_ieee = None


def rcp_ieee_lib():
    """The ORACLE_RCP_IEEE build: restatement choice 8 off (the tap reciprocal IEEE 1.0f / z instead
    of the gfx950 v_rcp_f32 table), every other choice as in lib()."""
    global _rcp_ieee
    if _rcp_ieee is None:
        _rcp_ieee = _load(os.path.join(HERE, "build", "liboracle_dpe_rcp_ieee.so"))
    return _rcp_ieee


def host_threads() -> int:
    """Host threads this process may use: OMP_NUM_THREADS when set (the GPU box sets it to its CPU
    share), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def run_pass(pass_input: dict, state: dict, threads: int = 0, library=None) -> dict:
    """One PatchMatch pass on the CPU (same semantics as dpe_pm_run); `library`: a literal_lib()."""
    if threads <= 0:
        threads = host_threads()
    L = library or lib()
    b = _abi.PassBuffers(pass_input, state)
    rc = L.oracle_pm_run(C.byref(b.inp), C.byref(b.st), int(threads))
    if rc != 0:
        raise RuntimeError("oracle_pm_run: " + L.oracle_last_error().decode())
    return {k: v.copy() for k, v in b.outputs().items()}


def ncc_old(pass_input: dict, x: int, y: int, view: int, plane) -> float:
    b = _abi.PassBuffers(pass_input, {"planes": np.zeros((pass_input["images"][0].size, 4), np.float32),
                                      "weak": np.zeros(pass_input["images"][0].shape, np.uint8),
                                      "sel": np.zeros(pass_input["images"][0].shape, np.uint32)})
    pl = (C.c_float * 4)(*[float(v) for v in plane])
    return float(lib().oracle_ncc_old(C.byref(b.inp), x, y, view, pl))


# ---- per-function entry points (tests/test_oracle_functions.py) ---------------------------------
def _kat_buffers(pass_input: dict) -> _abi.PassBuffers:
    h, w = pass_input["images"][0].shape
    return _abi.PassBuffers(pass_input, {"planes": np.zeros((h * w, 4), np.float32), "weak": np.zeros((h, w), np.uint8),
                                         "sel": np.zeros((h, w), np.uint32)})


def _f4(v):
    return (C.c_float * len(v))(*[float(x) for x in v])


def homography(pass_input: dict, view: int, plane) -> np.ndarray:
    """The restatement's homography of source `view` for a reference-frame plane (n, w): 9 floats."""
    b = _kat_buffers(pass_input)
    out = (C.c_float * 9)()
    lib().oracle_homography(C.byref(b.inp), view, _f4(plane), out)
    return np.array(out[:], np.float32)


def project(H, x: float, y: float) -> tuple:
    out = (C.c_float * 2)()
    lib().oracle_project(_f4(H), x, y, out)
    return out[0], out[1]


def ncc_new(pass_input: dict, weak, sel, neighbours, radius, x: int, y: int, view: int, plane) -> float:
    """ComputeBilateralNCCNew with the given weak [H,W] u8, sel [H,W] u32, neighbours [H,W,9,2] i16
    ((-1, -1) = none) and radius [H,W] i32 (or None)."""
    b = _kat_buffers(pass_input)
    wk = np.ascontiguousarray(weak, np.uint8)
    sl = np.ascontiguousarray(sel, np.uint32)
    nb = np.ascontiguousarray(neighbours, np.int16)
    rd = None if radius is None else np.ascontiguousarray(radius, np.int32)
    return float(lib().oracle_ncc_new(C.byref(b.inp), wk.ctypes.data, sl.ctypes.data, nb.ctypes.data,
                                      None if rd is None else rd.ctypes.data, x, y, view, _f4(plane)))


def geom_cost(pass_input: dict, x: int, y: int, view: int, plane) -> float:
    b = _kat_buffers(pass_input)
    return float(lib().oracle_geom_cost(C.byref(b.inp), x, y, view, _f4(plane)))


def filter_strong(planes, weak, costs, x: int, y: int) -> float:
    """CheckerboardFilterStrong at (x, y) over planes [H,W,4], weak [H,W], costs [H,W]: the new depth."""
    pl = np.ascontiguousarray(planes, np.float32)
    wk = np.ascontiguousarray(weak, np.uint8)
    co = np.ascontiguousarray(costs, np.float32)
    H, W = wk.shape
    return float(lib().oracle_filter_strong(W, H, pl.ctypes.data, wk.ctypes.data, co.ctypes.data, x, y))


def d2w_class(curve, weak_peak_radius: int) -> int:
    c = np.ascontiguousarray(curve, np.float32)
    assert c.size == 61
    return int(lib().oracle_d2w_class(c.ctypes.data_as(C.POINTER(C.c_float)), weak_peak_radius))


def depth_normal(cam, plane, x: int, y: int) -> np.ndarray:
    out = (C.c_float * 4)()
    lib().oracle_depth_normal(C.byref(cam), _f4(plane), x, y, out)
    return np.array(out[:], np.float32)


def local_refine_select(tc, ok, depths, cost_now: float, od: float) -> tuple:
    d = C.c_float()
    okv = (C.c_int * 11)(*[int(bool(v)) for v in ok])
    r = lib().oracle_local_refine_select(_f4(tc), okv, _f4(depths), cost_now, od, C.byref(d))
    return bool(r), d.value


def topk_views(costs, top_k: int) -> tuple:
    """Top-k selection of ComputeMultiViewInitialCostandSelectedViews on the given per-view costs."""
    c = np.ascontiguousarray(costs, np.float32)
    sel = C.c_uint32(0)
    cost = lib().oracle_topk_views(c.ctypes.data_as(C.POINTER(C.c_float)), c.size, top_k, C.byref(sel))
    return float(cost), sel.value


def initial_cost(costs, sel: int) -> tuple:
    """ComputeMultiViewInitialCost on the given per-view costs and view mask: (cost, new mask)."""
    c = np.ascontiguousarray(costs, np.float32)
    s = C.c_uint32(sel)
    cost = lib().oracle_initial_cost(c.ctypes.data_as(C.POINTER(C.c_float)), c.size, C.byref(s))
    return float(cost), s.value


def view_select(cost_array, priors, iter_: int, draws) -> tuple:
    """The joint view selection with cost_array [8][nv], priors [nv] and 15 uniform draws:
    (view weights [nv], selected mask, weight norm)."""
    nv = np.asarray(priors).size
    ca = np.zeros((8, 32), np.float32)
    ca[:, :nv] = cost_array
    pr = np.zeros(32, np.float32)
    pr[:nv] = priors
    dr = np.ascontiguousarray(draws, np.float32)
    vw = np.zeros(32, np.uint8)
    tsv, wn = C.c_uint32(0), C.c_float(0)
    lib().oracle_view_select(ca.ctypes.data_as(C.POINTER(C.c_float)), pr.ctypes.data_as(C.POINTER(C.c_float)), nv, iter_,
                             dr.ctypes.data_as(C.POINTER(C.c_float)), vw.ctypes.data_as(C.POINTER(C.c_uint8)),
                             C.byref(tsv), C.byref(wn))
    return vw[:nv].copy(), tsv.value, wn.value


def ransac_fit(pass_input: dict, planes, weak, neighbours, x: int, y: int, iter_: int = 0) -> tuple:
    """RANSACToGetFitPlane at (x, y): (fit plane [4], radius)."""
    b = _kat_buffers(pass_input)
    pl = np.ascontiguousarray(planes, np.float32)
    wk = np.ascontiguousarray(weak, np.uint8)
    nb = np.ascontiguousarray(neighbours, np.int16)
    out = (C.c_float * 4)()
    rad = C.c_int(0)
    lib().oracle_ransac_fit(C.byref(b.inp), pl.ctypes.data, wk.ctypes.data, nb.ctypes.data, x, y, iter_, out, C.byref(rad))
    return np.array(out[:], np.float32), rad.value


def philox(ctr, key) -> list:
    out = (C.c_uint32 * 4)()
    lib().oracle_philox(*[int(c) & 0xFFFFFFFF for c in ctr], *[int(k) & 0xFFFFFFFF for k in key], out)
    return list(out)


def sample(img: np.ndarray, sx: float, sy: float) -> float:
    im = np.ascontiguousarray(img, np.float32)
    return float(lib().oracle_sample(im.ctypes.data_as(C.POINTER(C.c_float)), im.shape[1], im.shape[0], sx, sy))


# ------------------------------------------------------------------------------ RunFusion
class OracleFusionView(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("cam", _abi.DpeCamera),
                ("depth", C.c_void_p), ("normal", C.c_void_p), ("weak", C.c_void_p), ("bgr", C.c_void_p),
                ("block", C.c_void_p), ("image_id", C.c_int), ("ns", C.c_int), ("src_ids", C.c_void_p)]


def fusion_candidates(views, ref: int, src) -> tuple:
    """oracle_fusion_candidates for views = [(depth, normal, DpeCamera)]: (idx int32 [L*ns], val f32 [L*ns*3])."""
    from DPE_MVS.native import fusion_view_array
    arr, keep = fusion_view_array(views)
    s = np.ascontiguousarray(src, np.int32)
    L = views[ref][0].size
    idx, val = np.empty(L * len(s), np.int32), np.empty(L * len(s) * 3, np.float32)
    f = lib().oracle_fusion_candidates
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    f.restype = C.c_int
    if f(None, arr, len(views), int(ref), s.ctypes.data, len(s), idx.ctypes.data, val.ctypes.data) != 0:
        raise RuntimeError("oracle_fusion_candidates failed")
    return idx, val


def fusion_runner():
    """(function pointer, user) of oracle_fusion_candidates: a dpe_fusion_fn for the host pipeline."""
    return (C.cast(lib().oracle_fusion_candidates, C.c_void_p), None)


def run_fusion(views: list) -> np.ndarray:
    """RunFusion's serial loop (DPE.cpp:1286-1367) over views = [dict(image_id, src_ids, cam, depth [H,W],
    normal [H,W,3], weak [H,W] u8, bgr [H,W,3] u8, block or None)] in problem order -> float32 [n, 6]
    points (x, y, z, b, g, r)."""
    keep, arr = [], (OracleFusionView * len(views))()
    for k, v in enumerate(views):
        d = np.ascontiguousarray(v["depth"], np.float32)
        n = np.ascontiguousarray(v["normal"], np.float32)
        w = np.ascontiguousarray(v["weak"], np.uint8)
        b = np.ascontiguousarray(v["bgr"], np.uint8)
        s = np.ascontiguousarray(v["src_ids"], np.int32)
        bl = None if v.get("block") is None else np.ascontiguousarray(v["block"], np.uint8)
        keep += [d, n, w, b, s, bl]
        arr[k] = OracleFusionView(d.shape[1], d.shape[0], v["cam"], d.ctypes.data, n.ctypes.data, w.ctypes.data,
                                  b.ctypes.data, bl.ctypes.data if bl is not None else None, int(v["image_id"]),
                                  len(s), s.ctypes.data)
    L = lib()
    L.oracle_run_fusion.argtypes = [C.POINTER(OracleFusionView), C.c_int, C.c_void_p, C.c_int]
    L.oracle_run_fusion.restype = C.c_int
    cnt = L.oracle_run_fusion(arr, len(views), None, 0)
    out = np.zeros((max(cnt, 1), 6), np.float32)
    L.oracle_run_fusion(arr, len(views), out.ctypes.data, cnt)
    return out[:cnt]
