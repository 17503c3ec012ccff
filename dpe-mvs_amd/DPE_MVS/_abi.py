"""ctypes mirror of include/dpe_mvs.h (the C-ABI boundary).

`DpeCamera` / `DpePatchMatchParams` are layout-compatible with the reference's `Camera`
(csrc/DPE-MVS/main.h:50-59) and `PatchMatchParams` (main.h:78-106).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

MAX_IMAGES = 32
NEIGHBOUR_NUM = 9

FIRST_INIT, REFINE_INIT, REFINE_ITER = 0, 1, 2          # main.h:66-70 RunState
WEAK, STRONG, UNKNOWN = 0, 1, 2                          # main.h:72-76 PixelState

DPE_OK = 0
DPE_OPT_GN_SLOTS = 1          # dpe_set_option: GenNeighbours support-point slots (include/dpe_mvs.h)
DPE_STAT_GN_DEFERRED = 1      # dpe_pm_last_stat: WEAK pixels handed to the scratch GenNeighbours
DPE_STAT_TEX_CLASS = 2        # dpe_pm_last_stat: 2 u8 / f16 texels, 1 f16 (quarter-integer grey levels), 0 f32


class DpeCamera(C.Structure):
    _fields_ = [
        ("K", C.c_float * 9),
        ("R", C.c_float * 9),
        ("t", C.c_float * 3),
        ("c", C.c_float * 3),
        ("height", C.c_int),
        ("width", C.c_int),
        ("depth_min", C.c_float),
        ("depth_max", C.c_float),
    ]


class DpeFusionView(C.Structure):   # include/dpe_mvs.h (RunFusion's projection tests)
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("cam", DpeCamera),
                ("depth", C.c_void_p), ("normal", C.c_void_p)]


class DpePatchMatchParams(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int),
        ("num_images", C.c_int),
        ("sigma_spatial", C.c_float),
        ("sigma_color", C.c_float),
        ("top_k", C.c_int),
        ("depth_min", C.c_float),
        ("depth_max", C.c_float),
        ("geom_consistency", C.c_bool),
        ("strong_radius", C.c_int),
        ("strong_increment", C.c_int),
        ("weak_radius", C.c_int),
        ("weak_increment", C.c_int),
        ("use_APD", C.c_bool),
        ("use_edge", C.c_bool),
        ("use_limit", C.c_bool),
        ("use_label", C.c_bool),
        ("use_radius", C.c_bool),
        ("high_res_img", C.c_bool),
        ("max_scale_size", C.c_int),
        ("scale_size", C.c_int),
        ("weak_peak_radius", C.c_int),
        ("rotate_time", C.c_int),
        ("ransac_threshold", C.c_float),
        ("geom_factor", C.c_float),
        ("state", C.c_int),
    ]


class DpePassInput(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("num_images", C.c_int),
        ("images", C.POINTER(C.POINTER(C.c_float))),
        ("cams", C.POINTER(DpeCamera)),
        ("depths", C.POINTER(C.POINTER(C.c_float))),
        ("edge", C.POINTER(C.c_uint8)),
        ("low_width", C.c_int),
        ("low_height", C.c_int),
        ("edge_low_res", C.POINTER(C.c_uint8)),
        ("label", C.POINTER(C.c_int32)),
        ("params", DpePatchMatchParams),
        ("seed", C.c_uint64),
        ("pass_salt", C.c_uint32),
        ("image_ids", C.POINTER(C.c_int32)),
    ]


class DpePassState(C.Structure):
    _fields_ = [
        ("planes", C.POINTER(C.c_float)),
        ("weak_info", C.POINTER(C.c_uint8)),
        ("selected_views", C.POINTER(C.c_uint32)),
        ("costs", C.POINTER(C.c_float)),
    ]


def default_params() -> DpePatchMatchParams:
    """PatchMatchParams defaults (main.h:78-106)."""
    p = DpePatchMatchParams()
    p.max_iterations = 3
    p.num_images = 5
    p.sigma_spatial = 5.0
    p.sigma_color = 3.0
    p.top_k = 4
    p.depth_min = 0.0
    p.depth_max = 1.0
    p.geom_consistency = False
    p.strong_radius = 5
    p.strong_increment = 2
    p.weak_radius = 5
    p.weak_increment = 5
    p.use_APD = True
    p.use_edge = True
    p.use_limit = True
    p.use_label = True
    p.use_radius = True
    p.high_res_img = True
    p.max_scale_size = 1
    p.scale_size = 1
    p.weak_peak_radius = 2
    p.rotate_time = 4
    p.ransac_threshold = 0.005
    p.geom_factor = 0.2
    p.state = FIRST_INIT
    return p


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class PassBuffers:
    """Owns the numpy arrays behind one DpePassInput / DpePassState pair (keeps them alive)."""

    def __init__(self, pass_input: dict, state: dict):
        imgs = [np.ascontiguousarray(i, dtype=np.float32) for i in pass_input["images"]]
        n = len(imgs)
        if n > MAX_IMAGES:
            raise ValueError(f"num_images {n} > {MAX_IMAGES} (DPE.cpp:762)")
        h, w = imgs[0].shape
        self._keep = [imgs]
        self.inp = DpePassInput()
        self.inp.width, self.inp.height, self.inp.num_images = w, h, n
        img_arr = (C.POINTER(C.c_float) * n)(*[_fptr(i) for i in imgs])
        self._keep.append(img_arr)
        self.inp.images = C.cast(img_arr, C.POINTER(C.POINTER(C.c_float)))
        cams = (DpeCamera * n)()
        for i, cam in enumerate(pass_input["cams"]):
            cams[i] = cam
        self._keep.append(cams)
        self.inp.cams = C.cast(cams, C.POINTER(DpeCamera))
        depths = pass_input.get("depths")
        if depths is not None:
            ds = [None if d is None else np.ascontiguousarray(d, dtype=np.float32) for d in depths]
            self._keep.append(ds)
            darr = (C.POINTER(C.c_float) * n)(*[(C.POINTER(C.c_float)() if d is None else _fptr(d)) for d in ds])
            self._keep.append(darr)
            self.inp.depths = C.cast(darr, C.POINTER(C.POINTER(C.c_float)))
        edge = pass_input.get("edge")
        if edge is not None:
            e = np.ascontiguousarray(edge, dtype=np.uint8)
            el = np.ascontiguousarray(pass_input["edge_low"], dtype=np.uint8)
            self._keep += [e, el]
            self.inp.edge = e.ctypes.data_as(C.POINTER(C.c_uint8))
            self.inp.edge_low_res = el.ctypes.data_as(C.POINTER(C.c_uint8))
            self.inp.low_height, self.inp.low_width = el.shape
        label = pass_input.get("label")
        if label is not None:
            lab = np.ascontiguousarray(label, dtype=np.int32)
            self._keep.append(lab)
            self.inp.label = lab.ctypes.data_as(C.POINTER(C.c_int32))
        self.inp.params = pass_input["params"]
        self.inp.params.num_images = n
        self.inp.seed = int(pass_input.get("seed", 1))
        self.inp.pass_salt = int(pass_input.get("pass_salt", 0))
        if pass_input.get("image_ids") is not None:
            ids = np.ascontiguousarray(pass_input["image_ids"], np.int32)
            self._keep.append(ids)
            self.inp.image_ids = ids.ctypes.data_as(C.POINTER(C.c_int32))
        self.planes = np.ascontiguousarray(state["planes"], dtype=np.float32).reshape(h, w, 4).copy()
        self.weak = np.ascontiguousarray(state["weak"], dtype=np.uint8).reshape(h, w).copy()
        self.sel = np.ascontiguousarray(state["sel"], dtype=np.uint32).reshape(h, w).copy()
        self.costs = np.zeros((h, w), dtype=np.float32)
        self.st = DpePassState()
        self.st.planes = _fptr(self.planes)
        self.st.weak_info = self.weak.ctypes.data_as(C.POINTER(C.c_uint8))
        self.st.selected_views = self.sel.ctypes.data_as(C.POINTER(C.c_uint32))
        self.st.costs = _fptr(self.costs)

    def outputs(self) -> dict:
        return {"planes": self.planes, "weak": self.weak, "sel": self.sel, "costs": self.costs}
