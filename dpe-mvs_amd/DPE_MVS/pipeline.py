"""Host pipeline around the HIP PatchMatch pass: the reference's RunDPEPipeline / ProcessProblem /
InuputInitialization (main.cpp:264-600, DPE.cpp:293-382, 733-1052, 1123-1168), restated for a
one-process-per-GPU deployment.

What it keeps from the reference:
  * the dense_folder contract: images/%08d.jpg, cams/%08d_cam.txt, pair.txt in; DPE/%08d/ results,
    edges_<s>.dmb / labels_<s>.dmb (EdgeSegment output) read from the result folders;
  * the coarse-to-fine schedule (ComputeRoundNum, FIRST_INIT/REFINE_INIT/REFINE_ITER parameters per
    round, main.cpp:390-408, 492-570) and the per-pass epilogue (main.cpp:423-446);
  * the .dmb / .npy file formats and the final depth.npy / normal.npy / weak.npy / edge.npy;
  * RescaleMatToTargetSize with its swapped x/y factors (DPE.cpp:1146-1168).

What it does differently (MI355X-first):
  * images are decoded once per run and their pyramid levels cached; per-image state (depth,
    normal, weak, selected views) stays in memory between passes instead of .dmb round trips;
  * one process per GPU: with torch.distributed initialised, problems are split into contiguous
    blocks per rank and, after every pass, the f32 depth maps are all-gathered (RCCL over xGMI with
    the "nccl" backend, gloo on CPU) -- the only cross-image data of the path;
  * schedule "reference" = the reference's serial order (later images see same-pass depths of
    earlier ones, Gauss-Seidel); "jacobi" = every pass reads the depths of the previous pass; the
    multi-rank run is Jacobi and is bit-identical to a 1-rank Jacobi run.

Not built here: EdgeSegment (edges/labels must already be in the result folders),
RunFusion (fusion=True raises), the viz medium results (ignored).
"""
from __future__ import annotations

import math
import os
import struct
import sys
from dataclasses import dataclass, field

import numpy as np

from . import _abi

OUT_NAME = "DPE"

# OpenCV type codes used by the .dmb files (cv::Mat::type())
CV_8UC1, CV_8SC1, CV_32SC1, CV_32FC1, CV_32FC3 = 0, 1, 4, 5, 21
_CV_DTYPE = {CV_8UC1: (np.uint8, 1), CV_8SC1: (np.int8, 1), CV_32SC1: (np.int32, 1), CV_32FC1: (np.float32, 1),
             CV_32FC3: (np.float32, 3)}


class PipelineError(RuntimeError):
    pass


# ------------------------------------------------------------------------------ file formats
def read_bin_mat(path: str) -> np.ndarray:
    """ReadBinMat (DPE.cpp:293-318): int32 version=1, rows, cols, type, then the raw rows."""
    with open(path, "rb") as f:
        hdr = f.read(16)
        if len(hdr) != 16:
            raise PipelineError(f"truncated .dmb header: {path}")
        version, rows, cols, typ = struct.unpack("<4i", hdr)
        if version != 1:
            raise PipelineError(f"Version error: {path}")
        if typ not in _CV_DTYPE:
            raise PipelineError(f"unsupported .dmb type {typ}: {path}")
        dt, ch = _CV_DTYPE[typ]
        n = rows * cols * ch
        a = np.frombuffer(f.read(n * np.dtype(dt).itemsize), dtype=dt)
        if a.size != n:
            raise PipelineError(f"truncated .dmb data: {path}")
    return a.reshape((rows, cols, ch) if ch > 1 else (rows, cols)).copy()


def write_bin_mat(path: str, mat: np.ndarray) -> None:
    """WriteBinMat (DPE.cpp:320-339)."""
    mat = np.ascontiguousarray(mat)
    ch = mat.shape[2] if mat.ndim == 3 else 1
    typ = {(np.dtype(np.uint8), 1): CV_8UC1, (np.dtype(np.int8), 1): CV_8SC1, (np.dtype(np.int32), 1): CV_32SC1,
           (np.dtype(np.uint32), 1): CV_32SC1, (np.dtype(np.float32), 1): CV_32FC1,
           (np.dtype(np.float32), 3): CV_32FC3}[(mat.dtype, ch)]
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", 1, mat.shape[0], mat.shape[1], typ))
        f.write(mat.tobytes())


def read_camera(path: str) -> _abi.DpeCamera:
    """ReadCamera (DPE.cpp:341-382): extrinsic 4x4, intrinsic 3x3, 'depth_min interval depth_num
    depth_max' (a value missing from the depth line reads as 0, as the failed stream extraction does)."""
    with open(path) as f:
        tok = f.read().split()
    cam = _abi.DpeCamera()
    pos = 1                                   # skip "extrinsic"
    vals = []
    for _ in range(3):
        row = [np.float32(tok[pos + k]) for k in range(4)]
        vals.append(row)
        pos += 4
    pos += 4                                  # last extrinsic row
    pos += 1                                  # "intrinsic"
    K = [np.float32(tok[pos + k]) for k in range(9)]
    pos += 9
    for i in range(3):
        cam.R[3 * i + 0], cam.R[3 * i + 1], cam.R[3 * i + 2] = (float(vals[i][0]), float(vals[i][1]), float(vals[i][2]))
        cam.t[i] = float(vals[i][3])
    for i in range(9):
        cam.K[i] = float(K[i])
    R, t = [float(np.float32(v)) for v in cam.R], [float(np.float32(v)) for v in cam.t]
    for j in range(3):
        cam.c[j] = float(np.float32(-(R[0 + j] * t[0] + R[3 + j] * t[1] + R[6 + j] * t[2])))
    depth = [float(np.float32(tok[pos + k])) if pos + k < len(tok) else 0.0 for k in range(4)]
    cam.depth_min, cam.depth_max = depth[0], depth[3]
    return cam


def write_camera(path: str, K: np.ndarray, R: np.ndarray, t: np.ndarray, dmin: float, dmax: float, depth_num: int = 192):
    """The cams/%08d_cam.txt format ReadCamera parses (4-number depth line)."""
    g = lambda v: repr(float(v))
    with open(path, "w") as f:
        f.write("extrinsic\n")
        for i in range(3):
            f.write(f"{g(R[i, 0])} {g(R[i, 1])} {g(R[i, 2])} {g(t[i])}\n")
        f.write("0.0 0.0 0.0 1.0\n\nintrinsic\n")
        for i in range(3):
            f.write(f"{g(K[i, 0])} {g(K[i, 1])} {g(K[i, 2])}\n")
        f.write(f"\n{g(dmin)} {g((dmax - dmin) / depth_num)} {depth_num} {g(dmax)}\n")


def write_npy(path: str, arr: np.ndarray) -> None:
    """WriteMatToNpy (main.cpp:47-96): .npy v1.0, C order."""
    np.save(path, np.ascontiguousarray(arr), allow_pickle=False)


def fmt_index(i: int) -> str:   # ToFormatIndex
    return f"{i:08d}"


def imread_gray(path: str) -> np.ndarray:
    """cv::imread(path, IMREAD_GRAYSCALE) -> uint8 [H][W].  Decoded with PIL (OpenCV is absent here;
    colour -> grey uses ITU-R 601 luma like OpenCV, JPEG IDCT rounding may differ by 1 level)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("L"), dtype=np.uint8).copy()


# ------------------------------------------------------------------------------ resampling
def _linear_taps(n_src: int, n_dst: int):
    """cv::resize INTER_LINEAR source index / weight per destination coordinate (float path)."""
    scale = 1.0 / (n_dst / n_src)
    d = np.arange(n_dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    hi = s >= n_src - 1
    f[hi], s[hi] = 0, n_src - 1
    s1 = np.minimum(s + 1, n_src - 1)
    return s, s1, (np.float32(1) - f).astype(np.float32), f


def resize_linear(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv::resize(src, dst, Size(new_w, new_h), 0, 0, INTER_LINEAR) for CV_32FC1: horizontal then
    vertical 2-tap pass in float32 (DPE.cpp:798-822).  Parity vs OpenCV is unpinned (no cv2 here)."""
    img = np.asarray(img, dtype=np.float32)
    h, w = img.shape
    if (w, h) == (new_w, new_h):
        return img.copy()
    xs0, xs1, ax0, ax1 = _linear_taps(w, new_w)
    ys0, ys1, ay0, ay1 = _linear_taps(h, new_h)
    rows = img[:, xs0] * ax0[None, :] + img[:, xs1] * ax1[None, :]
    out = rows[ys0, :] * ay0[:, None] + rows[ys1, :] * ay1[:, None]
    return out.astype(np.float32)


def rescale_to(src: np.ndarray, W: int, H: int) -> np.ndarray:
    """RescaleMatToTargetSize (DPE.cpp:1146-1168), nearest, with the reference's swapped factors:
    o_r = (int)(r / scale_x), o_c = (int)(c / scale_y).  Out-of-range taps keep 0 (uninitialised
    cv::Mat memory in the reference)."""
    h, w = src.shape[:2]
    if (w, h) == (W, H):
        return src
    sx = np.float32(W) / np.float32(w)
    sy = np.float32(H) / np.float32(h)
    r = np.arange(H, dtype=np.float32)
    c = np.arange(W, dtype=np.float32)
    o_r = (r / sx).astype(np.int64)
    o_c = (c / sy).astype(np.int64)
    dst = np.zeros((H, W) + src.shape[2:], dtype=src.dtype)
    vr = (o_r >= 0) & (o_r < h)
    vc = (o_c >= 0) & (o_c < w)
    dst[np.ix_(vr, vc)] = src[np.ix_(o_r[vr], o_c[vc])]
    return dst


# ------------------------------------------------------------------------------ problems
@dataclass
class Problem:   # main.h:108-118
    index: int
    ref_image_id: int
    src_image_ids: list
    dense_folder: str
    result_folder: str
    scale_size: int = 1
    params: _abi.DpePatchMatchParams = field(default_factory=_abi.default_params)
    show_medium_result: bool = False
    iteration: int = 0


def generate_sample_list(dense_folder: str, viz: bool = False) -> list:
    """GenerateSampleList (main.cpp:264-308): pair.txt; sources with score <= 0 are dropped."""
    with open(os.path.join(dense_folder, "pair.txt")) as f:
        lines = f.read().splitlines()
    n = int(lines[0].split()[0])
    problems = []
    li = 1
    for i in range(n):
        ref = int(lines[li].split()[0])
        tok = lines[li + 1].split()
        li += 2
        m = int(tok[0])
        srcs = []
        for j in range(m):
            sid, score = int(tok[1 + 2 * j]), float(np.float32(tok[2 + 2 * j]))
            if score <= 0.0:
                continue
            srcs.append(sid)
        rf = os.path.join(dense_folder, OUT_NAME, fmt_index(ref))
        os.makedirs(rf, exist_ok=True)
        problems.append(Problem(index=i, ref_image_id=ref, src_image_ids=srcs, dense_folder=dense_folder,
                                result_folder=rf, show_medium_result=viz))
    return problems


class ImageCache:
    """Decoded grey images (f32) and their INTER_LINEAR pyramid levels, decoded once per run."""

    def __init__(self, dense_folder: str):
        self.folder = os.path.join(dense_folder, "images")
        self._full = {}
        self._lvl = {}

    def full(self, idx: int) -> np.ndarray:
        if idx not in self._full:
            self._full[idx] = imread_gray(os.path.join(self.folder, fmt_index(idx) + ".jpg")).astype(np.float32)
        return self._full[idx]

    def level(self, idx: int, scale_size: int) -> np.ndarray:
        key = (idx, scale_size)
        if key not in self._lvl:
            img = self.full(idx)
            if scale_size == 1:
                self._lvl[key] = img
            else:
                factor = np.float32(1.0) / np.float32(scale_size)
                nw = _std_round(np.float32(img.shape[1]) * factor)
                nh = _std_round(np.float32(img.shape[0]) * factor)
                self._lvl[key] = resize_linear(img, nw, nh)
        return self._lvl[key]


def _std_round(v) -> int:
    """std::round (half away from zero) of a non-negative float."""
    return int(math.floor(float(v) + 0.5))


def check_images(problems: list, cache: ImageCache) -> bool:
    """CheckImages (main.cpp:310-329): every image decodes and has the first one's size."""
    if not problems:
        return False
    try:
        shape = cache.full(problems[0].ref_image_id).shape
        return all(cache.full(p.ref_image_id).shape == shape for p in problems[1:])
    except (OSError, ValueError):
        return False


def compute_round_num(problems: list, cache: ImageCache) -> int:
    """ComputeRoundNum (main.cpp:390-408): halve max(W, H) until <= 800; at least 2 rounds."""
    if not problems:
        return 0
    h, w = cache.full(problems[0].ref_image_id).shape
    max_size, rounds = max(w, h), 1
    while max_size > 800:
        max_size //= 2
        rounds += 1
    return max(rounds, 2)


def _scale_index(scale_size: int) -> int:
    s = 0
    while (1 << s) < scale_size:
        s += 1
    return s


@dataclass
class ImageState:
    """What the reference keeps in depths.dmb / normals.dmb / weak.bin / selected_views.bin."""
    depth: np.ndarray
    normal: np.ndarray
    weak: np.ndarray
    sel: np.ndarray


# ------------------------------------------------------------------------------ one problem
def input_initialization(problem: Problem, cache: ImageCache, states: dict, depth_src: dict,
                         base_seed: int) -> tuple:
    """InuputInitialization + SupportInitialization (DPE.cpp:733-914, 1025-1052) -> pass input/state."""
    P = problem.params
    ids = [problem.ref_image_id] + list(problem.src_image_ids)
    if len(ids) > _abi.MAX_IMAGES:
        raise PipelineError(f"Can't process so much images: {len(ids)}")
    full_h, full_w = cache.full(ids[0]).shape
    images, cams = [], []
    for idx in ids:
        cam = read_camera(os.path.join(problem.dense_folder, "cams", fmt_index(idx) + "_cam.txt"))
        cam.width, cam.height = full_w, full_h
        img = cache.level(idx, problem.scale_size)
        if problem.scale_size != 1:
            h, w = img.shape
            sx = np.float32(w) / np.float32(full_w)
            sy = np.float32(h) / np.float32(full_h)
            cam.K[0] = float(np.float32(cam.K[0]) * sx)
            cam.K[2] = float(np.float32(cam.K[2]) * sx)
            cam.K[4] = float(np.float32(cam.K[4]) * sy)
            cam.K[5] = float(np.float32(cam.K[5]) * sy)
            cam.width, cam.height = w, h
        images.append(img)
        cams.append(cam)
    H, W = images[0].shape
    P.depth_min = float(np.float32(cams[0].depth_min) * np.float32(0.6))
    P.depth_max = float(np.float32(cams[0].depth_max) * np.float32(1.2))
    P.num_images = len(images)
    depths = None
    if P.geom_consistency:
        depths = [None]
        for sid in problem.src_image_ids:
            if sid not in depth_src:
                raise PipelineError(f"no depth map of source image {sid} for the geometric-consistency pass")
            d = depth_src[sid]
            depths.append(rescale_to(d, W, H) if d.shape != (H, W) else d)
    st_prev = states.get(problem.ref_image_id)
    if P.use_APD:
        if st_prev is None:
            raise PipelineError(f"Can't find weak info of image {problem.ref_image_id}")
        weak = rescale_to(st_prev.weak, W, H).copy()
    else:
        weak = np.full((H, W), _abi.STRONG, np.uint8)
    planes = np.zeros((H, W, 4), np.float32)
    sel = np.zeros((H, W), np.uint32)
    if P.state != _abi.FIRST_INIT:
        if st_prev is None:
            raise PipelineError(f"no prior depth/normal for image {problem.ref_image_id}")
        d, n = st_prev.depth, st_prev.normal
        if d.shape != (H, W) or n.shape[:2] != (H, W):
            d, n = rescale_to(d, W, H), rescale_to(n, W, H)
        planes[..., :3] = n
        planes[..., 3] = d
        sel = rescale_to(st_prev.sel, W, H).copy()
    inp = dict(images=images, cams=cams, depths=depths, params=P,
               seed=(base_seed ^ (problem.ref_image_id * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF,
               pass_salt=problem.iteration)
    if P.use_edge or P.use_limit:
        s = _scale_index(problem.scale_size)
        max_s = _scale_index(P.max_scale_size) if P.high_res_img else s
        inp["edge"] = _read_support(problem, f"edges_{s}.dmb")
        inp["edge_low"] = _read_support(problem, f"edges_{max_s}.dmb")
    if P.use_label:
        inp["label"] = _read_support(problem, f"labels_{_scale_index(problem.scale_size)}.dmb")
    return inp, dict(planes=planes, weak=weak, sel=sel)


def _read_support(problem: Problem, name: str) -> np.ndarray:
    path = os.path.join(problem.result_folder, name)
    if not os.path.exists(path):
        raise PipelineError(f"{path} missing: the EdgeSegment edge/label precompute (DPE.cpp:9-291) is not part "
                            "of this build (SURVEY.md §8f); provide edges_<s>.dmb / labels_<s>.dmb")
    return read_bin_mat(path)


def epilogue(problem: Problem, out: dict) -> ImageState:
    """ProcessProblem epilogue (main.cpp:423-437): depth outside [dmin, dmax] -> 0 and UNKNOWN."""
    P = problem.params
    planes, weak = out["planes"], out["weak"].copy()
    depth = planes[..., 3].copy()
    bad = (depth < np.float32(P.depth_min)) | (depth > np.float32(P.depth_max))
    depth[bad] = 0.0
    weak[bad] = _abi.UNKNOWN
    return ImageState(depth=depth, normal=np.ascontiguousarray(planes[..., :3]), weak=weak, sel=out["sel"].copy())


# ------------------------------------------------------------------------------ runners
class NativeRunner:
    """The product pass executor: the HIP library through its C-ABI (no CPU fallback)."""

    def __init__(self, device: int = 0):
        from . import native
        self.ctx = native.PatchMatchContext(device)

    def run(self, pass_input: dict, state: dict) -> dict:
        return self.ctx.run(pass_input, state)

    def close(self):
        self.ctx.close()


# ------------------------------------------------------------------------------ the pipeline
def _pass_params(problem: Problem, i: int, j: int) -> None:
    """Per-pass parameters of RunDPEPipeline (main.cpp:510-556); j = -1 for the round's first pass."""
    p = problem.params
    if j < 0:
        if i == 0:
            p.state, p.use_APD, p.use_edge = _abi.FIRST_INIT, False, False
        else:
            p.state, p.use_APD, p.use_edge = _abi.REFINE_INIT, True, True
            p.ransac_threshold = float(np.float32(0.01 - i * 0.00125))
            p.rotate_time = min(int(2 ** i), 4)
        p.geom_consistency = False
        p.max_iterations = 3
        p.weak_peak_radius = 6
    else:
        p.state = _abi.REFINE_ITER
        p.use_APD = i != 0
        p.use_edge = i != 0
        p.ransac_threshold = float(np.float32(0.01 - i * 0.00125))
        p.rotate_time = min(int(2 ** i), 4)
        p.geom_consistency = True
        p.max_iterations = 3
        p.weak_peak_radius = max(4 - 2 * j, 2)


def _gather_depths(dist, mine: list, problems: list, blocks: list, depth_cur: dict, device) -> None:
    """All-gather of the f32 depth maps of every rank's problems (one collective per pass)."""
    import torch
    world = dist.get_world_size()
    nmax = max(len(b) for b in blocks)
    H, W = depth_cur[mine[0].ref_image_id].shape if mine else next(iter(depth_cur.values())).shape
    buf = torch.zeros((nmax, H, W), dtype=torch.float32)
    for k, p in enumerate(mine):
        buf[k] = torch.from_numpy(depth_cur[p.ref_image_id])
    buf = buf.to(device)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    for r in range(world):
        o = outs[r].cpu().numpy()
        for k, pi in enumerate(blocks[r]):
            depth_cur[problems[pi].ref_image_id] = o[k].copy()


def run_dpe_pipeline(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False,
                     viz: bool = False, depth: bool = True, normal: bool = False, weak: bool = False,
                     edge: bool = False, runner=None, schedule: str = "reference", dist=None,
                     base_seed: int = 0x5EED, keep_intermediate: bool = False) -> int:
    """RunDPEPipeline (main.cpp:474-600).  `runner` defaults to the HIP library on `gpu_index`.
    With `dist` (an initialised torch.distributed), problems are split in contiguous blocks per rank
    and depth maps are all-gathered after every pass (Jacobi schedule)."""
    if fusion:
        raise PipelineError("fusion=True: RunFusion (DPE.cpp:1220-1370) is not part of this build (SURVEY.md §8f)")
    if schedule not in ("reference", "jacobi"):
        raise ValueError("schedule must be 'reference' or 'jacobi'")
    os.makedirs(os.path.join(dense_folder, OUT_NAME), exist_ok=True)
    problems = generate_sample_list(dense_folder, viz)
    cache = ImageCache(dense_folder)
    if not check_images(problems, cache):
        print("Images may error, check it!", file=sys.stderr)
        return 1
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    if world > 1:
        schedule = "jacobi"
    n = len(problems)
    blocks = [list(range(r * n // world, (r + 1) * n // world)) for r in range(world)]
    mine = [problems[i] for i in blocks[rank]]
    own_runner = runner is None
    if own_runner:
        runner = NativeRunner(gpu_index)
    device = "cpu"
    if dist is not None and dist.get_backend() == "nccl":
        import torch
        device = torch.device("cuda", torch.cuda.current_device())
    try:
        round_num = compute_round_num(problems, cache)
        if verbose and rank == 0:
            print(f"There are {n} images to be processed!")
            print(f"There are {round_num} resolution stages for coarse-to-fine processing!")
            print(f"Iteration nums: {round_num * 4}")
        for p in problems:
            p.params.max_scale_size = max(1, int(2 ** (round_num - 1)))
        states = {}            # ref id -> ImageState (this rank's problems)
        depth_cur = {}         # ref id -> depth map seen by geometric-consistency passes
        iteration_index = 0
        for i in range(round_num):
            for j in range(-1, 3):
                depth_src = dict(depth_cur) if schedule == "jacobi" else depth_cur
                for p in mine:
                    p.iteration = iteration_index
                    p.scale_size = int(2 ** (round_num - 1 - i))
                    p.params.scale_size = p.scale_size
                    _pass_params(p, i, j)
                    inp, st = input_initialization(p, cache, states, depth_src, base_seed)
                    out = runner.run(inp, st)
                    states[p.ref_image_id] = s = epilogue(p, out)
                    depth_cur[p.ref_image_id] = s.depth
                    if keep_intermediate:
                        _write_intermediate(p, s)
                if world > 1:
                    _gather_depths(dist, mine, problems, blocks, depth_cur, device)
                if verbose and rank == 0:
                    print(f"Iteration {iteration_index + 1} / {round_num * 4} done")
                iteration_index += 1
        for p in mine:     # main.cpp:572-578
            s = states[p.ref_image_id]
            if depth:
                d = s.depth.copy()
                d[s.weak == _abi.UNKNOWN] = 0.0
                write_npy(os.path.join(p.result_folder, "depth.npy"), d)
            if normal:
                write_npy(os.path.join(p.result_folder, "normal.npy"), s.normal.astype(np.float32))
            if weak:
                enc = np.zeros(s.weak.shape, np.int8)
                enc[s.weak == _abi.WEAK] = 1
                enc[s.weak == _abi.STRONG] = 2
                write_npy(os.path.join(p.result_folder, "weak.npy"), enc)
            if edge:
                e = _first_edge_file(p.result_folder)
                if e is not None:
                    write_npy(os.path.join(p.result_folder, "edge.npy"), (read_bin_mat(e) > 0).astype(np.int8))
        if verbose and rank == 0:
            print("All done")
        return 0
    finally:
        if own_runner:
            runner.close()


def _first_edge_file(folder: str):
    for idx in range(8):
        c = os.path.join(folder, f"edges_{idx}.dmb")
        if os.path.exists(c):
            return c
    return None


def _write_intermediate(p: Problem, s: ImageState) -> None:
    write_bin_mat(os.path.join(p.result_folder, "depths.dmb"), s.depth)
    write_bin_mat(os.path.join(p.result_folder, "normals.dmb"), s.normal.astype(np.float32))
    write_bin_mat(os.path.join(p.result_folder, "weak.bin"), s.weak)
    write_bin_mat(os.path.join(p.result_folder, "selected_views.bin"), s.sel.view(np.int32))


def dpe_mvs(dense_folder: str, gpu_index: int = 0, verbose: bool = True, fusion: bool = False, viz: bool = False,
            depth: bool = True, normal: bool = False, weak: bool = False, edge: bool = False) -> int:
    """DPE_MVS.dpe_mvs (src/DPE_MVS/__init__.py:6-17, csrc/bindings.cpp:31-43): same signature,
    returns 0, raises RuntimeError on failure."""
    rc = run_dpe_pipeline(dense_folder, gpu_index, verbose, fusion, viz, depth, normal, weak, edge)
    if rc != 0:
        raise RuntimeError(f"DPE pipeline failed with code {rc}")
    return rc
