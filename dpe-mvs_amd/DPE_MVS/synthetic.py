"""Synthetic pinhole multi-view scenes with known ground truth.

No datasets are reachable (no network), so every parity test and the benchmark run on scenes made
here: cameras with fx = fy = 1.2 W and principal point (W/2, H/2) on a 30 degree arc of radius 5
around the look-at point (0, 0, 5); six slanted textured rectangles in front of a textured
background plane at depth 7; band-limited value-noise texture (grey levels 128 +- ~40) attached to
the surfaces, so every view sees the same texture; one constant-intensity patch (~20 % of the
reference image) that exercises the WEAK (textureless) path.

Edges / labels stand in for the reference's OpenCV EdgeSegment (DPE.cpp:136-291, out of scope):
edges = surface-id and patch boundaries ({0,255}, CV_8UC1), labels = region id + 1 with 0 on
boundary pixels (CV_32SC1, the labels_<s>.dmb convention).
"""
from __future__ import annotations

import math
import os

import numpy as np

from . import _abi

SCENE_SEED = 20251205


def _hash2(ix: np.ndarray, iy: np.ndarray, salt: int) -> np.ndarray:
    """Deterministic integer lattice hash -> float in [-1, 1]."""
    h = (ix.astype(np.int64) * 73856093) ^ (iy.astype(np.int64) * 19349663) ^ (salt * 83492791)
    h = h.astype(np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0x5BD1E995)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    return (h.astype(np.float64) / 4294967295.0) * 2.0 - 1.0


def _value_noise(u: np.ndarray, v: np.ndarray, cell: float, salt: int) -> np.ndarray:
    fu, fv = u / cell, v / cell
    iu, iv = np.floor(fu), np.floor(fv)
    tu, tv = fu - iu, fv - iv
    su, sv = tu * tu * (3 - 2 * tu), tv * tv * (3 - 2 * tv)
    iu, iv = iu.astype(np.int64), iv.astype(np.int64)
    a = _hash2(iu, iv, salt)
    b = _hash2(iu + 1, iv, salt)
    c = _hash2(iu, iv + 1, salt)
    d = _hash2(iu + 1, iv + 1, salt)
    return (a * (1 - su) + b * su) * (1 - sv) + (c * (1 - su) + d * su) * sv


def _look_at(C: np.ndarray, O: np.ndarray) -> np.ndarray:
    z = O - C
    z = z / np.linalg.norm(z)
    down = np.array([0.0, 1.0, 0.0])
    x = np.cross(down, z)
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])


class Surface:
    def __init__(self, p0, normal, a1, half_u=None, half_v=None, salt=0, flat_region=None):
        self.p0 = np.asarray(p0, float)
        n = np.asarray(normal, float)
        self.n = n / np.linalg.norm(n)
        a1 = np.asarray(a1, float)
        a1 = a1 - self.n * (a1 @ self.n)
        self.a1 = a1 / np.linalg.norm(a1)
        self.a2 = np.cross(self.n, self.a1)
        self.hu, self.hv = half_u, half_v
        self.salt = salt
        self.flat_region = flat_region   # (u0, u1, v0, v1) constant-intensity rectangle


def build_surfaces(rng: np.random.Generator) -> list[Surface]:
    surfs = [Surface([0, 0, 7.0], [0, 0, -1], [1, 0, 0], salt=1,
                     flat_region=(-2.9, -0.45, -2.2, -0.3))]
    centers = [(-0.9, -0.75, 3.4), (0.95, -0.7, 4.2), (0.25, -0.05, 5.3), (1.15, 0.65, 3.8),
               (-0.2, -0.9, 6.0), (0.55, 0.45, 4.9)]
    for k, c in enumerate(centers):
        tilt = math.radians(rng.uniform(10, 35))
        az = rng.uniform(0, 2 * math.pi)
        n = np.array([math.sin(tilt) * math.cos(az), math.sin(tilt) * math.sin(az), -math.cos(tilt)])
        surfs.append(Surface(c, n, [1, 0.2 * rng.uniform(-1, 1), 0], half_u=rng.uniform(0.35, 0.6),
                             half_v=rng.uniform(0.3, 0.5), salt=10 + k))
    return surfs


def make_camera(K: np.ndarray, R: np.ndarray, t: np.ndarray, W: int, H: int, dmin: float, dmax: float) -> _abi.DpeCamera:
    cam = _abi.DpeCamera()
    Kf, Rf, tf = K.astype(np.float32), R.astype(np.float32), t.astype(np.float32)
    for i in range(9):
        cam.K[i] = float(Kf.flat[i])
        cam.R[i] = float(Rf.flat[i])
    for i in range(3):
        cam.t[i] = float(tf[i])
    # camera centre exactly as ReadCamera computes it (DPE.cpp:363-367)
    for j in range(3):
        cam.c[j] = float(np.float32(-(float(Rf.flat[0 + j]) * float(tf[0]) + float(Rf.flat[3 + j]) * float(tf[1])
                                      + float(Rf.flat[6 + j]) * float(tf[2]))))
    cam.width, cam.height = W, H
    cam.depth_min, cam.depth_max = float(np.float32(dmin)), float(np.float32(dmax))
    return cam


def render_view(surfs, K, R, C, W, H, pix_world: float):
    """Ray-casts one view: returns depth (camera z), surface id, world normal, grey level (f32)."""
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    Kinv = np.linalg.inv(K)
    rays_cam = np.stack([xs, ys, np.ones_like(xs)], -1) @ Kinv.T     # z component == 1
    d = rays_cam @ R                                                   # world directions (R^T r)
    best_t = np.full((H, W), np.inf)
    sid = np.full((H, W), -1, np.int32)
    for k, s in enumerate(surfs):            # visibility first: nearest surface per ray
        denom = d @ s.n
        with np.errstate(divide="ignore", invalid="ignore"):
            t = ((s.p0 - C) @ s.n) / denom
        ok = (t > 0) & np.isfinite(t)
        if s.hu is not None:
            rel = C + t[..., None] * d - s.p0
            ok &= (np.abs(rel @ s.a1) <= s.hu) & (np.abs(rel @ s.a2) <= s.hv)
        take = ok & (t < best_t)
        best_t = np.where(take, t, best_t)
        sid = np.where(take, k, sid)
    tex = np.zeros((H, W))
    for k, s in enumerate(surfs):            # then texture only where surface k is visible
        m = sid == k
        if not m.any():
            continue
        rel = C + best_t[m][:, None] * d[m] - s.p0
        u, v = rel @ s.a1, rel @ s.a2
        n = (0.42 * _value_noise(u, v, 2.5 * pix_world, s.salt) + 0.38 * _value_noise(u, v, 6.0 * pix_world, s.salt + 101)
             + 0.3 * _value_noise(u, v, 15.0 * pix_world, s.salt + 202))
        val = 128.0 + 95.0 * n
        if s.flat_region is not None:
            u0, u1, v0, v1 = s.flat_region
            flat = (u >= u0) & (u <= u1) & (v >= v0) & (v <= v1)
            val = np.where(flat, 140.0, val)
            ids = sid[m]
            ids[flat] = 100 + k
            sid[m] = ids
        tex[m] = val
    normals = np.zeros((H, W, 3))
    for k, s in enumerate(surfs):
        for key in (k, 100 + k):
            m = sid == key
            if m.any():
                n = s.n.copy()
                if (n @ (s.p0 - C)) > 0:
                    n = -n
                normals[m] = n
    img = np.clip(np.rint(tex), 0, 255).astype(np.uint8).astype(np.float32)
    depth = best_t.astype(np.float32)
    return depth, sid, normals.astype(np.float32), img


def _edges_from_ids(sid: np.ndarray) -> np.ndarray:
    e = np.zeros(sid.shape, bool)
    e[:, 1:] |= sid[:, 1:] != sid[:, :-1]
    e[:, :-1] |= sid[:, 1:] != sid[:, :-1]
    e[1:, :] |= sid[1:, :] != sid[:-1, :]
    e[:-1, :] |= sid[1:, :] != sid[:-1, :]
    return e


def make_scene(W: int, H: int, n_views: int, seed: int = SCENE_SEED, low_scale: int = 2) -> dict:
    """Renders `n_views` views (index 0 = reference) at W x H with ground truth."""
    rng = np.random.default_rng(seed)
    surfs = build_surfaces(rng)
    fx = 1.2 * W
    K = np.array([[fx, 0, W / 2.0], [0, fx, H / 2.0], [0, 0, 1.0]])
    O = np.array([0.0, 0.0, 5.0])
    angles = [0.0]
    for i in range(1, n_views):
        k = (i + 1) // 2
        sgn = 1 if i % 2 == 1 else -1
        angles.append(sgn * 15.0 * k / max(1, (n_views) // 2))
    pix_world = 5.0 / fx

    def one(i):
        th = math.radians(angles[i])
        C = O + 5.0 * np.array([math.sin(th), 0.0, -math.cos(th)])
        C[1] += 0.25 * math.sin(1.7 * i)
        R = _look_at(C, O)
        t = -R @ C
        depth, sid, normals, img = render_view(surfs, K, R, C, W, H, pix_world)
        return dict(K=K, R=R, t=t, C=C, depth=depth, sid=sid, normals=normals, image=img)

    # views are independent and numpy releases the GIL in the large array operations: render them on
    # a few threads (same arrays as a serial loop)
    from concurrent.futures import ThreadPoolExecutor
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    workers = max(1, min(len(angles), ncpu, 8))   # ~0.5 GB of temporaries per worker at 1600x1200
    if workers == 1:
        views = [one(i) for i in range(len(angles))]
    else:
        with ThreadPoolExecutor(workers) as ex:
            views = list(ex.map(one, range(len(angles))))
    zmin = min(float(v["depth"][np.isfinite(v["depth"])].min()) for v in views)
    zmax = max(float(v["depth"][np.isfinite(v["depth"])].max()) for v in views)
    dmin, dmax = 0.75 * zmin, 1.25 * zmax
    cams = [make_camera(v["K"], v["R"], v["t"], W, H, dmin, dmax) for v in views]
    sid0 = views[0]["sid"]
    edge = _edges_from_ids(sid0)
    label = np.where(edge, 0, sid0 + 1).astype(np.int32)
    lw, lh = (W + low_scale - 1) // low_scale, (H + low_scale - 1) // low_scale
    pad = np.zeros((lh * low_scale, lw * low_scale), bool)
    pad[:H, :W] = edge
    edge_low = pad.reshape(lh, low_scale, lw, low_scale).any(axis=(1, 3))
    return dict(
        W=W, H=H, N=n_views, cams=cams, views=views, dmin=dmin, dmax=dmax,
        images=[v["image"] for v in views],
        edge=(edge * 255).astype(np.uint8), edge_low=(edge_low * 255).astype(np.uint8), label=label,
        weak_gt=np.isin(sid0, [100]),
    )


def gt_state(scene: dict, seed: int = 7, depth_noise: float = 0.01, normal_noise: float = 0.05, top_views: int = 4) -> dict:
    """A REFINE-pass prior from ground truth + noise: (world normal, depth), weak map, view mask."""
    rng = np.random.default_rng(seed)
    v0 = scene["views"][0]
    H, W = scene["H"], scene["W"]
    depth = v0["depth"] * (1.0 + depth_noise * rng.standard_normal((H, W)).astype(np.float32))
    n = v0["normals"] + normal_noise * rng.standard_normal((H, W, 3)).astype(np.float32)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    planes = np.concatenate([n, depth[..., None]], -1).astype(np.float32)
    weak = np.full((H, W), _abi.STRONG, np.uint8)
    weak[scene["weak_gt"]] = _abi.WEAK
    m = 6
    weak[:m, :] = _abi.UNKNOWN
    weak[-m:, :] = _abi.UNKNOWN
    weak[:, :m] = _abi.UNKNOWN
    weak[:, -m:] = _abi.UNKNOWN
    nv = scene["N"] - 1
    k = min(top_views, nv)
    sel = np.zeros((H, W), np.uint32)
    for _ in range(k):
        bit = rng.integers(0, nv, size=(H, W)).astype(np.uint32)
        sel |= (np.uint32(1) << bit)
    return dict(planes=planes, weak=weak, sel=sel)


def src_depths(scene: dict, seed: int = 11, noise: float = 0.01) -> list:
    rng = np.random.default_rng(seed)
    out = [None]
    for v in scene["views"][1:]:
        d = v["depth"] * (1.0 + noise * rng.standard_normal(v["depth"].shape).astype(np.float32))
        out.append(d.astype(np.float32))
    return out


def pass_input(scene: dict, params, depths=None, seed: int = 1, pass_salt: int = 0) -> dict:
    params.depth_min = float(np.float32(scene["cams"][0].depth_min) * np.float32(0.6))    # DPE.cpp:788
    params.depth_max = float(np.float32(scene["cams"][0].depth_max) * np.float32(1.2))    # DPE.cpp:789
    return dict(images=scene["images"], cams=scene["cams"], depths=depths, edge=scene["edge"],
                edge_low=scene["edge_low"], label=scene["label"], params=params, seed=seed, pass_salt=pass_salt)


def first_init_state(scene: dict) -> dict:
    H, W = scene["H"], scene["W"]
    return dict(planes=np.zeros((H, W, 4), np.float32), weak=np.full((H, W), _abi.STRONG, np.uint8),
                sel=np.zeros((H, W), np.uint32))


def _labels_edges_at(sid: np.ndarray, w: int, h: int):
    """Edges ({0,255} u8) and labels (region id + 1, 0 on edges, i32) of a surface-id map sampled
    (nearest) at w x h -- the stand-in for EdgeSegment's edges_<s>.dmb / labels_<s>.dmb."""
    H, W = sid.shape
    ry = np.minimum(((np.arange(h) + 0.5) * H / h).astype(np.int64), H - 1)
    rx = np.minimum(((np.arange(w) + 0.5) * W / w).astype(np.int64), W - 1)
    s = sid[np.ix_(ry, rx)]
    e = _edges_from_ids(s)
    return (e * 255).astype(np.uint8), np.where(e, 0, s + 1).astype(np.int32)


def write_dense_folder(folder: str, W: int, H: int, n_views: int, seed: int = SCENE_SEED, jpeg_quality: int = 95,
                       max_src: int = 8, with_edges: bool = True, scene: dict | None = None) -> dict:
    """Writes a complete DPE-MVS dense_folder for a synthetic scene: images/%08d.jpg (8-bit grey),
    cams/%08d_cam.txt (4-number depth line), pair.txt, and per reference image the EdgeSegment
    outputs DPE/%08d/edges_<s>.dmb and labels_<s>.dmb for every pyramid scale of the schedule."""
    import os
    from PIL import Image
    from . import pipeline
    sc = scene if scene is not None else make_scene(W, H, n_views, seed=seed)
    os.makedirs(os.path.join(folder, "images"), exist_ok=True)
    os.makedirs(os.path.join(folder, "cams"), exist_ok=True)
    for i, v in enumerate(sc["views"]):
        Image.fromarray(v["image"].astype(np.uint8), mode="L").save(
            os.path.join(folder, "images", f"{i:08d}.jpg"), format="JPEG", quality=jpeg_quality)
        pipeline.write_camera(os.path.join(folder, "cams", f"{i:08d}_cam.txt"), v["K"], v["R"], v["t"],
                              sc["dmin"], sc["dmax"])
    with open(os.path.join(folder, "pair.txt"), "w") as f:
        f.write(f"{n_views}\n")
        for i in range(n_views):
            others = sorted((j for j in range(n_views) if j != i), key=lambda j: (abs(j - i), j))[:max_src]
            f.write(f"{i}\n{len(others)} " + " ".join(f"{j} {100.0 - 5 * abs(i - j):.1f}" for j in others) + "\n")
    if not with_edges:      # leave the edge / label maps to the pipeline's EdgeSegment
        return sc
    max_size, rounds = max(W, H), 1
    while max_size > 800:
        max_size //= 2
        rounds += 1
    rounds = max(rounds, 2)
    for i, v in enumerate(sc["views"]):
        rf = os.path.join(folder, pipeline.OUT_NAME, f"{i:08d}")
        os.makedirs(rf, exist_ok=True)
        for s in range(rounds):
            f = 1.0 / (1 << s)
            w, h = pipeline.std_round(np.float32(W) * np.float32(f)), pipeline.std_round(np.float32(H) * np.float32(f))
            e, lab = _labels_edges_at(v["sid"], w, h)
            pipeline.write_bin_mat(os.path.join(rf, f"edges_{s}.dmb"), e)
            pipeline.write_bin_mat(os.path.join(rf, f"labels_{s}.dmb"), lab)
    return sc
