"""COLMAP sparse model -> DPE-MVS dense_folder (cams/%08d_cam.txt, pair.txt, images/%08d.jpg).

Rewrite of the reference's converter (src/DPE_MVS/colmap2mvsnet.py:305-499) without OpenCV: the
COLMAP readers follow COLMAP's documented text / binary formats, image I/O uses PIL.  Same command
line and the same outputs:

  * intrinsics K / scale_factor per camera model (:347-376);
  * extrinsics from the quaternion and translation (:383-391);
  * depth range per image from the 1 % / 99 % depth percentiles of its observed 3-D points,
    relaxed by x0.75 / x1.25; `max_d` depth samples (0: the inverse-depth count) (:393-427);
  * view selection: for every image pair the number of co-observed 3-D points, zeroed when the
    75th-percentile triangulation angle is below 1 degree; the 20 best views per image (:305-327,
    :429-447);
  * images padded to the largest size, nearest-resized by 1 / scale_factor, written as JPEG
    (:475-494).  cv2.imwrite and PIL are different JPEG encoders, so the written files are not
    byte-identical to the reference's (the pixels they encode are).

    python -m DPE_MVS.colmap2mvsnet --dense_folder D --save_folder S [--model_ext .txt|.bin]
"""
from __future__ import annotations

import argparse
import math
import os
import shutil
import struct
from dataclasses import dataclass, field

import numpy as np

# COLMAP camera models: id -> (name, number of parameters)
CAMERA_MODELS = {0: ("SIMPLE_PINHOLE", 3), 1: ("PINHOLE", 4), 2: ("SIMPLE_RADIAL", 4), 3: ("RADIAL", 5),
                 4: ("OPENCV", 8), 5: ("OPENCV_FISHEYE", 8), 6: ("FULL_OPENCV", 12), 7: ("FOV", 5),
                 8: ("SIMPLE_RADIAL_FISHEYE", 4), 9: ("RADIAL_FISHEYE", 5), 10: ("THIN_PRISM_FISHEYE", 12)}
PARAM_NAMES = {
    "SIMPLE_PINHOLE": ["f", "cx", "cy"], "PINHOLE": ["fx", "fy", "cx", "cy"],
    "SIMPLE_RADIAL": ["f", "cx", "cy", "k"], "SIMPLE_RADIAL_FISHEYE": ["f", "cx", "cy", "k"],
    "RADIAL": ["f", "cx", "cy", "k1", "k2"], "RADIAL_FISHEYE": ["f", "cx", "cy", "k1", "k2"],
    "OPENCV": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2"],
    "OPENCV_FISHEYE": ["fx", "fy", "cx", "cy", "k1", "k2", "k3", "k4"],
    "FULL_OPENCV": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "k4", "k5", "k6"],
    "FOV": ["fx", "fy", "cx", "cy", "omega"],
    "THIN_PRISM_FISHEYE": ["fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "k4", "sx1", "sy1"],
}


@dataclass
class Camera:
    id: int
    model: str
    width: int
    height: int
    params: np.ndarray


@dataclass
class Image:
    id: int
    qvec: np.ndarray
    tvec: np.ndarray
    camera_id: int
    name: str
    xys: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))
    point3D_ids: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))


@dataclass
class Point3D:
    id: int
    xyz: np.ndarray


# ------------------------------------------------------------------------------ COLMAP readers
def _lines(path):
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                yield line


def read_cameras_text(path) -> dict:
    cams = {}
    for line in _lines(path):
        e = line.split()
        cams[int(e[0])] = Camera(int(e[0]), e[1], int(e[2]), int(e[3]), np.array([float(v) for v in e[4:]]))
    return cams


def read_images_text(path) -> dict:
    imgs = {}
    it = _lines(path)
    for line in it:
        e = line.split()
        img = Image(int(e[0]), np.array([float(v) for v in e[1:5]]), np.array([float(v) for v in e[5:8]]),
                    int(e[8]), e[9])
        pts = next(it, "").split()
        if pts:
            a = np.array(pts, dtype=object).reshape(-1, 3)
            img.xys = a[:, :2].astype(float)
            img.point3D_ids = a[:, 2].astype(np.int64)
        imgs[img.id] = img
    return imgs


def read_points3d_text(path) -> dict:
    pts = {}
    for line in _lines(path):
        e = line.split()
        pts[int(e[0])] = Point3D(int(e[0]), np.array([float(v) for v in e[1:4]]))
    return pts


def _read(f, fmt):
    size = struct.calcsize("<" + fmt)
    return struct.unpack("<" + fmt, f.read(size))


def read_cameras_binary(path) -> dict:
    cams = {}
    with open(path, "rb") as f:
        for _ in range(_read(f, "Q")[0]):
            cid, mid, w, h = _read(f, "iiQQ")
            name, n = CAMERA_MODELS[mid]
            cams[cid] = Camera(cid, name, w, h, np.array(_read(f, "d" * n)))
    return cams


def read_images_binary(path) -> dict:
    imgs = {}
    with open(path, "rb") as f:
        for _ in range(_read(f, "Q")[0]):
            iid = _read(f, "i")[0]
            q = np.array(_read(f, "dddd"))
            t = np.array(_read(f, "ddd"))
            cid = _read(f, "i")[0]
            name = b""
            c = f.read(1)
            while c != b"\x00":
                name += c
                c = f.read(1)
            n = _read(f, "Q")[0]
            raw = np.frombuffer(f.read(24 * n), dtype=np.dtype([("x", "<f8"), ("y", "<f8"), ("id", "<i8")]))
            imgs[iid] = Image(iid, q, t, cid, name.decode(), np.stack([raw["x"], raw["y"]], 1), raw["id"].astype(np.int64))
    return imgs


def read_points3d_binary(path) -> dict:
    pts = {}
    with open(path, "rb") as f:
        for _ in range(_read(f, "Q")[0]):
            pid = _read(f, "Q")[0]
            xyz = np.array(_read(f, "ddd"))
            _read(f, "BBB")
            _read(f, "d")
            track = _read(f, "Q")[0]
            f.read(8 * track)
            pts[pid] = Point3D(pid, xyz)
    return pts


def read_model(path: str, ext: str):
    if ext == ".txt":
        return (read_cameras_text(os.path.join(path, "cameras.txt")), read_images_text(os.path.join(path, "images.txt")),
                read_points3d_text(os.path.join(path, "points3D.txt")))
    return (read_cameras_binary(os.path.join(path, "cameras.bin")), read_images_binary(os.path.join(path, "images.bin")),
            read_points3d_binary(os.path.join(path, "points3D.bin")))


def qvec2rotmat(q) -> np.ndarray:
    w, x, y, z = q
    return np.array([[1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
                     [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
                     [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y]])


# ------------------------------------------------------------------------------ conversion
def pair_score(i: int, j: int, images: dict, points3d: dict, extrinsic: dict) -> float:
    """Co-observed 3-D points of images i and j (1-based keys), 0 when the 75th-percentile
    triangulation angle is under 1 degree (reference :305-327)."""
    ids_j = set(int(v) for v in images[j].point3D_ids)
    common = [int(p) for p in images[i].point3D_ids if int(p) in ids_j and int(p) != -1]
    ci = -extrinsic[i][:3, :3].T @ extrinsic[i][:3, 3]
    cj = -extrinsic[j][:3, :3].T @ extrinsic[j][:3, 3]
    angles = []
    for pid in common:
        p = points3d[pid].xyz
        a, b = ci - p, cj - p
        angles.append((180 / math.pi) * math.acos(np.clip(np.dot(a, b) / np.linalg.norm(a) / np.linalg.norm(b), -1, 1)))
    score = float(len(common))
    if angles and sorted(angles)[int(len(angles) * 0.75)] < 1:
        score = 0.0
    return score


def convert(dense_folder: str, save_folder: str, max_d: int = 192, interval_scale: float = 1.0,
            scale_factor: float = 1.0, model_ext: str = ".txt", write_images: bool = True) -> dict:
    model_dir = os.path.join(dense_folder, "dslr_calibration_undistorted")
    image_dir = os.path.join(dense_folder, "images")
    cam_dir = os.path.join(save_folder, "cams")
    out_img = os.path.join(save_folder, "images")
    for d in (out_img, cam_dir):
        if os.path.exists(d):
            shutil.rmtree(d)
    os.makedirs(out_img)
    os.makedirs(cam_dir)
    cameras, images, points3d = read_model(model_dir, model_ext)
    intrinsic = {}
    for cid, cam in cameras.items():
        p = dict(zip(PARAM_NAMES[cam.model], cam.params))
        if "f" in p:
            p["fx"] = p["fy"] = p["f"]
        intrinsic[cid] = np.array([[p["fx"] / scale_factor, 0, p["cx"] / scale_factor],
                                   [0, p["fy"] / scale_factor, p["cy"] / scale_factor], [0, 0, 1]])
    images = {k + 1: images[iid] for k, iid in enumerate(sorted(images))}
    n = len(images)
    extrinsic = {}
    for k, img in images.items():
        e = np.zeros((4, 4))
        e[:3, :3] = qvec2rotmat(img.qvec)
        e[:3, 3] = img.tvec
        e[3, 3] = 1
        extrinsic[k] = e
    depth_ranges = {}
    for k in range(1, n + 1):
        zs = sorted(float((extrinsic[k] @ np.append(points3d[int(p)].xyz, 1.0))[2])
                    for p in images[k].point3D_ids if int(p) != -1)
        dmin = dmax = 0.0
        if zs:
            dmin = zs[int(len(zs) * .01)] * 0.75
            dmax = zs[int(len(zs) * .99)] * 1.25
        if max_d == 0:
            K = intrinsic[images[k].camera_id]
            R, t = extrinsic[k][:3, :3], extrinsic[k][:3, 3]
            P1 = np.linalg.inv(R) @ (np.linalg.inv(K) @ [K[0, 2], K[1, 2], 1] * dmin - t)
            P2 = np.linalg.inv(R) @ (np.linalg.inv(K) @ [K[0, 2] + 1, K[1, 2], 1] * dmin - t)
            depth_num = (1 / dmin - 1 / dmax) / (1 / dmin - 1 / (dmin + np.linalg.norm(P2 - P1)))
        else:
            depth_num = max_d
        depth_ranges[k] = (dmin, (dmax - dmin) / (depth_num - 1) / interval_scale, depth_num, dmax)
    score = np.zeros((n, n))
    for i in range(n):
        for j in range(i + 1, n):
            score[i, j] = score[j, i] = pair_score(i + 1, j + 1, images, points3d, extrinsic)
    num_view = min(20, n - 1)
    view_sel = [[(int(k), score[i, k]) for k in np.argsort(score[i])[::-1][:num_view]] for i in range(n)]
    for i in range(n):
        with open(os.path.join(cam_dir, "%08d_cam.txt" % i), "w") as f:
            f.write("extrinsic\n")
            for r in range(4):
                f.write("".join(str(extrinsic[i + 1][r, c]) + " " for c in range(4)) + "\n")
            f.write("\nintrinsic\n")
            K = intrinsic[images[i + 1].camera_id]
            for r in range(3):
                f.write("".join(str(K[r, c]) + " " for c in range(3)) + "\n")
            f.write("\n%f %f %f %f\n" % depth_ranges[i + 1])
    with open(os.path.join(save_folder, "pair.txt"), "w") as f:
        f.write("%d\n" % n)
        for i, sel in enumerate(view_sel):
            f.write("%d\n%d " % (i, len(sel)))
            for k, s in sel:
                f.write("%d %d " % (k, s))
            f.write("\n")
    if write_images:
        from PIL import Image as PILImage
        arrays = [np.asarray(PILImage.open(os.path.join(image_dir, images[k].name)).convert("RGB"))
                  for k in range(1, n + 1)]
        H = max(a.shape[0] for a in arrays)
        W = max(a.shape[1] for a in arrays)
        for i, a in enumerate(arrays):
            a = np.pad(a, ((0, H - a.shape[0]), (0, W - a.shape[1]), (0, 0)))
            nw, nh = int(W / scale_factor), int(H / scale_factor)
            if (nw, nh) != (W, H):   # cv2.INTER_NEAREST: source index floor(d * src / dst), clamped
                xs = np.minimum(np.floor(np.arange(nw) * (W / nw)).astype(int), W - 1)
                ys = np.minimum(np.floor(np.arange(nh) * (H / nh)).astype(int), H - 1)
                a = a[ys][:, xs]
            PILImage.fromarray(np.ascontiguousarray(a)).save(os.path.join(out_img, "%08d.jpg" % i), format="JPEG",
                                                             quality=95)
    return {"images": n, "view_sel": view_sel, "depth_ranges": depth_ranges}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Convert colmap camera")
    ap.add_argument("--dense_folder", required=True, type=str)
    ap.add_argument("--save_folder", required=True, type=str)
    ap.add_argument("--max_d", type=int, default=192)
    ap.add_argument("--interval_scale", type=float, default=1)
    ap.add_argument("--scale_factor", type=float, default=1)
    ap.add_argument("--theta0", type=float, default=5)     # accepted for compatibility (unused, as in the reference)
    ap.add_argument("--sigma1", type=float, default=1)
    ap.add_argument("--sigma2", type=float, default=10)
    ap.add_argument("--model_ext", type=str, default=".txt", choices=[".txt", ".bin"])
    a = ap.parse_args(argv)
    os.makedirs(a.save_folder, exist_ok=True)
    convert(a.dense_folder, a.save_folder, a.max_d, a.interval_scale, a.scale_factor, a.model_ext)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
