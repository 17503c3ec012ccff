"""colmap2mvsnet (reference src/DPE_MVS/colmap2mvsnet.py:305-499): COLMAP sparse model -> dense_folder.

A COLMAP model is synthesised from the synthetic scene (cameras, poses, 3-D points sampled on the
ground-truth surfaces with their observations), written in both the text and the binary format;
the converter must read both to the same dense_folder, reproduce K / R / t, the percentile depth
ranges and the co-visibility view selection, and the result must run through the pipeline."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from DPE_MVS import colmap2mvsnet as cm, pipeline, synthetic


def rotmat2qvec(R):
    Rxx, Ryx, Rzx, Rxy, Ryy, Rzy, Rxz, Ryz, Rzz = np.asarray(R, float).flat
    K = np.array([[Rxx - Ryy - Rzz, 0, 0, 0], [Ryx + Rxy, Ryy - Rxx - Rzz, 0, 0],
                  [Rzx + Rxz, Rzy + Ryz, Rzz - Rxx - Ryy, 0], [Ryz - Rzy, Rzx - Rxz, Rxy - Ryx, Rxx + Ryy + Rzz]]) / 3.0
    vals, vecs = np.linalg.eigh(K)
    q = vecs[[3, 0, 1, 2], np.argmax(vals)]
    return -q if q[0] < 0 else q


def make_model(root, W=64, H=48, n=5, npts=400, seed=3):
    sc = synthetic.make_scene(W, H, n)
    rng = np.random.default_rng(seed)
    v0 = sc["views"][0]
    K0, R0, t0 = (np.array(v0[k], float) for k in ("K", "R", "t"))
    # 3-D points: unprojected ground-truth depths of view 0
    us, vs = rng.integers(2, W - 2, npts), rng.integers(2, H - 2, npts)
    d = v0["depth"][vs, us].astype(float)
    Xc = np.linalg.inv(K0) @ np.stack([us, vs, np.ones(npts)]) * d
    Xw = (R0.T @ (Xc - t0[:, None])).T
    obs = {i: [] for i in range(n)}
    for i, v in enumerate(sc["views"]):
        K, R, t = (np.array(v[k], float) for k in ("K", "R", "t"))
        xc = (R @ Xw.T).T + t
        uv = (K @ xc.T).T
        u, w = uv[:, 0] / uv[:, 2], uv[:, 1] / uv[:, 2]
        for p in range(npts):
            if 0 <= u[p] < W and 0 <= w[p] < H and xc[p, 2] > 0 and (i == 0 or rng.random() < 0.9 - 0.15 * i):
                obs[i].append((u[p], w[p], p + 1))
    md = os.path.join(root, "dslr_calibration_undistorted")
    os.makedirs(md, exist_ok=True)
    os.makedirs(os.path.join(root, "images"), exist_ok=True)
    from PIL import Image
    with open(os.path.join(md, "cameras.txt"), "w") as f:
        f.write("# Camera list\n")
        for i, v in enumerate(sc["views"]):
            K = np.array(v["K"], float)
            f.write(f"{i + 1} PINHOLE {W} {H} {float(K[0, 0])!r} {float(K[1, 1])!r} {float(K[0, 2])!r} {float(K[1, 2])!r}\n")
    with open(os.path.join(md, "images.txt"), "w") as f:
        f.write("# Image list\n")
        for i, v in enumerate(sc["views"]):
            q = rotmat2qvec(v["R"])
            t = np.array(v["t"], float)
            f.write(f"{10 + i} {' '.join(repr(float(x)) for x in q)} {' '.join(repr(float(x)) for x in t)} {i + 1} img_{i}.png\n")
            f.write(" ".join(f"{float(u)!r} {float(w)!r} {pid}" for u, w, pid in obs[i]) + "\n")
            Image.fromarray(v["image"].astype(np.uint8), mode="L").save(os.path.join(root, "images", f"img_{i}.png"))
    with open(os.path.join(md, "points3D.txt"), "w") as f:
        for p in range(npts):
            f.write(f"{p + 1} {float(Xw[p, 0])!r} {float(Xw[p, 1])!r} {float(Xw[p, 2])!r} 128 128 128 0.5 1 0\n")
    # the binary model of the same content
    with open(os.path.join(md, "cameras.bin"), "wb") as f:
        f.write(struct.pack("<Q", n))
        for i, v in enumerate(sc["views"]):
            K = np.array(v["K"], float)
            f.write(struct.pack("<iiQQ", i + 1, 1, W, H) + struct.pack("<4d", K[0, 0], K[1, 1], K[0, 2], K[1, 2]))
    with open(os.path.join(md, "images.bin"), "wb") as f:
        f.write(struct.pack("<Q", n))
        for i, v in enumerate(sc["views"]):
            f.write(struct.pack("<i", 10 + i) + struct.pack("<4d", *rotmat2qvec(v["R"])) +
                    struct.pack("<3d", *np.array(v["t"], float)) + struct.pack("<i", i + 1) + f"img_{i}.png".encode() + b"\0")
            f.write(struct.pack("<Q", len(obs[i])))
            for u, w, pid in obs[i]:
                f.write(struct.pack("<ddq", u, w, pid))
    with open(os.path.join(md, "points3D.bin"), "wb") as f:
        f.write(struct.pack("<Q", npts))
        for p in range(npts):
            f.write(struct.pack("<Q3d3Bd", p + 1, *Xw[p], 128, 128, 128, 0.5) + struct.pack("<Q", 1) + struct.pack("<ii", 10, 0))
    return sc, obs, Xw


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("colmap"))
    sc, obs, Xw = make_model(root)
    return root, sc, obs, Xw


def test_text_and_binary_models_give_the_same_dense_folder(model, tmp_path):
    root, sc, obs, Xw = model
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a)
    os.makedirs(b)
    cm.main(["--dense_folder", root, "--save_folder", a, "--model_ext", ".txt"])
    cm.main(["--dense_folder", root, "--save_folder", b, "--model_ext", ".bin"])
    for f in ["pair.txt"] + [os.path.join("cams", f"{i:08d}_cam.txt") for i in range(5)]:
        assert open(os.path.join(a, f)).read() == open(os.path.join(b, f)).read(), f
    for i in range(5):
        assert np.array_equal(pipeline.read_bgr(os.path.join(a, "images", f"{i:08d}.jpg")),
                              pipeline.read_bgr(os.path.join(b, "images", f"{i:08d}.jpg")))


def test_cameras_depth_ranges_and_view_selection(model, tmp_path):
    root, sc, obs, Xw = model
    out = str(tmp_path / "o")
    os.makedirs(out)
    res = cm.convert(root, out)
    for i, v in enumerate(sc["views"]):
        cam = pipeline.read_camera(os.path.join(out, "cams", f"{i:08d}_cam.txt"))
        assert np.allclose(np.array(cam.K).reshape(3, 3), np.array(v["K"], float), atol=1e-4)
        assert np.allclose(np.array(cam.R).reshape(3, 3), np.array(v["R"], float), atol=1e-6)
        assert np.allclose(np.array(cam.t), np.array(v["t"], float), atol=1e-5)
        R, t = np.array(v["R"], float), np.array(v["t"], float)
        zs = sorted(((R @ Xw[pid - 1]) + t)[2] for _, _, pid in obs[i])
        assert cam.depth_min == pytest.approx(zs[int(len(zs) * .01)] * 0.75, rel=1e-5)
        assert cam.depth_max == pytest.approx(zs[int(len(zs) * .99)] * 1.25, rel=1e-5)
    # view selection: score = co-observed points; image 0 shares the most with 1, then 2, ...
    sel0 = [k for k, s in res["view_sel"][0] if s > 0]
    common = [len(set(p for *_, p in obs[0]) & set(p for *_, p in obs[j])) for j in range(1, 5)]
    assert sel0 == [j + 1 for j in np.argsort(common)[::-1]]
    lines = open(os.path.join(out, "pair.txt")).read().split()
    assert lines[0] == "5" and lines[1] == "0" and lines[2] == "4"


def test_converted_folder_runs_through_the_pipeline(model, tmp_path):
    root, sc, obs, Xw = model
    out = str(tmp_path / "dense")
    os.makedirs(out)
    cm.convert(root, out)
    import oracle
    threads = C.c_int(4)
    runner = (C.cast(oracle.lib().oracle_pass_runner, C.c_void_p), C.addressof(threads))
    assert pipeline.run_dpe_pipeline(out, runner=runner, verbose=False) == 0
    dep = np.load(os.path.join(out, "DPE", "00000000", "depth.npy"))
    gt = sc["views"][0]["depth"]
    m = dep > 0
    assert m.mean() > 0.3 and np.median(np.abs(dep[m] - gt[m]) / gt[m]) < 0.05
