"""RunFusion (DPE.cpp:1220-1370) + ExportPointCloud (:532-572) and the colour decode it reads images with
(cv::imread IMREAD_COLOR, DPE.cpp:1253).

The product splits RunFusion in two: the per-(pixel, source view) projection tests (HIP kernel
dpe_fusion_candidates; on CPU the oracle's oracle_fusion_candidates) and the order-dependent rest
(host/fusion.cpp).  The oracle also restates RunFusion as the reference writes it, one serial loop
(oracle_run_fusion); the tests check the split pipeline against that loop point for point.  There
is no reference output for fusion (parity unpinned vs the CUDA/OpenCV binary)."""
import ctypes as C
import io
import os
import shutil
import socket

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, pipeline, synthetic

_THREADS = C.c_int(4)


def oracle_runner():
    return (C.cast(oracle.lib().oracle_pass_runner, C.c_void_p), C.addressof(_THREADS))


def read_ply(path):
    data = open(path, "rb").read()
    head, body = data.split(b"end_header\n", 1)
    lines = head.decode().splitlines()
    assert lines[0] == "ply" and lines[1] == "format binary_little_endian 1.0"
    n = int([l for l in lines if l.startswith("element vertex")][0].split()[-1])
    assert [l for l in lines if l.startswith("property")] == [
        "property float x", "property float y", "property float z", "property uchar diffuse_blue",
        "property uchar diffuse_green", "property uchar diffuse_red"]
    assert len(body) == 15 * n
    rec = np.frombuffer(body, dtype=np.dtype([("xyz", "<f4", 3), ("bgr", "u1", 3)]), count=n)
    return rec["xyz"].copy(), rec["bgr"].copy()


# ------------------------------------------------------------------------------ colour decode
@pytest.mark.parametrize("sub,restart,shape", [(0, 0, (61, 83)), (1, 0, (61, 83)), (2, 0, (61, 83)), (2, 4, (64, 96)),
                                               (2, 0, (17, 9)), (1, 3, (33, 50))])
def test_jpeg_colour_matches_libjpeg(tmp_path, sub, restart, shape):
    from PIL import Image
    rng = np.random.default_rng(sum(shape) + sub)
    h, w = shape
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
    img = np.clip(img + rng.integers(-30, 30, img.shape), 0, 255).astype(np.uint8)
    kw = dict(format="JPEG", quality=90, subsampling=sub)
    if restart:
        kw["restart_marker_blocks"] = restart
    bio = io.BytesIO()
    Image.fromarray(img, mode="RGB").save(bio, **kw)
    p = str(tmp_path / "c.jpg")
    open(p, "wb").write(bio.getvalue())
    ref = np.asarray(Image.open(io.BytesIO(bio.getvalue())).convert("RGB"))[..., ::-1]   # libjpeg-turbo, BGR
    ours = pipeline.read_bgr(p)
    assert ours.shape == ref.shape and np.array_equal(ours, ref)


def test_grey_jpeg_reads_as_three_equal_channels(tmp_path):
    from PIL import Image
    a = (np.arange(40 * 30) % 251).astype(np.uint8).reshape(30, 40)
    p = str(tmp_path / "g.jpg")
    Image.fromarray(a, mode="L").save(p, format="JPEG", quality=95)
    c = pipeline.read_bgr(p)
    g = pipeline.read_gray(p)
    assert np.array_equal(c[..., 0], g) and np.array_equal(c[..., 1], g) and np.array_equal(c[..., 2], g)


# ------------------------------------------------------------------------------ fusion
@pytest.fixture(scope="module")
def fused(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("fuse"))
    synthetic.write_dense_folder(d, 64, 48, 4)
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(), fusion=True,
                                     verbose=False, keep_intermediate=True) == 0
    return d


def _final_views(d, n):
    views = []
    pairs = open(os.path.join(d, "pair.txt")).read().split()
    pos, srcs = 1, {}
    for _ in range(int(pairs[0])):
        ref, k = int(pairs[pos]), int(pairs[pos + 1])
        srcs[ref] = [int(pairs[pos + 2 + 2 * q]) for q in range(k) if float(pairs[pos + 3 + 2 * q]) > 0]
        pos += 2 + 2 * k
    for i in range(n):
        rf = os.path.join(d, "DPE", f"{i:08d}")
        dep = pipeline.read_bin_mat(os.path.join(rf, "depths.dmb"))
        nrm = pipeline.read_bin_mat(os.path.join(rf, "normals.dmb"))
        wk = pipeline.read_bin_mat(os.path.join(rf, "weak.bin"))
        cam = pipeline.read_camera(os.path.join(d, "cams", f"{i:08d}_cam.txt"))
        cam.width, cam.height = dep.shape[1], dep.shape[0]
        bgr = pipeline.read_bgr(os.path.join(d, "images", f"{i:08d}.jpg"))
        views.append(dict(image_id=i, src_ids=srcs[i], cam=cam, depth=dep, normal=nrm, weak=wk, bgr=bgr, block=None))
    return views


def test_fusion_writes_ply_equal_to_serial_runfusion(fused):
    xyz, bgr = read_ply(os.path.join(fused, "DPE", "DPE.ply"))
    assert len(xyz) > 100        # strict tests (2 px, 1 %, 10 deg) on a 64x48 reconstruction
    ref = oracle.run_fusion(_final_views(fused, 4))
    assert ref.shape[0] == xyz.shape[0]
    assert np.array_equal(ref[:, :3].view(np.uint32), xyz.view(np.uint32))          # bit-identical points
    assert np.array_equal(ref[:, 3:].astype(np.uint8), bgr)                        # static_cast<uchar>


def test_fused_points_lie_on_the_scene(fused):
    xyz, _ = read_ply(os.path.join(fused, "DPE", "DPE.ply"))
    sc = synthetic.make_scene(64, 48, 4)
    v = sc["views"][0]
    K, R, t = np.array(v["K"], np.float64), np.array(v["R"], np.float64), np.array(v["t"], np.float64)
    cam = (R @ xyz.astype(np.float64).T).T + t
    uv = (K @ cam.T).T
    u, w_, z = uv[:, 0] / uv[:, 2], uv[:, 1] / uv[:, 2], cam[:, 2]
    ok = (u >= 0) & (u < 63.5) & (w_ >= 0) & (w_ < 47.5) & (z > 0)
    gt = v["depth"][np.rint(w_[ok]).astype(int), np.rint(u[ok]).astype(int)]
    rel = np.abs(z[ok] - gt) / gt
    assert ok.sum() > 50 and np.median(rel) < 0.02


def test_intermediate_maps_deleted_without_keep(tmp_path):
    d = str(tmp_path / "clean")
    synthetic.write_dense_folder(d, 64, 48, 3)
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), verbose=False) == 0     # main.cpp:581-595
    rf = os.path.join(d, "DPE", "00000000")
    assert not [f for f in os.listdir(rf) if f.startswith(("edges_", "labels_"))]
    assert os.path.exists(os.path.join(rf, "depth.npy"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, folder):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert pipeline.run_dpe_pipeline(folder, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(),
                                         fusion=True, verbose=False, dist=dist) == 0
    finally:
        dist.destroy_process_group()


def test_two_rank_fusion_matches_one_rank(tmp_path):
    import torch.multiprocessing as mp
    one, two = str(tmp_path / "one"), str(tmp_path / "two")
    synthetic.write_dense_folder(one, 64, 48, 4)
    shutil.copytree(one, two)
    assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(), fusion=True,
                                     schedule="jacobi", verbose=False) == 0
    mp.start_processes(_rank_main, args=(2, _free_port(), two), nprocs=2, join=True, start_method="spawn")
    a = open(os.path.join(one, "DPE", "DPE.ply"), "rb").read()
    b = open(os.path.join(two, "DPE", "DPE.ply"), "rb").read()
    assert a == b


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_fusion_candidates_match_oracle(fused):
    from DPE_MVS import native
    lib = native.load_library()
    views = _final_views(fused, 4)
    keep = []
    arr = (_abi.DpeFusionView * 4)() if hasattr(_abi, "DpeFusionView") else None
    assert arr is not None
    for k, v in enumerate(views):
        d, n = np.ascontiguousarray(v["depth"], np.float32), np.ascontiguousarray(v["normal"], np.float32)
        keep += [d, n]
        arr[k] = _abi.DpeFusionView(d.shape[1], d.shape[0], v["cam"], d.ctypes.data, n.ctypes.data)
    ctx = lib.dpe_create(0)
    try:
        lib.dpe_fusion_stage.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.dpe_fusion_candidates.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        assert lib.dpe_fusion_stage(ctx, arr, 4) == 0
        of = oracle.lib().oracle_fusion_candidates
        of.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        for ref in range(4):
            src = np.array([s for s in views[ref]["src_ids"]], np.int32)
            L = views[ref]["depth"].size
            gi, gv = np.empty(L * len(src), np.int32), np.empty(L * len(src) * 3, np.float32)
            ci, cv = np.empty_like(gi), np.empty_like(gv)
            assert lib.dpe_fusion_candidates(ctx, ref, src.ctypes.data, len(src), gi.ctypes.data, gv.ctypes.data) == 0
            assert of(None, arr, 4, ref, src.ctypes.data, len(src), ci.ctypes.data, cv.ctypes.data) == 0
            assert np.array_equal(gi, ci)
            m = np.repeat(gi >= 0, 3)
            assert np.array_equal(gv[m].view(np.uint32), cv[m].view(np.uint32))
            assert (gi >= 0).sum() > 100
    finally:
        lib.dpe_destroy(ctx)


@pytest.mark.gpu
def test_gpu_pipeline_fusion_ply_matches_cpu(tmp_path, fused):
    a = str(tmp_path / "hip")
    synthetic.write_dense_folder(a, 64, 48, 4)
    from DPE_MVS import dpe_mvs
    assert dpe_mvs(a, 0, False, True, False, True, False, False, False) == 0       # HIP pass + HIP fusion tests
    assert open(os.path.join(a, "DPE", "DPE.ply"), "rb").read() == open(os.path.join(fused, "DPE", "DPE.ply"), "rb").read()


@pytest.mark.gpu
def test_gpu_candidates_into_pinned_buffers(fused):
    """The host fusion pins its candidate buffers (dpe_host_pin): the copies into page-locked memory
    give the same candidates as into pageable memory, and unpinning succeeds."""
    from DPE_MVS import native
    lib = native.load_library()
    lib.dpe_host_pin.argtypes = [C.c_void_p, C.c_size_t]
    lib.dpe_host_unpin.argtypes = [C.c_void_p]
    views = _final_views(fused, 4)
    keep = []
    arr = (_abi.DpeFusionView * 4)()
    for k, v in enumerate(views):
        d, n = np.ascontiguousarray(v["depth"], np.float32), np.ascontiguousarray(v["normal"], np.float32)
        keep += [d, n]
        arr[k] = _abi.DpeFusionView(d.shape[1], d.shape[0], v["cam"], d.ctypes.data, n.ctypes.data)
    ctx = lib.dpe_create(0)
    try:
        lib.dpe_fusion_stage.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.dpe_fusion_candidates.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        assert lib.dpe_fusion_stage(ctx, arr, 4) == 0
        src = np.array(views[0]["src_ids"], np.int32)
        L = views[0]["depth"].size
        gi, gv = np.empty(L * len(src), np.int32), np.empty(L * len(src) * 3, np.float32)
        pi, pv = np.empty_like(gi), np.empty_like(gv)
        assert lib.dpe_host_pin(pi.ctypes.data, pi.nbytes) == 0 and lib.dpe_host_pin(pv.ctypes.data, pv.nbytes) == 0
        try:
            assert lib.dpe_fusion_candidates(ctx, 0, src.ctypes.data, len(src), gi.ctypes.data, gv.ctypes.data) == 0
            assert lib.dpe_fusion_candidates(ctx, 0, src.ctypes.data, len(src), pi.ctypes.data, pv.ctypes.data) == 0
            assert np.array_equal(gi, pi)
            m = np.repeat(gi >= 0, 3)
            assert np.array_equal(gv[m].view(np.uint32), pv[m].view(np.uint32))
        finally:
            assert lib.dpe_host_unpin(pi.ctypes.data) == 0 and lib.dpe_host_unpin(pv.ctypes.data) == 0
    finally:
        lib.dpe_destroy(ctx)



def test_fusion_with_block_masks_matches_serial_runfusion(tmp_path):
    """dense_folder/blocks/mask_<id>.jpg (DPE.cpp:1252-1262, 1290-1292): reference pixels whose block
    mask is < 128 are skipped.  The round-6 fusion (parallel terms, sparse serial walk) gives the
    serial restatement's points bit for bit with the masks present, and fewer points than without."""
    from PIL import Image
    d = str(tmp_path / "blk")
    synthetic.write_dense_folder(d, 64, 48, 4)
    os.makedirs(os.path.join(d, "blocks"))
    for i in range(4):
        m = np.zeros((48, 64), np.uint8)
        m[:, 16 + 6 * i:] = 255
        Image.fromarray(m, mode="L").save(os.path.join(d, "blocks", f"mask_{i}.jpg"), quality=95)
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(), fusion=True,
                                     verbose=False, keep_intermediate=True) == 0
    xyz, bgr = read_ply(os.path.join(d, "DPE", "DPE.ply"))
    views = _final_views(d, 4)
    for i, v in enumerate(views):
        v["block"] = pipeline.read_gray(os.path.join(d, "blocks", f"mask_{i}.jpg"))
    ref = oracle.run_fusion(views)
    assert ref.shape[0] == xyz.shape[0] > 0
    assert np.array_equal(ref[:, :3].view(np.uint32), xyz.view(np.uint32))
    assert np.array_equal(ref[:, 3:].astype(np.uint8), bgr)
    for v in views:
        v["block"] = None
    assert oracle.run_fusion(views).shape[0] > xyz.shape[0]
