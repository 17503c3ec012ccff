"""Host pipeline (C++ libdpe_host, include/dpe_host.h): file formats, JPEG luma decode, resampling
quirks, the coarse-to-fine schedule and the multi-rank (one process per GPU) schedule.

The pass executor is injected through the C-ABI runner hook: CPU tests hand the C++ pipeline the
oracle's `oracle_pass_runner` (tests may use the oracle; the product entries -- dpe_mvs(), bin/dpe --
always use the HIP library); the GPU test runs the same pipeline on the HIP library and checks
the outputs are bit-identical.
"""
import ctypes as C
import io
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, pipeline, synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUTS = ("depth.npy", "normal.npy", "weak.npy", "edge.npy")
_THREADS = C.c_int(4)


def oracle_runner():
    fn = oracle.lib().oracle_pass_runner
    return (C.cast(fn, C.c_void_p), C.addressof(_THREADS))


def _outputs(folder, n):
    return {(i, f): np.load(os.path.join(folder, "DPE", f"{i:08d}", f)) for i in range(n) for f in OUTS}


@pytest.fixture(scope="module")
def dense4(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("dense4"))
    synthetic.write_dense_folder(d, 64, 48, 4)
    return d


def _copy(src, tmp_path, name):
    dst = str(tmp_path / name)
    shutil.copytree(src, dst)
    return dst


# ------------------------------------------------------------------------------ formats
def test_bin_mat_roundtrip(tmp_path):
    for a in (np.arange(12, dtype=np.float32).reshape(3, 4), np.arange(24, dtype=np.float32).reshape(2, 4, 3),
              np.array([[0, 1, 2]], np.uint8), np.array([[-1, 0, 7]], np.int32)):
        p = str(tmp_path / "m.dmb")
        pipeline.write_bin_mat(p, a)
        assert np.frombuffer(open(p, "rb").read()[:16], np.int32)[0] == 1
        b = pipeline.read_bin_mat(p)
        assert b.dtype == a.dtype and b.shape == a.shape and np.array_equal(a, b)


def test_camera_reader(tmp_path):
    sc = synthetic.make_scene(32, 24, 2)
    v = sc["views"][1]
    p = str(tmp_path / "c.txt")
    pipeline.write_camera(p, v["K"], v["R"], v["t"], 2.5, 9.0)
    cam = pipeline.read_camera(p)                                    # C++ ReadCamera
    assert np.allclose(np.array(cam.K[:]).reshape(3, 3), v["K"], rtol=1e-6)
    assert np.allclose(np.array(cam.R[:]).reshape(3, 3), v["R"], atol=1e-6)
    assert np.allclose(cam.c[:], v["C"], atol=1e-5)                 # c = -R^T t (DPE.cpp:363-367)
    assert cam.depth_min == pytest.approx(2.5) and cam.depth_max == pytest.approx(9.0)


def test_camera_two_number_depth_line_gives_zero_max(tmp_path):
    p = str(tmp_path / "dtu.txt")
    with open(p, "w") as f:
        f.write("extrinsic\n1 0 0 0\n0 1 0 0\n0 0 1 0\n0 0 0 1\n\nintrinsic\n100 0 50\n0 100 40\n0 0 1\n\n425 2.5\n")
    cam = pipeline.read_camera(p)
    assert cam.depth_min == 425.0 and cam.depth_max == 0.0


# ------------------------------------------------------------------------------ JPEG luma decode
def _pil_luma(buf):
    from PIL import Image
    im = Image.open(io.BytesIO(buf))
    im.draft("L", im.size)          # libjpeg JCS_GRAYSCALE output, as cv::imread(IMREAD_GRAYSCALE)
    return np.asarray(im.convert("L"))


@pytest.mark.parametrize("mode,sub,restart", [("L", None, 0), ("L", None, 3), ("RGB", 0, 0), ("RGB", 2, 0),
                                              ("RGB", 2, 5), ("RGB", 1, 0)])
def test_jpeg_luma_matches_libjpeg(tmp_path, mode, sub, restart):
    from PIL import Image
    rng = np.random.default_rng(3)
    h, w = 61, 83                                                    # not multiples of 8 / 16
    base = synthetic.make_scene(w, h, 1)["images"][0].astype(np.uint8)
    img = np.stack([base, np.roll(base, 7, 1), 255 - base], -1) if mode == "RGB" else base
    img = np.clip(img.astype(int) + rng.integers(-20, 20, img.shape), 0, 255).astype(np.uint8)
    kw = dict(format="JPEG", quality=88)
    if sub is not None:
        kw["subsampling"] = sub
    if restart:
        kw["restart_marker_blocks"] = restart
    bio = io.BytesIO()
    Image.fromarray(img, mode=mode).save(bio, **kw)
    p = str(tmp_path / "x.jpg")
    open(p, "wb").write(bio.getvalue())
    ours = pipeline.read_gray(p)
    ref = _pil_luma(bio.getvalue())
    assert ours.shape == ref.shape and np.array_equal(ours, ref)


def test_pgm_and_unsupported(tmp_path):
    p = str(tmp_path / "a.pgm")
    a = np.arange(12, dtype=np.uint8).reshape(3, 4)
    open(p, "wb").write(b"P5\n4 3\n255\n" + a.tobytes())
    assert np.array_equal(pipeline.read_gray(p), a)
    q = str(tmp_path / "b.png")
    open(q, "wb").write(b"\x89PNG....")
    with pytest.raises(pipeline.PipelineError):
        pipeline.read_gray(q)


# ------------------------------------------------------------------------------ resampling
def test_resize_linear_half_is_2x2_mean():
    img = np.random.default_rng(0).integers(0, 256, (8, 10)).astype(np.float32)
    out = pipeline.resize_linear(img, 5, 4)
    assert np.allclose(out, img.reshape(4, 2, 5, 2).mean(axis=(1, 3)), atol=1e-5)


def test_resize_linear_identity_and_border_clamp():
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    assert np.array_equal(pipeline.resize_linear(img, 4, 3), img)
    up = pipeline.resize_linear(img, 8, 6)
    assert up[0, 0] == img[0, 0] and up[-1, -1] == img[-1, -1]


def test_rescale_swapped_factors_quirk():
    # RescaleMatToTargetSize uses o_r = r / scale_x, o_c = c / scale_y (DPE.cpp:1157-1158)
    src = np.arange(6 * 4, dtype=np.int32).reshape(6, 4)
    dst = pipeline.rescale_to(src, 8, 12)                            # scale_x = scale_y = 2
    assert dst.shape == (12, 8) and dst[5, 3] == src[5 // 2, 3 // 2]
    src2 = np.arange(4 * 8, dtype=np.int32).reshape(4, 8)
    d2 = pipeline.rescale_to(src2, 16, 4)                            # scale_x = 2, scale_y = 1
    assert d2[3, 5] == src2[int(3 / 2.0), 5]
    assert d2[3, 9] == 0                                             # o_c = 9 >= cols: left unset
    n = np.arange(2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3)    # 3-channel (normals)
    assert np.array_equal(pipeline.rescale_to(n, 6, 4)[3, 5], n[1, 2])


# ------------------------------------------------------------------------------ pipeline
def test_missing_edge_map_is_regenerated(tmp_path, dense4):
    # GetProblemEdges (main.cpp:331-388): a missing edges_<s>.dmb is computed by EdgeSegment
    d = _copy(dense4, tmp_path, "noedge")
    p = os.path.join(d, "DPE", "00000000", "edges_1.dmb")
    os.remove(p)
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), verbose=False, keep_intermediate=True) == 0
    img = pipeline.read_gray(os.path.join(d, "images", "00000000.jpg"))
    half = pipeline.resize_linear(img, 32, 24)
    e = pipeline.read_bin_mat(p)
    assert np.array_equal(e, pipeline.edge_segment(1, np.rint(half).astype(np.uint8), 0, True, True))




def test_pipeline_end_to_end(tmp_path, dense4):
    d = _copy(dense4, tmp_path, "e2e")
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), normal=True, weak=True, edge=True, verbose=False,
                                     keep_intermediate=True) == 0
    out = _outputs(d, 4)
    gt = synthetic.make_scene(64, 48, 4)["views"][0]["depth"]
    dep = out[(0, "depth.npy")]
    assert dep.dtype == np.float32 and dep.shape == (48, 64)
    m = dep > 0
    assert m.mean() > 0.4
    assert np.median(np.abs(dep[m] - gt[m]) / gt[m]) < 0.03           # JPEG-decoded input, coarse-to-fine
    w = out[(0, "weak.npy")]
    assert w.dtype == np.int8 and set(np.unique(w)) <= {0, 1, 2}
    assert np.all(dep[w == 0] == 0)                                    # UNKNOWN -> depth 0
    assert out[(0, "normal.npy")].shape == (48, 64, 3)
    assert set(np.unique(out[(0, "edge.npy")])) <= {0, 1}
    dmb = pipeline.read_bin_mat(os.path.join(d, "DPE", "00000000", "depths.dmb"))
    wk = pipeline.read_bin_mat(os.path.join(d, "DPE", "00000000", "weak.bin"))
    assert np.array_equal(np.where(wk == _abi.UNKNOWN, 0, dmb), dep)


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
        assert pipeline.run_dpe_pipeline(folder, runner=oracle_runner(), normal=True, weak=True, edge=True,
                                         verbose=False, dist=dist) == 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_jacobi_matches_one_rank(tmp_path, dense4, world):
    """2 ranks split the 4 problems evenly; 3 ranks unevenly (blocks {0}, {1}, {2, 3}, so ranks 0 and
    1 pad their all-gather message to nmax = 2 maps, host/pipeline.cpp): both byte-identical to a
    1-rank Jacobi run."""
    import torch.multiprocessing as mp
    one = _copy(dense4, tmp_path, "one")
    many = _copy(dense4, tmp_path, "many")
    assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), schedule="jacobi", normal=True, weak=True,
                                     edge=True, verbose=False) == 0
    mp.start_processes(_rank_main, args=(world, _free_port(), many), nprocs=world, join=True, start_method="spawn")
    a, b = _outputs(one, 4), _outputs(many, 4)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].tobytes() == b[k].tobytes(), k


def _rank_fusion_main(rank, world, port, folder, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert pipeline.run_dpe_pipeline(folder, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(),
                                         fusion=True, normal=True, weak=True, verbose=False, dist=dist) == 0
        q.put((rank, _timings()))
    finally:
        dist.destroy_process_group()


def test_eight_ranks_sixteen_images_match_one_rank(tmp_path):
    """BASELINE configs[3]/[4]'s split at small size: 16 reference images over 8 gloo ranks (blocks of 2
    per rank, main.cpp:537-558's serial problem loop sharded), the depth maps all-gathered between the
    passes and the final normals / pixel states gathered for RunFusion on rank 0: every .npy output
    and the fused PLY byte-identical to a 1-rank Jacobi run, and every rank reporting its exchanges."""
    import torch.multiprocessing as mp
    one, many = str(tmp_path / "one"), str(tmp_path / "many")
    synthetic.write_dense_folder(one, 40, 30, 16, max_src=4)
    shutil.copytree(one, many)
    assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), fusion_runner=oracle.fusion_runner(), fusion=True,
                                     normal=True, weak=True, schedule="jacobi", verbose=False) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_rank_fusion_main, args=(8, _free_port(), many, q), nprocs=8, join=True, start_method="spawn")
    got = dict(q.get(timeout=10) for _ in range(8))
    assert sorted(got) == list(range(8))
    for rank, (n, t) in got.items():
        assert n == 8 and t[5] > 0.0 and 0.0 < t[6] <= t[3], (rank, t)
        assert t[7] > 0.0, (rank, t)   # rank 0 fuses; every rank joins the normal / state exchange before it
    outs = ("depth.npy", "normal.npy", "weak.npy")
    for i in range(16):
        for f in outs:
            a = np.load(os.path.join(one, "DPE", f"{i:08d}", f))
            b = np.load(os.path.join(many, "DPE", f"{i:08d}", f))
            assert a.dtype == b.dtype and a.tobytes() == b.tobytes(), (i, f)
    pa = open(os.path.join(one, "DPE", "DPE.ply"), "rb").read()
    assert len(pa) > 200 and pa == open(os.path.join(many, "DPE", "DPE.ply"), "rb").read()


def _timings():
    ph = (C.c_double * 8)()
    n = pipeline.lib().dpe_pipeline_last_timings(ph, 8)
    return n, [float(v) for v in ph]


def _rank_timing_main(rank, world, port, folder, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        assert pipeline.run_dpe_pipeline(folder, runner=oracle_runner(), verbose=False, dist=dist) == 0
        q.put((rank, _timings()))
    finally:
        dist.destroy_process_group()


def test_pipeline_timings_decompose(tmp_path, dense4):
    """dpe_pipeline_last_timings (bench.py's pipeline_config4/5 decomposition): 8 entries, the pass
    work and the exchanges inside the passes' share, the exchanges 0 on one rank and > 0 on each of 2
    gloo ranks, the fusion time 0 without fusion and inside the outputs phase with it."""
    import torch.multiprocessing as mp
    one = _copy(dense4, tmp_path, "t1")
    assert pipeline.run_dpe_pipeline(one, runner=oracle_runner(), verbose=False) == 0
    n, t = _timings()
    assert n == 8 and all(v >= 0.0 for v in t), t
    assert t[5] == 0.0 and 0.0 < t[6] <= t[3] <= t[0] and t[7] == 0.0, t
    two = _copy(dense4, tmp_path, "t2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_rank_timing_main, args=(2, _free_port(), two, q), nprocs=2, join=True, start_method="spawn")
    got = dict(q.get(timeout=10) for _ in range(2))
    for rank, (n, t) in got.items():
        assert n == 8 and t[5] > 0.0 and 0.0 < t[6] <= t[3] <= t[0], (rank, t)
        assert t[5] + t[6] <= t[3] * 1.05 + 1e-3, (rank, t)


def test_failed_collective_aborts_peers(tmp_path, dense4):
    """A collective that fails on this rank calls DpePipelineOptions.abort_collectives (bin/dpe passes
    ncclCommAbort) so that peers waiting in theirs fail fast, and the run reports the failure."""
    d = _copy(dense4, tmp_path, "abort")
    o = pipeline.DpePipelineOptions()
    pipeline.lib().dpe_pipeline_default_options(C.byref(o))
    o.verbose = False
    o.rank, o.world_size = 0, 2
    calls = {"allgather": 0, "abort": 0}

    def failing_allgather(_user, send, count, recv):
        calls["allgather"] += 1
        return -1

    def abort(_user):
        calls["abort"] += 1
        return 0
    ag = pipeline.ALLGATHER_FN(failing_allgather)
    ab = C.CFUNCTYPE(C.c_int, C.c_void_p)(abort)
    o.allgather = ag
    o.abort_collectives = C.cast(ab, C.c_void_p)
    runner = oracle_runner()
    o.runner = C.cast(runner[0], C.c_void_p)
    o.runner_user = C.cast(runner[1], C.c_void_p) if runner[1] is not None else None
    rc = pipeline.lib().dpe_run_pipeline(d.encode(), C.byref(o))
    assert rc != 0 and "all-gather failed" in pipeline.lib().dpe_pipeline_last_error().decode()
    assert calls["allgather"] >= 1 and calls["abort"] >= 1, calls


def _rank_fail_main(rank, world, port, folder, mode, q):
    """One rank of a 2-rank run that must fail on every rank without hanging: `mode` "one_problem"
    (world_size > problems) or "rank1_runner" (rank 1's pass runner fails in its third pass)."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    runner = oracle_runner()
    keep = None
    if mode == "rank1_runner" and rank == 1:
        base = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)(runner[0].value)
        calls = [0]

        def failing(user, inp, st):
            calls[0] += 1
            return -7 if calls[0] == 3 else base(user, inp, st)
        keep = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)(failing)
        runner = (C.cast(keep, C.c_void_p).value, runner[1])
    try:
        pipeline.run_dpe_pipeline(folder, runner=runner, verbose=False, dist=dist)
        q.put((rank, "returned 0"))
    except pipeline.PipelineError as e:
        q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["one_problem", "rank1_runner"])
def test_multi_rank_failure_ends_every_rank(tmp_path, dense4, mode):
    """A failure on one rank (or a world larger than the problem list) ends every rank with an error
    at the same collective instead of leaving the others blocked in the all-gather."""
    import torch.multiprocessing as mp
    if mode == "one_problem":
        d = str(tmp_path / "one")
        synthetic.write_dense_folder(d, 64, 48, 1)
    else:
        d = _copy(dense4, tmp_path, "fail")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_rank_fail_main, args=(2, _free_port(), d, mode, q), nprocs=2, join=True, start_method="spawn")
    got = dict(q.get(timeout=10) for _ in range(2))
    assert set(got) == {0, 1}
    if mode == "one_problem":
        assert all("exceeds" in m for m in got.values()), got
    else:
        assert "rank 1 failed" in got[0], got
        assert "PatchMatch pass failed (-7)" in got[1], got


def test_reference_schedule_reconstructs(tmp_path, dense4):
    d = _copy(dense4, tmp_path, "gs")
    assert pipeline.run_dpe_pipeline(d, runner=oracle_runner(), verbose=False) == 0
    dep = np.load(os.path.join(d, "DPE", "00000001", "depth.npy"))
    gt = synthetic.make_scene(64, 48, 4)["views"][1]["depth"]
    m = dep > 0
    assert np.median(np.abs(dep[m] - gt[m]) / gt[m]) < 0.03


def test_cli_usage():
    exe = os.path.join(ROOT, "dpe-mvs_amd", "bin", "dpe")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode != 0 and "USAGE" in r.stderr
    from DPE_MVS.__main__ import main
    assert main(["DPE"]) == 1


def test_pybind_streams_go_to_python(tmp_path, dense4, capsys):
    # the reference binding routes std::cout / std::cerr into sys.stdout / sys.stderr
    # (csrc/bindings.cpp:23-24); an unreadable image ends the run on the host, before any device work
    d = _copy(dense4, tmp_path, "broken")
    os.remove(os.path.join(d, "images", "00000002.jpg"))
    from DPE_MVS import dpe_mvs
    with pytest.raises(RuntimeError, match="Images may error"):
        dpe_mvs(d, 0, True, False, False, True, False, False, False)
    assert "Images may error, check it!" in capsys.readouterr().err


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_pybind_verbose_lines_reach_sys_stdout(tmp_path, dense4, capsys):
    # config-1-sized run through the pybind entry with verbose=True: main.cpp:489, 504's progress
    # lines and the per-iteration lines arrive on Python's sys.stdout
    a = _copy(dense4, tmp_path, "verbose")
    from DPE_MVS import dpe_mvs
    assert dpe_mvs(a, 0, True, False, False, True, False, False, False) == 0
    out = capsys.readouterr().out
    assert "There are 4 images to be processed!" in out
    assert "resolution stages for coarse-to-fine processing!" in out
    assert "Iteration 1 / 8 done" in out and "All done" in out


@pytest.mark.gpu
def test_pipeline_hip_matches_oracle(tmp_path, dense4):
    a = _copy(dense4, tmp_path, "hip")
    b = _copy(dense4, tmp_path, "cpu")
    from DPE_MVS import dpe_mvs
    assert dpe_mvs(a, 0, False, False, False, True, True, True, False) == 0              # pybind entry, HIP
    assert pipeline.run_dpe_pipeline(b, runner=oracle_runner(), normal=True, weak=True, verbose=False) == 0
    for i in range(4):
        for f in ("depth.npy", "normal.npy", "weak.npy"):
            x = np.load(os.path.join(a, "DPE", f"{i:08d}", f))
            y = np.load(os.path.join(b, "DPE", f"{i:08d}", f))
            assert x.tobytes() == y.tobytes(), (i, f)


@pytest.mark.gpu
def test_cli_runs_on_gpu(tmp_path, dense4):
    a = _copy(dense4, tmp_path, "cli")
    exe = os.path.join(ROOT, "dpe-mvs_amd", "bin", "dpe")
    r = subprocess.run([exe, a, "0", "1", "0", "0", "1", "1", "1", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert "All done" in r.stdout
    for f in OUTS:
        assert os.path.exists(os.path.join(a, "DPE", "00000003", f))


@pytest.mark.gpu
def test_gpu_torch_nccl_hooks_single_rank():
    """The torch "nccl" (RCCL) all-gather hooks that bench.py's multi-GPU pipeline lines and
    dpe_mvs(dist=...) hand the C++ pipeline: the device hook on the library's own HBM buffers and the
    host hook, called as the pipeline calls them, through a real RCCL communicator (one rank: the
    box has one GPU; the multi-rank transport is the driver's 8-GPU run)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "torch_hooks_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "HOOKS_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
