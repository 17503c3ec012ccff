"""Host pipeline (DPE_MVS.pipeline): file formats, resampling quirks, the coarse-to-fine schedule and
the multi-rank (one process per GPU) schedule.

The pass executor is injected: CPU tests use the oracle (tests are allowed to; the product entry
dpe_mvs() always uses the HIP library), the GPU test compares the HIP library with the oracle
through the whole pipeline.
"""
import os
import shutil
import socket

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, pipeline, synthetic


class OracleRunner:
    def run(self, pass_input, state):
        return oracle.run_pass(pass_input, state, threads=4)

    def close(self):
        pass


OUTS = ("depth.npy", "normal.npy", "weak.npy", "edge.npy")


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
        raw = open(p, "rb").read()
        assert np.frombuffer(raw[:16], np.int32)[0] == 1            # version
        b = pipeline.read_bin_mat(p)
        assert b.dtype == a.dtype and b.shape == a.shape and np.array_equal(a, b)


def test_bin_mat_rejects_bad_version(tmp_path):
    p = str(tmp_path / "bad.dmb")
    with open(p, "wb") as f:
        f.write(np.array([2, 1, 1, 5], np.int32).tobytes() + b"\0\0\0\0")
    with pytest.raises(pipeline.PipelineError):
        pipeline.read_bin_mat(p)


def test_camera_roundtrip_and_centre(tmp_path):
    sc = synthetic.make_scene(32, 24, 2)
    v = sc["views"][1]
    p = str(tmp_path / "c.txt")
    pipeline.write_camera(p, v["K"], v["R"], v["t"], 2.5, 9.0)
    cam = pipeline.read_camera(p)
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


def test_pair_parsing_drops_nonpositive_scores(tmp_path):
    with open(tmp_path / "pair.txt", "w") as f:
        f.write("2\n0\n3 1 10.0 2 0.0 3 -1\n1\n1 0 5.5\n")
    probs = pipeline.generate_sample_list(str(tmp_path))
    assert [p.ref_image_id for p in probs] == [0, 1]
    assert probs[0].src_image_ids == [1] and probs[1].src_image_ids == [0]
    assert os.path.isdir(tmp_path / "DPE" / "00000001")


# ------------------------------------------------------------------------------ resampling
def test_resize_linear_half_is_2x2_mean():
    img = np.random.default_rng(0).integers(0, 256, (8, 10)).astype(np.float32)
    out = pipeline.resize_linear(img, 5, 4)
    ref = img.reshape(4, 2, 5, 2).mean(axis=(1, 3))
    assert np.allclose(out, ref, atol=1e-5)


def test_resize_linear_identity_and_border_clamp():
    img = np.arange(12, dtype=np.float32).reshape(3, 4)
    assert np.array_equal(pipeline.resize_linear(img, 4, 3), img)
    up = pipeline.resize_linear(img, 8, 6)
    assert up[0, 0] == img[0, 0] and up[-1, -1] == img[-1, -1]


def test_rescale_swapped_factors_quirk():
    # RescaleMatToTargetSize uses o_r = r / scale_x, o_c = c / scale_y (DPE.cpp:1157-1158)
    src = np.arange(6 * 4, dtype=np.int32).reshape(6, 4)            # rows 6, cols 4
    dst = pipeline.rescale_to(src, 8, 12)                            # scale_x = 2, scale_y = 2
    assert dst.shape == (12, 8)
    assert dst[5, 3] == src[5 // 2, 3 // 2]
    src2 = np.arange(4 * 8, dtype=np.int32).reshape(4, 8)
    d2 = pipeline.rescale_to(src2, 16, 4)                            # scale_x = 2, scale_y = 1
    # row index divided by the x factor, column index by the y factor
    assert d2[3, 5] == src2[int(3 / 2.0), int(5 / 1.0)]
    assert d2[3, 9] == 0                                              # o_c = 9 >= cols: left unset


def test_schedule_parameters():
    p = pipeline.Problem(0, 0, [1], "", "")
    pipeline._pass_params(p, 0, -1)
    assert p.params.state == _abi.FIRST_INIT and not p.params.use_APD and not p.params.geom_consistency
    pipeline._pass_params(p, 1, -1)
    assert p.params.state == _abi.REFINE_INIT and p.params.use_edge and p.params.weak_peak_radius == 6
    assert p.params.rotate_time == 2 and p.params.ransac_threshold == pytest.approx(0.00875)
    pipeline._pass_params(p, 1, 0)
    assert p.params.state == _abi.REFINE_ITER and p.params.geom_consistency and p.params.weak_peak_radius == 4
    pipeline._pass_params(p, 2, 2)
    assert p.params.rotate_time == 4 and p.params.weak_peak_radius == 2


def test_missing_edges_is_a_clear_error(tmp_path, dense4):
    d = _copy(dense4, tmp_path, "noedge")
    os.remove(os.path.join(d, "DPE", "00000000", "edges_1.dmb"))
    with pytest.raises(pipeline.PipelineError, match="EdgeSegment"):
        pipeline.run_dpe_pipeline(d, runner=OracleRunner(), verbose=False)


def test_fusion_not_built(dense4):
    with pytest.raises(pipeline.PipelineError, match="RunFusion"):
        pipeline.run_dpe_pipeline(dense4, runner=OracleRunner(), fusion=True, verbose=False)


# ------------------------------------------------------------------------------ end to end
def test_pipeline_end_to_end(tmp_path, dense4):
    d = _copy(dense4, tmp_path, "e2e")
    assert pipeline.run_dpe_pipeline(d, runner=OracleRunner(), normal=True, weak=True, edge=True, verbose=False) == 0
    out = _outputs(d, 4)
    sc = synthetic.make_scene(64, 48, 4)
    gt = sc["views"][0]["depth"]
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
        rc = pipeline.run_dpe_pipeline(folder, runner=OracleRunner(), normal=True, weak=True, edge=True,
                                       verbose=False, dist=dist)
        assert rc == 0
    finally:
        dist.destroy_process_group()


def test_two_rank_jacobi_matches_one_rank(tmp_path, dense4):
    import torch.multiprocessing as mp
    one = _copy(dense4, tmp_path, "one")
    two = _copy(dense4, tmp_path, "two")
    assert pipeline.run_dpe_pipeline(one, runner=OracleRunner(), schedule="jacobi", normal=True, weak=True,
                                     edge=True, verbose=False) == 0
    mp.start_processes(_rank_main, args=(2, _free_port(), two), nprocs=2, join=True, start_method="spawn")
    a, b = _outputs(one, 4), _outputs(two, 4)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].tobytes() == b[k].tobytes(), k


def test_reference_schedule_differs_from_jacobi_only_by_order(tmp_path, dense4):
    # same pipeline, serial (Gauss-Seidel) order: a valid reconstruction of similar quality
    d = _copy(dense4, tmp_path, "gs")
    assert pipeline.run_dpe_pipeline(d, runner=OracleRunner(), verbose=False) == 0
    dep = np.load(os.path.join(d, "DPE", "00000001", "depth.npy"))
    gt = synthetic.make_scene(64, 48, 4)["views"][1]["depth"]
    m = dep > 0
    assert np.median(np.abs(dep[m] - gt[m]) / gt[m]) < 0.03


@pytest.mark.gpu
def test_pipeline_hip_matches_oracle(tmp_path, dense4):
    a = _copy(dense4, tmp_path, "hip")
    b = _copy(dense4, tmp_path, "cpu")
    assert pipeline.run_dpe_pipeline(a, normal=True, weak=True, verbose=False) == 0        # HIP runner
    assert pipeline.run_dpe_pipeline(b, runner=OracleRunner(), normal=True, weak=True, verbose=False) == 0
    for i in range(4):
        for f in ("depth.npy", "normal.npy", "weak.npy"):
            x = np.load(os.path.join(a, "DPE", f"{i:08d}", f))
            y = np.load(os.path.join(b, "DPE", f"{i:08d}", f))
            assert x.tobytes() == y.tobytes(), (i, f)


def test_cli_usage():
    from DPE_MVS.__main__ import main
    assert main(["DPE"]) == 1
