"""EdgeSegment's data-parallel stages on the GPU (include/dpe_mvs.h dpe_canny / dpe_resize_u8 /
dpe_resize_linear / dpe_roberts_threshold, csrc/pass_edges.h) against the host restatement
(host/edges.cpp, host/hostio.cpp) that the CPU tests pin with known answers: bit-identical outputs on
the known-answer images, a 1600x1200 synthetic view (the headline size) and random images of odd
sizes; then the whole pipeline pre-pass (edges_<s>.dmb / labels_<s>.dmb written with the GPU stages)
against EdgeSegment on the host."""
import os
import time

import numpy as np
import pytest

from DPE_MVS import native, pipeline, synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = native.PatchMatchContext(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def view1600():
    return synthetic.make_scene(1600, 1200, 2)["images"][0].astype(np.uint8)


def _images(view1600):
    rng = np.random.default_rng(5)
    step = np.zeros((40, 60), np.uint8)
    step[:, 30:] = 200
    two = np.zeros((40, 80), np.uint8)
    two[:, 20:] = 200
    two[:, 60:] = 220
    bridge = two.copy()
    bridge[10, 20:60] = 0
    noise = rng.integers(0, 256, (97, 131), dtype=np.uint8)
    smooth = (128 + 60 * np.sin(np.arange(77)[:, None] / 5.0) * np.cos(np.arange(53)[None, :] / 7.0)).astype(np.uint8)
    return {"step": step, "two_steps": two, "bridge": bridge, "noise": noise, "smooth": smooth, "view1600": view1600}


@pytest.mark.parametrize("thr", [(50, 100), (100, 10), (50, 300), (20, 60), (0, 0)])
def test_canny_matches_host(ctx, view1600, thr):
    for name, img in _images(view1600).items():
        assert np.array_equal(ctx.canny(img, *thr), pipeline.canny(img, *thr)), name


def test_canny_edge_segment_thresholds_on_the_view(ctx, view1600):
    # EdgeSegment's thresholds (DPE.cpp:216-226): median of the histogram, t1 = 0.33 median
    med = int(np.searchsorted(np.cumsum(np.bincount(view1600.ravel(), minlength=256)), view1600.size // 2, side="right"))
    t1, t2 = int((1 - 0.67) * med), med
    e = ctx.canny(view1600, t1, t2)
    assert e.any() and np.array_equal(e, pipeline.canny(view1600, t1, t2))


@pytest.mark.parametrize("shape,new", [((48, 64), (32, 24)), ((1200, 1600), (800, 600)), ((600, 800), (400, 300)),
                                       ((97, 131), (200, 150)), ((97, 131), (50, 33)), ((300, 400), (1600, 1200)),
                                       ((33, 17), (17, 33))])
def test_resize_u8_matches_host(ctx, view1600, shape, new):
    rng = np.random.default_rng(shape[0] * 7 + new[0])
    img = view1600[:shape[0], :shape[1]] if shape[0] <= 1200 else rng.integers(0, 256, shape, dtype=np.uint8)
    img = np.ascontiguousarray(img)
    assert np.array_equal(ctx.resize_u8(img, *new), pipeline.resize_u8(img, *new))
    bin_img = np.where(rng.random(shape) < 0.3, 255, 0).astype(np.uint8)   # the label path resizes 0/255 maps
    assert np.array_equal(ctx.resize_u8(bin_img, *new), pipeline.resize_u8(bin_img, *new))


@pytest.mark.parametrize("new", [(800, 600), (400, 300), (1067, 800), (1600, 1200), (131, 97)])
def test_resize_linear_matches_host(ctx, view1600, new):
    img = view1600.astype(np.float32)
    a = ctx.resize_linear(img, *new)
    b = pipeline.resize_linear(img, *new)
    assert a.dtype == np.float32 and a.view(np.uint32).tobytes() == b.view(np.uint32).tobytes()


def _roberts_threshold(img, thr):   # DPE.cpp:9-25 + cv::threshold, restated in numpy
    h, w = img.shape
    t1 = np.full((h, w), 50, np.int64)
    t2 = np.full((h, w), 50, np.int64)
    s = img.astype(np.int64)
    t1[1:-1, 1:-1] = s[1:-1, 1:-1] - s[2:, 2:]
    t2[1:-1, 1:-1] = s[2:, 1:-1] - s[1:-1, 2:]
    r = np.sqrt((t1 * t1 + t2 * t2).astype(np.float64)).astype(np.int64).astype(np.uint8)
    return np.where(r > thr, 255, 0).astype(np.uint8)


@pytest.mark.parametrize("thr", [4, 6])
def test_roberts_threshold_matches_restatement(ctx, view1600, thr):
    for name, img in _images(view1600).items():
        assert np.array_equal(ctx.roberts_threshold(img, thr), _roberts_threshold(img, thr)), name


def test_pipeline_prepass_on_gpu_matches_host_edge_segment(tmp_path):
    """The native pipeline computes the missing edges_<s>.dmb / labels_<s>.dmb with the GPU stages;
    they must equal EdgeSegment on the host.  Reports the pre-pass time per image at 1600x1200."""
    d = str(tmp_path / "dense")
    synthetic.write_dense_folder(d, 1600, 1200, 3, with_edges=False)
    t0 = time.perf_counter()
    assert pipeline.run_dpe_pipeline(d, verbose=False, keep_intermediate=True, max_iterations=1) == 0
    wall = time.perf_counter() - t0
    for i in range(3):
        img = pipeline.read_gray(os.path.join(d, "images", f"{i:08d}.jpg"))
        rf = os.path.join(d, "DPE", f"{i:08d}")
        for s in (0, 1):
            e = pipeline.read_bin_mat(os.path.join(rf, f"edges_{s}.dmb"))
            if s == 0:
                ref = pipeline.edge_segment(0, img, 0, True, True)
            else:
                small = pipeline.resize_linear(img.astype(np.float32), 800, 600)
                small = np.clip(np.rint(small), 0, 255).astype(np.uint8)
                ref = pipeline.edge_segment(1, small, 0, True, True)
            assert np.array_equal(e, ref), (i, "edges", s)
            lab = pipeline.read_bin_mat(os.path.join(rf, f"labels_{s}.dmb"))
            assert np.array_equal(lab, pipeline.edge_segment(s, img, 1, False, True)), (i, "labels", s)
    print(f"pipeline with GPU pre-pass, 3 images 1600x1200, 1 iteration per pass: {wall:.2f} s")
