"""EdgeSegment edge/label precompute (host/edges.cpp; reference DPE.cpp:9-291, main.cpp:331-388) and the
OpenCV operations it restates (cv::Canny, cv::resize INTER_LINEAR 8U, cv::HoughLinesP, cv::line).

OpenCV is absent from this environment and the reference's tests hold no edge/label fixtures, so
agreement with OpenCV itself is parity unpinned: these tests pin each restated operation with known
answers derived by hand from the published algorithms (Sobel + squared-magnitude NMS + hysteresis,
11-bit fixed-point bilinear, the INTER_AREA fast path at exactly 1/2, cv::RNG's multiply-with-carry)."""
import os
import shutil

import numpy as np
import pytest

from DPE_MVS import pipeline, synthetic


# ------------------------------------------------------------------------------ cv::Canny
def test_canny_vertical_step_marks_left_column():
    img = np.zeros((40, 60), np.uint8)
    img[:, 30:] = 200
    e = pipeline.canny(img, 50, 100)
    assert set(np.unique(e)) == {0, 255}
    ys, xs = np.nonzero(e)
    # |gx| is 800 at x = 29 and x = 30; NMS keeps m > left && m >= right -> the left one
    assert set(xs.tolist()) == {29} and len(set(ys.tolist())) == 40


def test_canny_horizontal_step_marks_upper_row():
    img = np.zeros((40, 60), np.uint8)
    img[20:, :] = 200
    ys, xs = np.nonzero(pipeline.canny(img, 50, 100))
    assert set(ys.tolist()) == {19} and len(set(xs.tolist())) == 60


def test_canny_constant_and_threshold_order():
    assert pipeline.canny(np.full((16, 16), 77, np.uint8), 10, 20).sum() == 0
    img = np.zeros((30, 30), np.uint8)
    img[:, 15:] = 100
    assert np.array_equal(pipeline.canny(img, 100, 10), pipeline.canny(img, 10, 100))   # swapped like OpenCV


def test_canny_hysteresis_keeps_only_connected_weak_edges():
    # two vertical steps: a strong one (contrast 200) and a weak one (contrast 20) that is far away
    img = np.zeros((40, 80), np.uint8)
    img[:, 20:] = 200
    img[:, 60:] = 220
    # |gx| = 4 * 200 = 800 (strong), 4 * 20 = 80 (weak); low = 50, high = 300 (L2: squared)
    e = pipeline.canny(img, 50, 300)
    xs = set(np.nonzero(e)[1].tolist())
    assert 19 in xs and 59 not in xs
    # join the weak step to the strong one with a contrast-rich bridge row: the weak column survives
    img2 = img.copy()
    img2[10, 20:60] = 0
    e2 = pipeline.canny(img2, 50, 300)
    assert e2[:, 59].sum() > 0 or e2[:, 60].sum() > 0


# ------------------------------------------------------------------------------ cv::resize INTER_LINEAR 8U
def test_resize_half_is_area_fast_round_half_up():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (24, 32), dtype=np.uint8)
    got = pipeline.resize_u8(a, 16, 12)
    s = a.reshape(12, 2, 16, 2).astype(np.int32).sum(axis=(1, 3))
    assert np.array_equal(got, ((s + 2) >> 2).astype(np.uint8))


def test_resize_identity_and_constant_upsample():
    a = np.arange(35, dtype=np.uint8).reshape(5, 7)
    assert np.array_equal(pipeline.resize_u8(a, 7, 5), a)
    c = np.full((10, 13), 173, np.uint8)
    assert np.all(pipeline.resize_u8(c, 52, 40) == 173)


def _fixed_point_reference(a, nw, nh):
    """cv::resize INTER_LINEAR 8U restated in numpy (11-bit weights; 16/8-lane vector formula on the
    vector part of each row, (v + 2^21) >> 22 on the scalar tail)."""
    h, w = a.shape

    def tab(ns, nd):
        ofs, al = [], []
        sc = 1.0 / (nd / ns)
        xmax = nd
        for d in range(nd):
            f = np.float32((d + 0.5) * sc - 0.5)
            s = int(np.floor(f))
            f = np.float32(f - np.float32(s))
            if s < 0:
                f, s = np.float32(0), 0
            if s + 1 >= ns:
                xmax = min(xmax, d)
                if s >= ns - 1:
                    f, s = np.float32(0), ns - 1
            ofs.append(s)
            al.append((int(np.rint((np.float32(1) - f) * np.float32(2048))), int(np.rint(f * np.float32(2048)))))
        return ofs, al, xmax
    ox, ax, xmax = tab(w, nw)
    oy, ay, _ = tab(h, nh)
    rows = np.zeros((h, nw), np.int64)
    for y in range(h):
        for x in range(nw):
            s = ox[x]
            rows[y, x] = (int(a[y, s]) * ax[x][0] + int(a[y, s + 1]) * ax[x][1]) if x < xmax else int(a[y, s]) * 2048
    out = np.zeros((nh, nw), np.uint8)
    for y in range(nh):
        s0, s1 = oy[y], min(oy[y] + 1, h - 1)
        b0, b1 = ay[y]
        nvec = (nw // 16) * 16
        while nvec < nw - 8:
            nvec += 8
        for x in range(nw):
            if x < nvec:
                p0, p1 = int(rows[s0, x]) >> 4, int(rows[s1, x]) >> 4
                v = ((p0 * b0) >> 16) + ((p1 * b1) >> 16)
                out[y, x] = min(255, max(0, (v + 2) >> 2))
            else:
                out[y, x] = min(255, max(0, (int(rows[s0, x]) * b0 + int(rows[s1, x]) * b1 + (1 << 21)) >> 22))
    return out


@pytest.mark.parametrize("shape,new", [((6, 10), (40, 24)), ((7, 9), (13, 5)), ((12, 20), (27, 31))])
def test_resize_fixed_point_bilinear(shape, new):
    rng = np.random.default_rng(sum(shape) + sum(new))
    a = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(pipeline.resize_u8(a, *new), _fixed_point_reference(a, *new))


# ------------------------------------------------------------------------------ Connect
def test_connect_labels_and_counts():
    img = np.zeros((10, 12), np.uint8)
    img[:, 5] = 255                                   # a wall: two regions
    img[3, 8:] = 255                                  # the right region is cut in two again
    lab, cnt = pipeline.connect(img)
    assert np.all(lab[img == 255] == 0)
    assert cnt[0] == int((img == 255).sum())
    # left 10x5 = 50; right of the wall: rows 0-2 x cols 6-11 (18) and the L below (rows 3-9 x cols
    # 6-7 + rows 4-9 x cols 8-11 = 14 + 24), joined through cols 6-7
    assert len(cnt) == 3 and sorted(cnt[1:].tolist()) == [50, 56]
    assert lab[0, 0] == 1                             # first-seen root gets label 1
    assert len(np.unique(lab[:, :5])) == 1 and cnt[lab[0, 0]] == 50
    assert cnt[1:].sum() == (img == 0).sum()


def test_connect_u_shape_merges():
    img = np.full((6, 7), 255, np.uint8)
    img[1:5, 1] = 0
    img[1:5, 5] = 0
    img[4, 1:6] = 0                                   # U: both arms join at the bottom
    lab, cnt = pipeline.connect(img)
    assert len(cnt) == 2 and cnt[1] == (img == 0).sum()


# ------------------------------------------------------------------------------ cv::HoughLinesP
def test_hough_finds_segments():
    img = np.zeros((100, 100), np.uint8)
    img[50, 10:90] = 255
    for t in range(20, 80):
        img[t, t] = 255
    lines = pipeline.hough_lines_p(img, 1, np.pi / 180, 10, 10, 3)
    segs = {tuple(sorted([(l[0], l[1]), (l[2], l[3])])) for l in lines.tolist()}
    assert ((10, 50), (89, 50)) in segs
    assert ((20, 20), (79, 79)) in segs


def test_hough_short_segment_rejected():
    img = np.zeros((60, 60), np.uint8)
    img[30, 10:16] = 255                              # 6 px < min_len 20
    assert len(pipeline.hough_lines_p(img, 1, np.pi / 180, 3, 20, 2)) == 0


# ------------------------------------------------------------------------------ EdgeSegment
def _square(h=96, w=128, lo=60, hi=180):
    """a bright square over the middle half of the image (rows h/4..3h/4, columns w/4..3w/4)"""
    img = np.full((h, w), lo, np.uint8)
    img[h // 4:3 * h // 4, w // 4:3 * w // 4] = hi
    return img


def test_edge_segment_mode0_outlines_the_square():
    img = _square()
    e = pipeline.edge_segment(0, img, 0, True, True)
    assert e.shape == img.shape and e.dtype == np.uint8 and set(np.unique(e)) <= {0, 255}
    # the Canny thresholds come from the median (60): (0.33 * 60, 60); the square's outline is found
    assert e[26:70, 31].all() and not e[26:70, 32].any()          # left side of the step, as NMS picks
    assert e[40, 60] == 0 and e[5, 5] == 0
    assert np.array_equal(e, pipeline.canny(img, int(np.float32(1 - np.float32(0.67)) * np.float32(60)), 60))


def test_edge_segment_mode1_labels():
    img = _square(192, 256)
    lab = pipeline.edge_segment(0, img, 1, False, True)
    assert lab.shape == (192, 256) and lab.dtype == np.int32
    assert lab.min() >= -1
    inside, outside = lab[96, 128], lab[10, 10]
    assert inside > 0 and outside > 0 and inside != outside       # two large textureless regions
    lab1 = pipeline.edge_segment(1, img, 1, False, True)
    assert lab1.shape == (96, 128)


def test_edge_segment_frame_rule():
    img = np.zeros((32, 48), np.uint8)
    img[:, 24:] = 255
    e = pipeline.edge_segment(0, img, 0, True, False)
    # DPE.cpp:238-249: a frame pixel whose inner neighbour is 0 is cleared
    assert np.all(e[0, e[1, :] == 0] == 0) and np.all(e[-1, e[-2, :] == 0] == 0)
    assert np.all(e[e[:, 1] == 0, 0] == 0) and np.all(e[e[:, -2] == 0, -1] == 0)
    assert e[1:-1, 23].all()                                           # the step itself survives


def test_pipeline_generates_missing_edges_and_labels(tmp_path):
    d = str(tmp_path / "dense")
    synthetic.write_dense_folder(d, 64, 48, 3)
    for i in range(3):
        rf = os.path.join(d, "DPE", f"{i:08d}")
        for f in os.listdir(rf):
            if f.startswith(("edges_", "labels_")):
                os.remove(os.path.join(rf, f))
    import ctypes as C
    import oracle
    threads = C.c_int(4)
    runner = (C.cast(oracle.lib().oracle_pass_runner, C.c_void_p), C.addressof(threads))
    assert pipeline.run_dpe_pipeline(d, runner=runner, verbose=False, keep_intermediate=True) == 0
    img = pipeline.read_gray(os.path.join(d, "images", "00000000.jpg"))
    rf = os.path.join(d, "DPE", "00000000")
    e0 = pipeline.read_bin_mat(os.path.join(rf, "edges_0.dmb"))
    assert np.array_equal(e0, pipeline.edge_segment(0, img, 0, True, True))
    l1 = pipeline.read_bin_mat(os.path.join(rf, "labels_1.dmb"))
    assert l1.dtype == np.int32 and np.array_equal(l1, pipeline.edge_segment(1, img, 1, False, True))
    e1 = pipeline.read_bin_mat(os.path.join(rf, "edges_1.dmb"))
    assert e1.shape == (24, 32)
    dep = np.load(os.path.join(rf, "depth.npy"))
    assert dep.shape == (48, 64) and (dep > 0).mean() > 0.3
