"""Per-function known answers for the CPU restatement (oracle/dpe_oracle.cpp), SURVEY.md §8(c)(2).

The reference cannot run here and ships no vectors (parity unpinned), so each
deterministic piece of the restatement is defended on its own: every expected value below comes
from this file -- a literal transcription of the reference's float32 expression, a float64
evaluation of the geometry it computes, or a hand-built input whose answer follows from the
reference's code -- never from the oracle.

  ComputeHomography + ComputeCorrespondingPoint  DPE.cu:453-522   (the restatement re-associates
                                                                   H = M - b g^T: bounded against
                                                                   the literal float32 sequence)
  ComputeBilateralNCCNew                         DPE.cu:557-690
  ComputeGeomConsistencyCost                     DPE.cu:915-953
  CheckerboardFilterStrong                       DPE.cu:1957-2067 (+ callers :2069-2101)
  DepthToWeak classification                     DPE.cu:2700-2745
  GetDepthandNormal                              DPE.cu:1940-1955
  LocalRefine selection / acceptance             DPE.cu:2796-2834
"""
import math

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi

f32 = np.float32


# ------------------------------------------------------------------------------ cameras
def look_at(C, O):
    z = (O - C) / np.linalg.norm(O - C)
    x = np.cross(np.array([0.0, 1.0, 0.0]), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])


def camera(K, R, t, W, H, dmin=2.0, dmax=8.0):
    c = _abi.DpeCamera()
    for i in range(9):
        c.K[i] = float(K.flat[i])
        c.R[i] = float(R.flat[i])
    for i in range(3):
        c.t[i] = float(t[i])
    Cc = -R.T @ t
    for i in range(3):
        c.c[i] = float(Cc[i])
    c.width, c.height, c.depth_min, c.depth_max = W, H, dmin, dmax
    return c


def cam_arrays(c):
    """float64 K, R, t of a DpeCamera exactly as stored (float32 values)."""
    K = np.array([c.K[i] for i in range(9)], np.float64).reshape(3, 3)
    R = np.array([c.R[i] for i in range(9)], np.float64).reshape(3, 3)
    t = np.array([c.t[i] for i in range(3)], np.float64)
    return K, R, t


def rig(rng, W=1600, H=1200, n=3):
    """Reference + n-1 source cameras on an arc around (0, 0, 5), random look-at jitter."""
    fx = 1.2 * W
    K = np.array([[fx, 0, W / 2.0], [0, fx * (1 + 0.01 * rng.standard_normal()), H / 2.0], [0, 0, 1.0]])
    O = np.array([0.0, 0.0, 5.0])
    cams = []
    for i in range(n):
        th = math.radians(0 if i == 0 else rng.uniform(-20, 20))
        C = O + 5.0 * np.array([math.sin(th), 0.3 * rng.standard_normal(), -math.cos(th)])
        R = look_at(C, O + 0.2 * rng.standard_normal(3))
        cams.append(camera(K, R, -R @ C, W, H))
    return cams


def pass_input(cams, images=None, depths=None, **params):
    W, H = cams[0].width, cams[0].height
    if images is None:
        images = [np.zeros((H, W), np.float32) for _ in cams]
    p = _abi.default_params()
    for k, v in params.items():
        setattr(p, k, v)
    return dict(images=images, cams=cams, depths=depths, params=p)


# ------------------------------------------------------------------------------ homography
def literal_homography(ref, src, plane):
    """DPE.cu:453-513, statement by statement in float32 (each operation rounded once)."""
    rR = [f32(ref.R[i]) for i in range(9)]
    rt = [f32(ref.t[i]) for i in range(3)]
    sR = [f32(src.R[i]) for i in range(9)]
    st = [f32(src.t[i]) for i in range(3)]
    rK = [f32(ref.K[i]) for i in range(9)]
    sK = [f32(src.K[i]) for i in range(9)]
    px, py, pz, pw = (f32(v) for v in plane)
    ref_C = [-(rR[0 + j] * rt[0] + rR[3 + j] * rt[1] + rR[6 + j] * rt[2]) for j in range(3)]
    src_C = [-(sR[0 + j] * st[0] + sR[3 + j] * st[1] + sR[6 + j] * st[2]) for j in range(3)]
    Rr = [sR[3 * r + 0] * rR[3 * c + 0] + sR[3 * r + 1] * rR[3 * c + 1] + sR[3 * r + 2] * rR[3 * c + 2]
          for r in range(3) for c in range(3)]
    Cr = [ref_C[j] - src_C[j] for j in range(3)]
    tr = [sR[3 * r + 0] * Cr[0] + sR[3 * r + 1] * Cr[1] + sR[3 * r + 2] * Cr[2] for r in range(3)]
    Hh = [Rr[3 * r + c] - tr[r] * (px, py, pz)[c] / pw for r in range(3) for c in range(3)]
    tmp = []
    for r in range(3):
        tmp += [Hh[3 * r] / rK[0], Hh[3 * r + 1] / rK[4],
                -Hh[3 * r] * rK[2] / rK[0] - Hh[3 * r + 1] * rK[5] / rK[4] + Hh[3 * r + 2]]
    return [sK[0] * tmp[0] + sK[2] * tmp[6], sK[0] * tmp[1] + sK[2] * tmp[7], sK[0] * tmp[2] + sK[2] * tmp[8],
            sK[4] * tmp[3] + sK[5] * tmp[6], sK[4] * tmp[4] + sK[5] * tmp[7], sK[4] * tmp[5] + sK[5] * tmp[8],
            sK[8] * tmp[6], sK[8] * tmp[7], sK[8] * tmp[8]]


def literal_point(Hm, x, y):
    """ComputeCorrespondingPoint (DPE.cu:515-522) in float32."""
    x, y = f32(x), f32(y)
    X = Hm[0] * x + Hm[1] * y + Hm[2]
    Y = Hm[3] * x + Hm[4] * y + Hm[5]
    Z = Hm[6] * x + Hm[7] * y + Hm[8]
    return float(X / Z), float(Y / Z)


def exact_point(ref, src, plane, x, y):
    """The same projection in float64 from the stored camera values: ray of (x, y) in the reference
    camera meets the plane n.X + w = 0 (reference frame), then projects into the source."""
    rK, rR, rt = cam_arrays(ref)
    sK, sR, st = cam_arrays(src)
    n, w = np.array(plane[:3], np.float64), float(plane[3])
    ray = np.linalg.solve(rK, np.array([x, y, 1.0]))
    Xr = ray * (-w / (n @ ray))
    Xw = rR.T @ (Xr - rt)
    q = sK @ (sR @ Xw + st)
    return q[0] / q[2], q[1] / q[2]


def test_homography_restatement_matches_the_literal_float_sequence():
    """The restatement builds H = M_v - b_v g^T from per-view constants computed in double and
    projects with fma and x * (1/z); DPE.cu builds H per plane in float32 and divides.  Over random
    rigs, planes and pixels both stay within float32 rounding of the exact projection, and the
    restatement is never meaningfully further from it than the reference's own sequence."""
    rng = np.random.default_rng(7)
    err_lit, err_orc, diff = [], [], []
    for trial in range(40):
        cams = rig(rng)
        inp = pass_input(cams)
        for _ in range(5):
            n = rng.standard_normal(3) * 0.3 + np.array([0.0, 0.0, -1.0])
            n /= np.linalg.norm(n)
            depth = rng.uniform(3.0, 7.0)
            plane = [float(f32(v)) for v in n] + [float(f32(-depth * n[2]))]   # passes through (0, 0, depth)
            v = int(rng.integers(1, len(cams)))
            Ho = oracle.homography(inp, v, plane)
            Hl = literal_homography(cams[0], cams[v], plane)
            for _ in range(10):
                x, y = int(rng.integers(0, 1600)), int(rng.integers(0, 1200))
                e = exact_point(cams[0], cams[v], plane, x, y)
                lp = literal_point(Hl, x, y)
                op = oracle.project(Ho, float(x), float(y))
                if not (0 <= e[0] < 1600 and 0 <= e[1] < 1200):
                    continue
                err_lit.append(math.hypot(lp[0] - e[0], lp[1] - e[1]))
                err_orc.append(math.hypot(op[0] - e[0], op[1] - e[1]))
                diff.append(math.hypot(op[0] - lp[0], op[1] - lp[1]))
    err_lit, err_orc, diff = map(np.array, (err_lit, err_orc, diff))
    assert len(diff) > 500
    # both are float32 evaluations of the same map: sub-millipixel, the restatement no worse
    assert err_lit.max() < 5e-3 and err_orc.max() < 5e-3, (err_lit.max(), err_orc.max())
    assert np.median(err_orc) <= 1.5 * np.median(err_lit) + 1e-5, (np.median(err_orc), np.median(err_lit))
    # what the re-association moves a projected tap by: far below the 1/256-px texture weight step
    assert diff.max() < 2e-3 and np.median(diff) < 2e-4, (diff.max(), np.median(diff))


def test_homography_of_identical_cameras_is_the_identity():
    rng = np.random.default_rng(3)
    cams = rig(rng, n=1)
    cams = [cams[0], cams[0]]
    inp = pass_input(cams)
    Hm = oracle.homography(inp, 1, [0.1, -0.2, -0.97, 4.0])
    assert np.allclose(Hm.reshape(3, 3) / Hm[8], np.eye(3), atol=1e-4)   # t is stored in float32: C is not exact
    for x, y in [(0, 0), (799, 600), (1599, 1199)]:
        px, py = oracle.project(Hm, float(x), float(y))
        assert abs(px - x) < 1e-3 and abs(py - y) < 1e-3


# ------------------------------------------------------------------------------ NCC-New
def _ncc_new_case(W=48, H=40, shift=0):
    """Reference image of random texture; source camera = reference camera with its principal point
    moved by `shift` px, source image = reference image moved by the same amount, so the homography
    is a pure integer translation for every plane and every inside patch matches exactly."""
    rng = np.random.default_rng(11)
    ref = rng.integers(0, 256, (H, W)).astype(np.float32)
    K = np.array([[60.0, 0, W / 2.0], [0, 60.0, H / 2.0], [0, 0, 1.0]])
    R = np.eye(3)
    t = np.zeros(3)
    K2 = K.copy()
    K2[0, 2] += shift
    c0, c1 = camera(K, R, t, W, H), camera(K2, R, t, W, H)
    src = np.zeros_like(ref)
    if shift >= 0:
        src[:, shift:] = ref[:, :W - shift]
        src[:, :shift] = ref[:, :1]
    return ref, src, c0, c1


def test_ncc_new_known_answers():
    W, H = 48, 40
    ref, src, c0, c1 = _ncc_new_case(W, H, shift=4)
    inp = pass_input([c0, c1], images=[ref, src], weak_radius=2, weak_increment=2)
    plane = [0.0, 0.0, -1.0, 5.0]
    weak = np.full((H, W), _abi.WEAK, np.uint8)
    sel = np.zeros((H, W), np.uint32)
    nb = np.full((H, W, 9, 2), -1, np.int16)
    x, y = 20, 20
    nb[y, x, 0] = (x, y)                               # k = 0: the pixel itself
    rad = np.full((H, W), 5, np.int32)                 # use_radius: the centre patch's radius map (DPE.cu:617-620)
    # identical content under the translation: every patch NCC is 0
    for k, (dx, dy) in enumerate([(6, 0), (-6, 0), (0, 6), (0, -6)], start=1):
        nb[y, x, k] = (x + dx, y + dy)
    assert oracle.ncc_new(inp, weak, sel, nb, rad, x, y, 1, plane) == 0.0
    # two neighbours projecting past the right border (x + 4 >= W): counted as cost 2 only where
    # the neighbour's own view mask selects the view (bit v - 1), skipped otherwise (DPE.cu:605-613)
    nb[y, x, 5] = (W - 2, y)
    nb[y, x, 6] = (W - 1, y + 2)
    sel[y, W - 2] = 1                                  # view 1 selected at the first one only
    got = oracle.ncc_new(inp, weak, sel, nb, rad, x, y, 1, plane)
    strong = f32(2.0) / f32(5)                         # 4 inside neighbours at 0 + one 2.0, count 5
    assert got == float(f32(0.25 * 0.0 + 0.75 * float(min(strong, f32(2.0)))))
    # the centre projecting outside: 2.0 (DPE.cu:577-579)
    assert oracle.ncc_new(inp, weak, sel, nb, rad, W - 3, y, 1, plane) == 2.0
    # not a WEAK pixel: the reference prints "error" and returns 0 (DPE.cu:685-687)
    w2 = weak.copy()
    w2[y, x] = _abi.STRONG
    assert oracle.ncc_new(inp, w2, sel, nb, rad, x, y, 1, plane) == 0.0
    # black source: every patch has variance 0 < 1e-5 -> 2 each; 0.25 * 2 + 0.75 * min(2, 2) = 2
    # (a constant grey level g > 0 need not: s_ss - s_src^2 keeps a rounding residue of order g^2 ulp)
    flat = np.zeros_like(ref)
    inp2 = pass_input([c0, c1], images=[ref, flat], weak_radius=2, weak_increment=2)
    nb2 = nb.copy()
    nb2[y, x, 5:] = -1
    assert oracle.ncc_new(inp2, weak, sel, nb2, rad, x, y, 1, plane) == 2.0
    # no support points at all: the centre cost alone
    nb3 = np.full((H, W, 9, 2), -1, np.int16)
    nb3[y, x, 0] = (x, y)
    assert oracle.ncc_new(inp2, weak, sel, nb3, rad, x, y, 1, plane) == 2.0
    assert oracle.ncc_new(inp, weak, sel, nb3, rad, x, y, 1, plane) == 0.0
    # the radius map drives the centre patch: radius 3 -> increment max(2, round(1.2)) = 2, still a
    # match; radius 0 -> a one-tap patch of zero variance -> 2 (the radius map is per pixel)
    assert oracle.ncc_new(inp, weak, sel, nb3, np.full((H, W), 3, np.int32), x, y, 1, plane) == 0.0
    assert oracle.ncc_new(inp, weak, sel, nb3, np.zeros((H, W), np.int32), x, y, 1, plane) == 2.0


# ------------------------------------------------------------------------------ geometric cost
def _geom_rig():
    W, H = 64, 48
    K = np.array([[70.0, 0, 32.0], [0, 70.0, 24.0], [0, 0, 1.0]])
    c0 = camera(K, np.eye(3), np.zeros(3), W, H)
    C1 = np.array([0.6, 0.1, 0.0])
    R1 = look_at(C1, np.array([0.0, 0.0, 5.0]))
    c1 = camera(K, R1, -R1 @ C1, W, H)
    return W, H, c0, c1


def _src_depth_of_plane(c1, W, H, plane, scale=1.0):
    """Depth map of the plane n.X + w = 0 (reference = world frame) seen by camera c1, float64."""
    K, R, t = cam_arrays(c1)
    n, w = np.array(plane[:3]), plane[3]
    Cw = -R.T @ t
    d = np.zeros((H, W), np.float32)
    for v in range(H):
        for u in range(W):
            ray_w = R.T @ np.linalg.solve(K, np.array([u, v, 1.0]))
            s = -(w + n @ Cw) / (n @ ray_w)              # X = Cw + s * ray_w
            d[v, u] = (R @ (Cw + s * ray_w) + t)[2] * scale
    return d


def src_point(c0, c1, plane, x, y):
    K0, R0, t0 = cam_arrays(c0)
    K1, R1, t1 = cam_arrays(c1)
    n, w = np.array(plane[:3]), plane[3]
    ray = np.linalg.solve(K0, np.array([x, y, 1.0]))
    q = K1 @ (R1 @ (R0.T @ (ray * (-w / (n @ ray)) - t0)) + t1)
    return q[0] / q[2], q[1] / q[2]


def expected_geom(c0, c1, dmap, plane, x, y):
    """DPE.cu:915-953 in float64: depth of the plane at (x, y), world point, projection into the
    source, the depth texel at the truncated coordinate (+0.5 texel centre), back-projection,
    reprojection into the reference, distance capped at 3."""
    K0, R0, t0 = cam_arrays(c0)
    K1, R1, t1 = cam_arrays(c1)
    n, w = np.array(plane[:3]), plane[3]
    ray = np.linalg.solve(K0, np.array([x, y, 1.0]))
    Xr = ray * (-w / (n @ ray))
    Xw = R0.T @ (Xr - t0)
    q = K1 @ (R1 @ Xw + t1)
    sx, sy = q[0] / q[2], q[1] / q[2]
    H, W = dmap.shape
    ix, iy = min(max(int(sx), 0), W - 1), min(max(int(sy), 0), H - 1)
    sd = float(dmap[iy, ix])
    if sd == 0.0:
        return 3.0
    Xs = np.linalg.solve(K1, np.array([sx, sy, 1.0])) * sd
    Xw2 = R1.T @ (Xs - t1)
    q2 = K0 @ (R0 @ Xw2 + t0)
    return min(3.0, math.hypot(x - q2[0] / q2[2], y - q2[1] / q2[2]))


def test_geometric_consistency_known_answers():
    W, H, c0, c1 = _geom_rig()
    plane = [0.0, 0.0, -1.0, 5.0]                          # Z = 5 in the reference frame
    exact = _src_depth_of_plane(c1, W, H, plane)
    # pixels whose source projection is not within 0.01 px of a texel boundary (where float32
    # rounding could pick the neighbouring depth texel)
    pts = []
    for y in range(4, H - 4, 5):
        for x in range(4, W - 4, 5):
            sx, sy = src_point(c0, c1, plane, x, y)
            if 0 <= sx < W and 0 <= sy < H and min(sx % 1, 1 - sx % 1, sy % 1, 1 - sy % 1) > 0.01:
                pts.append((x, y))
    assert len(pts) > 30
    for dmap in (exact, _src_depth_of_plane(c1, W, H, plane, 1.02)):
        inp = pass_input([c0, c1], depths=[None, dmap], geom_consistency=True)
        for x, y in pts:
            got = oracle.geom_cost(inp, x, y, 1, plane)
            want = expected_geom(c0, c1, dmap, plane, x, y)
            assert abs(got - want) < 2e-3, (x, y, got, want)
    # the exact depth map reprojects onto the pixel up to the texel truncation: below ~1 px
    inp = pass_input([c0, c1], depths=[None, exact], geom_consistency=True)
    assert max(oracle.geom_cost(inp, x, y, 1, plane) for x, y in pts) < 1.0
    # an empty source depth: the maximum cost 3 (DPE.cu:941-943)
    inp0 = pass_input([c0, c1], depths=[None, np.zeros((H, W), np.float32)], geom_consistency=True)
    assert oracle.geom_cost(inp0, 32, 24, 1, plane) == 3.0
    # a far-off source depth: capped at 3
    inpf = pass_input([c0, c1], depths=[None, exact * 4.0], geom_consistency=True)
    assert oracle.geom_cost(inpf, 32, 24, 1, plane) == 3.0


# ------------------------------------------------------------------------------ median filter
FILTER_TAPS = [   # (dx, dy, condition) in DPE.cu:1997-2055 order
    (0, -1, lambda x, y, W, H: y > 0), (0, -3, lambda x, y, W, H: y > 2), (0, -5, lambda x, y, W, H: y > 4),
    (0, 1, lambda x, y, W, H: y < H - 1), (0, 3, lambda x, y, W, H: y < H - 3), (0, 5, lambda x, y, W, H: y < H - 5),
    (-1, 0, lambda x, y, W, H: x > 0), (-3, 0, lambda x, y, W, H: x > 2), (-5, 0, lambda x, y, W, H: x > 4),
    (1, 0, lambda x, y, W, H: x < W - 1), (3, 0, lambda x, y, W, H: x < W - 3), (5, 0, lambda x, y, W, H: x < W - 5),
    (2, -1, lambda x, y, W, H: y > 0 and x < W - 2), (2, 1, lambda x, y, W, H: y < H - 1 and x < W - 2),
    (-2, -1, lambda x, y, W, H: y > 0 and x > 1), (-2, 1, lambda x, y, W, H: y < H - 1 and x > 1),
    (-1, -2, lambda x, y, W, H: x > 0 and y > 2), (1, -2, lambda x, y, W, H: x < W - 1 and y > 2),
    (-1, 2, lambda x, y, W, H: x > 0 and y < H - 2), (1, 2, lambda x, y, W, H: x < W - 1 and y < H - 2),
]


def expected_median(planes, weak, costs, x, y):
    H, W = weak.shape
    if weak[y, x] == _abi.WEAK or costs[y, x] < f32(0.001):
        return float(planes[y, x, 3])
    vals = [planes[y, x, 3]]
    for dx, dy, cond in FILTER_TAPS:
        if cond(x, y, W, H) and weak[y + dy, x + dx] == _abi.STRONG:
            vals.append(planes[y + dy, x + dx, 3])
    vals = sorted(vals)
    m = len(vals) // 2
    return float((vals[m - 1] + vals[m]) / f32(2)) if len(vals) % 2 == 0 else float(vals[m])


def test_median_filter_known_answers():
    rng = np.random.default_rng(5)
    H, W = 16, 18
    for trial in range(60):
        planes = rng.uniform(1, 9, (H, W, 4)).astype(np.float32)
        weak = rng.choice([_abi.WEAK, _abi.STRONG, _abi.UNKNOWN], (H, W), p=[0.2, 0.6, 0.2]).astype(np.uint8)
        costs = rng.choice([0.0005, 0.3], (H, W), p=[0.1, 0.9]).astype(np.float32)
        for x, y in [(8, 8), (0, 0), (1, 3), (W - 1, H - 1), (W - 3, 2), (4, H - 2), (int(rng.integers(W)), int(rng.integers(H)))]:
            assert oracle.filter_strong(planes, weak, costs, x, y) == expected_median(planes, weak, costs, x, y), (trial, x, y)
    # an all-STRONG interior neighbourhood with known values: 21 taps -> the 11th smallest
    planes = np.zeros((H, W, 4), np.float32)
    x, y = 9, 8
    vals = np.arange(21, dtype=np.float32)[::-1]
    planes[y, x, 3] = vals[0]
    for (dx, dy, _), v in zip(FILTER_TAPS, vals[1:]):
        planes[y + dy, x + dx, 3] = v
    weak = np.full((H, W), _abi.STRONG, np.uint8)
    costs = np.full((H, W), 0.5, np.float32)
    assert oracle.filter_strong(planes, weak, costs, x, y) == 10.0
    weak[y - 1, x] = _abi.UNKNOWN                        # tap "up" (value 19) drops out: 20 taps
    assert oracle.filter_strong(planes, weak, costs, x, y) == 9.5


# ------------------------------------------------------------------------------ DepthToWeak classes
def curve(dips, base=1.0):
    c = np.full(61, base, np.float32)
    for i, v in dips.items():
        c[i] = v
    return c


@pytest.mark.parametrize("dips,radius,want", [
    ({}, 4, _abi.WEAK),                                  # no local minimum: min_peak 0, far from 30
    ({30: 0.10}, 4, _abi.STRONG),                        # one peak at the centre, <= 0.15
    ({30: 0.15}, 4, _abi.STRONG),
    ({30: 0.16}, 4, _abi.WEAK),                          # one peak above 0.15
    ({30: 0.51}, 4, _abi.WEAK),                          # best peak above 0.5
    ({34: 0.10}, 4, _abi.STRONG),                        # |34 - 30| = 4 <= radius
    ({35: 0.10}, 4, _abi.WEAK),                          # off by 5 > radius 4
    ({35: 0.10}, 6, _abi.STRONG),
    ({30: 0.10, 10: 0.50}, 4, _abi.STRONG),              # var = sqrt(0.4^2) / 1 = 0.4 > 0.2
    ({30: 0.10, 10: 0.25}, 4, _abi.WEAK),                # 0.15 <= 0.2
    ({30: 0.10, 10: 0.30, 50: 0.30}, 4, _abi.WEAK),      # sqrt(0.08) / 2 = 0.141
    ({30: 0.10, 10: 0.60, 50: 0.60}, 4, _abi.STRONG),    # sqrt(0.5) / 2 = 0.354
    ({1: 0.0, 59: 0.0, 30: 0.1}, 4, _abi.STRONG),        # samples 1 and 59 are never peaks
    ({28: 0.10, 32: 0.10}, 4, _abi.WEAK),                # equal peaks: the first is the minimum, var 0
])
def test_depth_to_weak_classification(dips, radius, want):
    assert oracle.d2w_class(curve(dips), radius) == want


# ------------------------------------------------------------------------------ GetDepthandNormal
def test_get_depth_and_normal_known_answers():
    rng = np.random.default_rng(9)
    for _ in range(50):
        K = np.array([[rng.uniform(500, 2000), 0, rng.uniform(300, 900)], [0, rng.uniform(500, 2000), rng.uniform(200, 700)], [0, 0, 1.0]])
        C = rng.standard_normal(3)
        R = look_at(C, C + np.array([rng.standard_normal(), rng.standard_normal(), 5.0]))
        cam = camera(K, R, -R @ C, 1600, 1200)
        Kf, Rf, _ = cam_arrays(cam)
        n = np.array([rng.standard_normal() * 0.3, rng.standard_normal() * 0.3, -1.0])
        n /= np.linalg.norm(n)
        w = rng.uniform(2, 8)
        plane = [float(f32(v)) for v in n] + [float(f32(w))]
        x, y = int(rng.integers(0, 1600)), int(rng.integers(0, 1200))
        got = oracle.depth_normal(cam, plane, x, y)
        ray = np.array([(x - Kf[0, 2]) / Kf[0, 0], (y - Kf[1, 2]) / Kf[1, 1], 1.0])
        depth = -plane[3] / (np.array(plane[:3]) @ ray)        # the ray's z where n.X + w = 0
        assert abs(got[3] - depth) <= 1e-5 * abs(depth) + 1e-6, (got[3], depth)
        assert np.allclose(got[:3], Rf.T @ np.array(plane[:3]), atol=1e-6)   # world-frame normal


# ------------------------------------------------------------------------------ LocalRefine
def test_local_refine_selection_known_answers():
    d = [float(f32(3.0 + 0.1 * k)) for k in range(11)]
    ok = [1] * 11
    tc = [1.0] * 11
    tc[3] = 0.7
    assert oracle.local_refine_select(tc, ok, d, 1.0, 9.0) == (True, d[3])         # improves by 0.3
    tc[7] = 0.7
    assert oracle.local_refine_select(tc, ok, d, 1.0, 9.0) == (True, d[3])         # ties: the first
    ok2 = list(ok)
    ok2[3] = 0
    assert oracle.local_refine_select(tc, ok2, d, 1.0, 9.0) == (True, d[7])        # out-of-range skipped
    # acceptance is strict and in double of the float difference (DPE.cu:2832)
    cost_now = float(f32(0.8))
    tc2 = [float(f32(0.7))] * 11
    diff = float(f32(cost_now) - f32(tc2[0]))
    assert oracle.local_refine_select(tc2, ok, d, cost_now, 9.0)[0] == (diff > 0.1)
    assert oracle.local_refine_select([0.95] * 11, ok, d, 1.0, 9.0)[0] is False    # 0.05 <= 0.1
    # no hypothesis in range: min_cost stays 2, best depth stays the current one
    acc, dep = oracle.local_refine_select([0.1] * 11, [0] * 11, d, 2.5, 9.0)
    assert (acc, dep) == (True, 9.0)
    assert oracle.local_refine_select([0.1] * 11, [0] * 11, d, 2.05, 9.0)[0] is False


# ------------------------------------------------------------------------------ NCC-Old (strong cost)
def literal_tex2d(img, x, y):
    """tex2D<float>(img, x, y) with cudaFilterModeLinear, cudaAddressModeClamp and unnormalised
    coordinates (DPE.cpp:919-935), as the CUDA programming guide's "Linear Filtering" appendix
    specifies it: x_B = x - 0.5, i = floor(x_B), alpha = frac(x_B) held with 8 fractional bits
    (taken here as round-to-nearest of 256 x_B), clamp addressing, then
    (1-a)(1-b) T[i,j] + a(1-b) T[i+1,j] + (1-a) b T[i,j+1] + a b T[i+1,j+1]."""
    H, W = img.shape
    xb = f32(f32(x) - f32(0.5))
    yb = f32(f32(y) - f32(0.5))
    ux = math.floor(float(xb) * 256.0 + 0.5)
    uy = math.floor(float(yb) * 256.0 + 0.5)
    i, j = ux >> 8, uy >> 8
    a, b = (ux & 255) / 256.0, (uy & 255) / 256.0
    ci = lambda v, n: min(max(v, 0), n - 1)   # noqa: E731
    t00, t10 = float(img[ci(j, H), ci(i, W)]), float(img[ci(j, H), ci(i + 1, W)])
    t01, t11 = float(img[ci(j + 1, H), ci(i, W)]), float(img[ci(j + 1, H), ci(i + 1, W)])
    return f32((1 - a) * (1 - b) * t00 + a * (1 - b) * t10 + (1 - a) * b * t01 + a * b * t11)


def _literal_point_fn(ref, src, plane):
    Hm = literal_homography(ref, src, plane)

    def point(x, y):
        x, y = f32(x), f32(y)
        X = Hm[0] * x + Hm[1] * y + Hm[2]
        Y = Hm[3] * x + Hm[4] * y + Hm[5]
        Z = Hm[6] * x + Hm[7] * y + Hm[8]
        return X / Z, Y / Z
    return point


def _literal_patch(ref_img, src_img, point, cx, cy, center, radius, increment, ss, sc):
    """One bilateral patch NCC (the body shared by DPE.cu:715-775 and :609-668) in float32."""
    cost_max = f32(2.0)
    ss, sc = f32(ss), f32(sc)
    s_ref = s_rr = s_src = s_ss = s_rs = s_w = f32(0)
    for i in range(-radius, radius + 1, increment):
        r_ref = r_rr = r_src = r_ss = r_rs = r_w = f32(0)
        for j in range(-radius, radius + 1, increment):
            rx, ry = cx + i, cy + j
            rp = literal_tex2d(ref_img, f32(rx) + f32(0.5), f32(ry) + f32(0.5))
            sx, sy = point(rx, ry)
            sp = literal_tex2d(src_img, sx + f32(0.5), sy + f32(0.5))
            sd = f32(math.sqrt(float(f32(i) * f32(i) + f32(j) * f32(j))))
            w = f32(np.exp(-sd / (f32(2.0) * ss * ss) - abs(rp - center) / (f32(2.0) * sc * sc)))
            r_ref += w * rp
            r_rr += w * rp * rp
            r_src += w * sp
            r_ss += w * sp * sp
            r_rs += w * rp * sp
            r_w += w
        s_ref += r_ref; s_rr += r_rr; s_src += r_src; s_ss += r_ss; s_rs += r_rs; s_w += r_w
    inv = f32(1.0) / s_w
    s_ref *= inv; s_rr *= inv; s_src *= inv; s_ss *= inv; s_rs *= inv
    var_ref = s_rr - s_ref * s_ref
    var_src = s_ss - s_src * s_src
    if var_ref < f32(1e-5) or var_src < f32(1e-5):
        return cost_max
    cov = s_rs - s_ref * s_src
    vrs = f32(math.sqrt(float(var_ref * var_src)))
    return max(f32(0), min(cost_max, f32(1.0) - cov / vrs))


def literal_ncc_old(ref_img, src_img, ref, src, plane, px, py, radius=5, increment=2, ss=5.0, sc=3.0):
    """ComputeBilateralNCCOld + ComputeBilateralWeight (DPE.cu:550-555, 692-778) statement by
    statement in float32 (each operation rounded once), the homography and projection of
    DPE.cu:453-522 (literal_homography / literal_point's expressions) and literal_tex2d.

    Deviation from the reference's arithmetic, stated: the reference is built --use_fast_math
    (CMakeLists.txt:72, 113), i.e. approximate division, __expf and flush-to-zero; this
    transcription uses IEEE division and np.exp, and the texture unit's 8-fractional-bit rounding
    is taken as round-to-nearest.  The 1/256 tap-coordinate rounding of restatement choice 7 is
    therefore not pinned by any reference fixture; tests/test_literal_drift.py measures what choices
    3 and 7 move over whole passes, with a * (1 / b) as a model of the approximate division."""
    point = _literal_point_fn(ref, src, plane)
    ptx, pty = point(px, py)
    if ptx >= src.width or ptx < 0 or pty >= src.height or pty < 0:
        return 2.0
    center = literal_tex2d(ref_img, f32(px) + f32(0.5), f32(py) + f32(0.5))
    return float(_literal_patch(ref_img, src_img, point, px, py, center, radius, increment, ss, sc))


def literal_ncc_new(ref_img, src_img, ref, src, plane, px, py, neighbours, sel, radius_map, view,
                    strong_radius=5, strong_increment=2, weak_radius=5, weak_increment=5, ss=5.0, sc=3.0,
                    use_radius=True):
    """ComputeBilateralNCCNew (DPE.cu:557-690) of a WEAK pixel, literal float32 (the centre patch
    k = 0 and the deformable neighbours k = 1..8; 0.25 centre + 0.75 mean of the neighbours)."""
    point = _literal_point_fn(ref, src, plane)
    W, H = ref.width, ref.height
    ptx, pty = point(px, py)
    if ptx >= src.width or ptx < 0 or pty >= src.height or pty < 0:
        return 2.0
    center = literal_tex2d(ref_img, f32(px) + f32(0.5), f32(py) + f32(0.5))
    center_cost, strong_cost, strong_count = f32(0), f32(0), 0
    for k in range(9):
        nx, ny = int(neighbours[k][0]), int(neighbours[k][1])
        if nx == -1 or ny == -1:
            continue
        nsx, nsy = point(nx, ny)
        if nsx < 0 or nsy < 0 or nsx >= W or nsy >= H:
            if k != 0:
                if (int(sel[ny, nx]) >> (view - 1)) & 1:
                    strong_cost += f32(2.0)
                    strong_count += 1
                continue
            return 2.0
        radius = strong_radius if k == 0 else weak_radius
        increment = strong_increment if k == 0 else weak_increment
        if use_radius and k == 0:
            radius = int(radius_map[py, px])
            increment = max(2, int(2.0 * radius / 5.0))
        tc = _literal_patch(ref_img, src_img, point, nx, ny, center, radius, increment, ss, sc)
        if k == 0:
            center_cost = tc
        else:
            strong_cost += tc
            strong_count += 1
    if strong_count == 0:
        return float(center_cost)
    strong_cost = strong_cost / f32(strong_count)
    strong_cost = min(strong_cost, f32(2.0))
    return float(f32(0.25 * float(center_cost) + 0.75 * float(strong_cost)))


def _textured_pair(rng, cams, plane, W, H):
    """A reference image of smooth random texture (8-bit grey levels) and a source image that is its
    warp under the true plane (float64 bilinear, rounded to 8 bits)."""
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    tex = np.zeros((H, W))
    for _ in range(6):
        fx, fy, ph = rng.uniform(0.03, 0.35), rng.uniform(0.03, 0.35), rng.uniform(0, 6.3)
        tex += rng.uniform(10, 40) * np.sin(fx * xx + fy * yy + ph)
    ref_img = np.clip(np.rint(128 + tex + rng.normal(0, 3, (H, W))), 0, 255).astype(np.float32)
    rK, rR, rt = cam_arrays(cams[0])
    sK, sR, st = cam_arrays(cams[1])
    n, w = np.array(plane[:3]), plane[3]
    # source pixel -> reference pixel through the plane (world = reference-camera frame rotated)
    src_img = np.zeros((H, W), np.float32)
    Cs = -sR.T @ st
    for v in range(H):
        rays = sR.T @ np.linalg.solve(sK, np.stack([np.arange(W), np.full(W, v), np.ones(W)]))
        # points Cs + s * ray in world; in the reference frame X_r = rR X_w + rt, on n.X_r + w = 0
        a = n @ (rR @ rays)
        b = n @ (rR @ Cs + rt) + w
        s = -b / a
        Xr = rR @ (Cs[:, None] + rays * s) + rt[:, None]
        q = rK @ Xr
        u_, v_ = q[0] / q[2], q[1] / q[2]
        u0 = np.clip(np.floor(u_).astype(int), 0, W - 1)
        v0 = np.clip(np.floor(v_).astype(int), 0, H - 1)
        u1, v1 = np.clip(u0 + 1, 0, W - 1), np.clip(v0 + 1, 0, H - 1)
        au, av = np.clip(u_ - u0, 0, 1), np.clip(v_ - v0, 0, 1)
        val = ((1 - au) * (1 - av) * ref_img[v0, u0] + au * (1 - av) * ref_img[v0, u1] +
               (1 - au) * av * ref_img[v1, u0] + au * av * ref_img[v1, u1])
        src_img[v] = np.clip(np.rint(val), 0, 255)
    return ref_img, src_img


def test_ncc_old_matches_the_literal_float_sequence():
    """The restated strong-sweep cost (oracle NCCOld: the re-associated homography, fma projection,
    the single-rounding fixed-point tap coordinate of restatement choice 7, row-major tap order) is
    within a stated bound of a literal float32 transcription of ComputeBilateralNCCOld with CUDA's
    linear-filter texture semantics, over random rigs, textures and planes at costs between the
    degenerate 0 and 2.  The two differ only where a tap coordinate sits within float32 rounding of a
    1/256-px weight step (one weight step moves that tap by (b - a) / 256 grey levels)."""
    rng = np.random.default_rng(21)
    W, H = 160, 120
    diffs, costs = [], []
    for trial in range(6):
        cams = rig(rng, W=W, H=H, n=2)
        n0 = rng.standard_normal(3) * 0.2 + np.array([0.0, 0.0, -1.0])
        n0 /= np.linalg.norm(n0)
        depth = rng.uniform(4.0, 6.0)
        true_plane = [float(f32(v)) for v in n0] + [float(f32(-depth * n0[2]))]
        ref_img, src_img = _textured_pair(rng, cams, true_plane, W, H)
        inp = pass_input(cams, images=[ref_img, src_img])
        for k in range(40):
            if k % 4 == 0:
                plane = true_plane
            else:                                          # perturbed normal / depth: intermediate costs
                n = np.array(true_plane[:3]) + rng.standard_normal(3) * 0.1 * (k % 4)
                n /= np.linalg.norm(n)
                plane = [float(f32(v)) for v in n] + [float(f32(true_plane[3] * rng.uniform(0.94, 1.06)))]
            x, y = int(rng.integers(8, W - 8)), int(rng.integers(8, H - 8))
            got = oracle.ncc_old(inp, x, y, 1, plane)
            want = literal_ncc_old(ref_img, src_img, cams[0], cams[1], plane, x, y)
            if 0.0 < want < 2.0:
                diffs.append(abs(got - want))
                costs.append(want)
    diffs, costs = np.array(diffs), np.array(costs)
    # measured (seed 21): 207 NCCs, costs median 0.09 / max 1.86; |diff| median 2.6e-6, 90th
    # percentile 1.5e-5, max 5.5e-5
    assert len(diffs) > 150 and np.median(costs) > 0.05 and costs.max() > 1.0, (len(diffs), np.median(costs))
    assert np.median(diffs) <= 1e-5, np.median(diffs)
    assert np.percentile(diffs, 90) <= 5e-5, np.percentile(diffs, 90)
    assert diffs.max() <= 2e-4, diffs.max()


def test_ncc_new_matches_the_literal_float_sequence():
    """NCC-New at non-degenerate costs: the restatement (tabulated in the weak sweep, PatchNCC in the
    oracle) against the literal float32 transcription of DPE.cu:557-690, for WEAK pixels with eight
    deformable support points (some projecting outside, with and without the view in their mask) over
    random rigs, textures and planes."""
    rng = np.random.default_rng(33)
    W, H = 160, 120
    diffs, costs = [], []
    for trial in range(4):
        cams = rig(rng, W=W, H=H, n=2)
        n0 = rng.standard_normal(3) * 0.2 + np.array([0.0, 0.0, -1.0])
        n0 /= np.linalg.norm(n0)
        depth = rng.uniform(4.0, 6.0)
        true_plane = [float(f32(v)) for v in n0] + [float(f32(-depth * n0[2]))]
        ref_img, src_img = _textured_pair(rng, cams, true_plane, W, H)
        inp = pass_input(cams, images=[ref_img, src_img], weak_radius=5, weak_increment=5)
        weak = np.full((H, W), _abi.WEAK, np.uint8)
        sel = (rng.integers(0, 2, (H, W)) * 1).astype(np.uint32)
        rad = rng.choice([3, 5, 6, 8], (H, W)).astype(np.int32)
        for k in range(12):
            x, y = int(rng.integers(12, W - 12)), int(rng.integers(12, H - 12))
            nb = np.full((H, W, 9, 2), -1, np.int16)
            nb[y, x, 0] = (x, y)
            for j in range(1, 9):
                if rng.random() < 0.85:
                    nb[y, x, j] = (int(np.clip(x + rng.integers(-30, 31), 0, W - 1)),
                                   int(np.clip(y + rng.integers(-30, 31), 0, H - 1)))
            if k % 3 == 0:
                plane = true_plane
            else:
                n = np.array(true_plane[:3]) + rng.standard_normal(3) * 0.1 * (k % 3)
                n /= np.linalg.norm(n)
                plane = [float(f32(v)) for v in n] + [float(f32(true_plane[3] * rng.uniform(0.94, 1.06)))]
            got = oracle.ncc_new(inp, weak, sel, nb, rad, x, y, 1, plane)
            want = literal_ncc_new(ref_img, src_img, cams[0], cams[1], plane, x, y, nb[y, x], sel, rad, 1)
            if 0.0 < want < 2.0:
                diffs.append(abs(got - want))
                costs.append(want)
    diffs, costs = np.array(diffs), np.array(costs)
    assert len(diffs) > 30 and np.median(costs) > 0.05 and costs.max() > 0.5, (len(diffs), np.median(costs), costs.max())
    assert np.median(diffs) <= 2e-5, np.median(diffs)
    assert diffs.max() <= 5e-4, diffs.max()


# ------------------------------------------------------------------------------ view selection
def literal_topk(costs, top_k):
    """ComputeMultiViewInitialCostandSelectedViews' selection (DPE.cu:780-826): cost vectors
    initialised { 2.0f } (element 0 only), insertion sort (sort_small, DPE.cu:5-14) of the nv costs,
    mean of the top-k valid ones, views whose cost is <= the k-th smallest."""
    nv = len(costs)
    cv = [f32(2.0)] + [f32(0.0)] * 31
    for i, c in enumerate(costs):
        cv[i] = f32(c)
    copy = list(cv)
    num_valid = sum(1 for c in costs if f32(c) < f32(2.0))
    for i in range(1, nv):                                      # sort_small
        tmp, j = cv[i], i
        while j >= 1 and tmp < cv[j - 1]:
            cv[j] = cv[j - 1]
            j -= 1
        cv[j] = tmp
    k = min(num_valid, top_k)
    if k <= 0:
        return 2.0, 0
    cost = f32(0)
    for i in range(k):
        cost += cv[i]
    thr = cv[k - 1]
    sel = 0
    for i in range(nv):
        if copy[i] <= thr:
            sel |= 1 << i
    return float(cost / f32(k)), sel


def literal_initial_cost(costs, sel):
    """ComputeMultiViewInitialCost (DPE.cu:828-857) with unSetBit's quirk (DPE.cu:77-80: the mask
    0xFFFFFFFE << n clears bits 0..n, not bit n alone)."""
    cost, count = f32(0), 0
    for i in range(1, len(costs) + 1):
        if (sel >> (i - 1)) & 1:
            c = f32(costs[i - 1])
            if c < f32(2.0):
                count += 1
                cost += c
            else:
                sel &= (0xFFFFFFFE << (i - 1)) & 0xFFFFFFFF
    return (2.0 if count == 0 else float(cost / f32(count))), sel


def test_topk_view_selection_known_answers():
    rng = np.random.default_rng(41)
    for trial in range(300):
        nv = int(rng.integers(1, 32))
        c = rng.choice([0.1, 0.25, 0.5, 2.0], nv).astype(np.float32) if trial % 3 == 0 else \
            np.where(rng.random(nv) < 0.2, 2.0, rng.uniform(0, 2, nv)).astype(np.float32)
        top_k = int(rng.integers(1, 9))
        got = oracle.topk_views(c, top_k)
        want = literal_topk(c, top_k)
        assert got[1] == want[1] and got[0] == pytest.approx(want[0], abs=0), (trial, c, top_k, got, want)
    # ties at the threshold select every tied view; invalid (2.0) views never count
    assert oracle.topk_views(np.array([0.3, 0.1, 0.3, 2.0, 0.3], np.float32), 2) == (pytest.approx(0.2), 0b10111)
    assert oracle.topk_views(np.array([2.0, 2.0], np.float32), 4) == (2.0, 0)


def test_initial_cost_unsetbit_quirk():
    rng = np.random.default_rng(43)
    for trial in range(300):
        nv = int(rng.integers(1, 32))
        c = np.where(rng.random(nv) < 0.3, 2.0, rng.uniform(0, 2, nv)).astype(np.float32)
        sel = int(rng.integers(0, 1 << nv))
        assert oracle.initial_cost(c, sel) == pytest.approx(literal_initial_cost(c, sel), abs=0), (trial, c, sel)
    # views {0, 2, 3} with view 2 invalid: bits 0..2 cleared, only view 3 stays
    got_cost, got_sel = oracle.initial_cost(np.array([0.2, 0.9, 2.0, 0.4], np.float32), 0b1101)
    assert got_sel == 0b1000 and got_cost == pytest.approx(float((f32(0.2) + f32(0.4)) / f32(2)))


def literal_view_select(cost_array, priors, it, draws):
    """The joint view selection (DPE.cu:1566-1615): per-view sampling probability from the 8
    candidates' costs, times the neighbour prior, to a CDF (TransformPDFToCDF :293-307), then 15
    draws u - FLT_EPSILON, each counted on the first view whose CDF exceeds it."""
    nv = len(priors)
    thr = f32(0.8 * float(np.exp(f32(it * it) / f32(-90.0))))
    sp = [f32(0)] * nv
    for i in range(nv):
        count, count_false, tmpw = f32(0), 0, f32(0)
        for j in range(8):
            c = f32(cost_array[j][i])
            if c < thr:
                tmpw += f32(np.exp(c * c / f32(-0.18)))
                count += f32(1)
            if c > f32(1.2):
                count_false += 1
        if count > 2 and count_false < 3:
            sp[i] = tmpw / count
        elif count_false < 3:
            sp[i] = f32(np.exp(thr * thr / f32(-0.32)))
        sp[i] = sp[i] * f32(priors[i])
    tot = f32(0)
    for i in range(nv):
        tot += sp[i]
    inv = f32(1.0) / tot
    cum = f32(0)
    cdf = []
    for i in range(nv):
        cum += sp[i] * inv
        cdf.append(cum)
    vw = [0] * nv
    margin = []
    for d in draws:
        rp = f32(d) - f32(np.finfo(np.float32).eps)
        margin.append(min(abs(float(c) - float(rp)) for c in cdf))
        for i in range(nv):
            if cdf[i] > rp:
                vw[i] += 1
                break
    return np.array(vw, np.uint8), min(margin)


def test_view_selection_known_answers():
    """Weights and the CDF sampling from a fixed uniform sequence.  Cases whose draws fall within
    1e-6 of a CDF step are skipped (the restated expf may differ from numpy's by an ulp there)."""
    rng = np.random.default_rng(47)
    checked = 0
    for trial in range(400):
        nv = int(rng.integers(2, 12))
        it = int(rng.integers(0, 4))
        ca = np.where(rng.random((8, nv)) < 0.15, rng.uniform(1.2, 2.0, (8, nv)),
                      rng.uniform(0, 1.0, (8, nv))).astype(np.float32)
        priors = rng.choice([0.0, 0.1, 0.2, 0.4, 0.9, 1.0, 1.8, 3.6], nv).astype(np.float32)
        if priors.sum() == 0:
            priors[0] = 0.9
        draws = rng.uniform(1e-6, 1.0, 15).astype(np.float32)
        want, margin = literal_view_select(ca, priors, it, draws)
        if margin < 1e-6:
            continue
        vw, tsv, wn = oracle.view_select(ca, priors, it, draws)
        assert np.array_equal(vw, want), (trial, vw, want)
        assert tsv == sum(1 << i for i in range(nv) if want[i] > 0) and wn == float(want.sum())
        checked += 1
    assert checked > 350


# ------------------------------------------------------------------------------ RANSAC plane fit
def _ransac_case(W=64, H=48, support=((20, 12), (44, 14), (32, 38)), plane=(0.1, -0.05, -1.0, 5.0)):
    K = np.array([[80.0, 0, 32.0], [0, 80.0, 24.0], [0, 0, 1.0]])
    cam = camera(K, np.eye(3), np.zeros(3), W, H, dmin=1.0, dmax=20.0)
    n = np.array(plane[:3], np.float64)
    n /= np.linalg.norm(n)
    w = plane[3]
    pl = [float(f32(v)) for v in n] + [float(f32(w))]
    planes = np.zeros((H, W, 4), np.float32)
    planes[:, :] = pl
    weak = np.full((H, W), _abi.STRONG, np.uint8)
    nb = np.full((H, W, 9, 2), -1, np.int16)
    x, y = 32, 24
    weak[y, x] = _abi.WEAK
    nb[y, x, 0] = (x, y)
    for k, (sx, sy) in enumerate(support, start=1):
        nb[y, x, k] = (sx, sy)
    return cam, planes, weak, nb, x, y, pl


def _expected_radius(A, B, C, x, y, strong_radius=5, edge_limit=False):
    """DPE.cu:3057-3110 in float64 for the winning triangle (A, B, C): the triangle's radius, capped by
    the nearest corner, rounded down to a multiple of 2.5 (the (r << 1) % 5 loop), then the
    strong-radius rule without (0 / strong) or with (max) edge_limit."""
    a, b, c = (math.dist(A, B), math.dist(B, C), math.dist(C, A))
    p = (a + b + c) / 2
    S = math.sqrt(p * (p - a) * (p - b) * (p - c))
    r = int(math.floor(math.sqrt(S) / 2.0))
    md = min(math.dist(A, (x, y)), math.dist(B, (x, y)), math.dist(C, (x, y)))
    if 2.5 * md < r:
        r = int(md)
    while (r << 1) % 5 != 0:
        r -= 1
    if not edge_limit:
        return 0 if r > strong_radius else strong_radius
    return r if r > strong_radius else strong_radius


def test_ransac_fit_known_answers():
    # three support points around the pixel, their depths on one plane: the fit is that plane (its
    # normal turned against the viewing ray), and the radius follows the triangle
    for sup, pln in [(((20, 12), (44, 14), (32, 38)), (0.1, -0.05, -1.0, 5.0)),
                     (((28, 20), (37, 21), (31, 29)), (-0.2, 0.1, -1.0, 4.0)),
                     (((2, 2), (62, 3), (30, 46)), (0.0, 0.0, 1.0, -6.0))]:
        for lim in (False, True):
            cam, planes, weak, nb, x, y, pl = _ransac_case(support=sup, plane=pln)
            inp = pass_input([cam, cam], use_limit=lim, use_edge=False, use_label=False, use_radius=True,
                             geom_consistency=False, strong_radius=5)
            fit, rad = oracle.ransac_fit(inp, planes, weak, nb, x, y)
            n = np.array(pl[:3], np.float64)
            ray = np.array([(x - 32.0) / 80.0, (y - 24.0) / 80.0, 1.0])
            sgn = -1.0 if n @ ray > 0 else 1.0            # DPE.cu:3049-3055: facing the camera
            assert np.allclose(fit[:3], sgn * n, atol=2e-5), (fit, sgn * n)
            assert abs(fit[3] - sgn * pl[3]) <= 2e-5 * abs(pl[3]) + 1e-5, (fit, pl)
            assert rad == _expected_radius(*sup, x, y, edge_limit=lim), (sup, lim, rad)
    # the pixel outside every support triangle: no plane (zeros), radius = strong_radius
    cam, planes, weak, nb, x, y, pl = _ransac_case(support=((40, 5), (60, 6), (50, 40)))
    inp = pass_input([cam, cam], use_limit=False, use_edge=False, use_label=False, use_radius=True, strong_radius=5)
    fit, rad = oracle.ransac_fit(inp, planes, weak, nb, x, y)
    assert np.all(fit == 0) and rad == 5
    # fewer than three support points: the pixel's own plane, radius untouched
    cam, planes, weak, nb, x, y, pl = _ransac_case(support=((20, 12), (44, 14)))
    planes[y, x] = (0.3, 0.2, -0.9, 7.0)
    fit, rad = oracle.ransac_fit(inp, planes, weak, nb, x, y)
    assert np.array_equal(fit, planes[y, x]) and rad == 5
