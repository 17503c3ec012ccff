"""Soundness of the clamp-free tap condition (round 6, `taps_unclamped` in
dpe-mvs_amd/csrc/pass_common.h): whenever it holds for a patch box, every tap's computed
t = fma(Qx, iz, kTexMagic + 1) lies strictly inside the clamp range (kTexMagic, kTexMagic + W + 1),
and likewise for y, so the skipped `v_med3_f32` would have returned t unchanged.

The condition and the taps are restated here in float32 with emulated FMAs (float64 products are
exact for float32 operands), and the tap reciprocal is taken as the correctly rounded 1/qz and both
of its float32 neighbours (v_rcp_f32 is within 1 ulp, DESIGN.md §4 choice 8).  Homographies come
from random camera pairs and planes (the plane-induced H = K2 (R - t n^T / d) K1^-1) and from
fully random matrices.  The GPU side (same bits with and without the clamps) is covered by the
`-m gpu` parity suite; this test checks the error argument itself.
"""
import numpy as np

F = np.float32
MAGIC = F(49152.0)   # kTexMagic, 1.5 * 2^15


def fma(a, b, c):
    return F(np.float64(F(a)) * np.float64(F(b)) + np.float64(F(c)))


def taps_unclamped(h, x0, x1, y0, y1, wm1, hm1):
    """pass_common.h taps_unclamped, operation for operation."""
    b0, b1 = fma(h[6], x0, h[8]), fma(h[6], x1, h[8])
    q = [fma(h[7], y0, b0), fma(h[7], y1, b0), fma(h[7], y0, b1), fma(h[7], y1, b1)]
    mn, mx = min(q), max(q)
    amax = max(abs(b0), abs(b1), abs(mn), abs(mx))
    sg = F(1.0) if mn > 0 else F(-1.0)
    lo = mn if mn > 0 else -mx
    bx = [fma(h[0], x0, h[2]), fma(h[0], x1, h[2])]
    by = [fma(h[3], x0, h[5]), fma(h[3], x1, h[5])]
    bmax = max(abs(bx[0]), abs(bx[1]), abs(by[0]), abs(by[1]))
    ok = lo >= F(amax * F(0.015625)) and bmax <= F(lo * F(65536.0))
    ys = [y0, y1]
    m = F(3.40282347e38)
    for k in range(4):
        qz = F(q[k] * sg)
        X = F(fma(h[1], ys[k & 1], bx[k >> 1]) * sg)
        Y = F(fma(h[4], ys[k & 1], by[k >> 1]) * sg)
        m = min(m, X, Y, fma(wm1, qz, -X), fma(hm1, qz, -Y))
    return bool(ok and m >= 0)


def rcp_range_ok(h, x0, x1, y0, y1):
    """pass_common.h rcp_range_ok (the condition the clamp-free test is taken under)."""
    b0, b1 = fma(h[6], x0, h[8]), fma(h[6], x1, h[8])
    q = [fma(h[7], y0, b0), fma(h[7], y1, b0), fma(h[7], y0, b1), fma(h[7], y1, b1)]
    mn, mx = min(q), max(q)
    amax = max(abs(b0), abs(b1), abs(mn), abs(mx))
    lo = mn if mn > 0 else -mx
    return bool((mn > 0 or mx < 0) and lo > amax * F(9.5367431640625e-07) and lo > F(7.888609052210118e-31)
                and amax < F(1.2676506002282294e30))


def taps_inside(h, px, py, W, H):
    """Every tap's t (with the reciprocal and its two float32 neighbours) strictly inside the range."""
    tmx, tmy = F(MAGIC + F(W + 1)), F(MAGIC + F(H + 1))
    for a in range(6):
        x = F(px - 5 + 2 * a)
        bx, by, bz = fma(h[0], x, h[2]), fma(h[3], x, h[5]), fma(h[6], x, h[8])
        for b in range(6):
            y = F(py - 5 + 2 * b)
            qx, qy, qz = fma(h[1], y, bx), fma(h[4], y, by), fma(h[7], y, bz)
            iz0 = F(F(1.0) / qz)
            for iz in (np.nextafter(iz0, F(-np.inf)), iz0, np.nextafter(iz0, F(np.inf))):
                tx, ty = fma(qx, iz, MAGIC + F(1.0)), fma(qy, iz, MAGIC + F(1.0))
                if not (MAGIC < tx < tmx and MAGIC < ty < tmy):
                    return False
    return True


def plane_homography(rng, W, H):
    f = rng.uniform(0.6, 1.6) * W
    K1 = np.array([[f, 0, W / 2 + rng.normal(0, 20)], [0, f, H / 2 + rng.normal(0, 20)], [0, 0, 1]])
    K2 = K1 * np.array([[rng.uniform(0.9, 1.1)], [rng.uniform(0.9, 1.1)], [1]])
    ang = rng.normal(0, 0.15, 3)
    th = np.linalg.norm(ang)
    k = ang / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    t = rng.normal(0, 0.3, 3)
    n = rng.normal(0, 1, 3) + np.array([0, 0, -3])
    n /= np.linalg.norm(n)
    d = rng.uniform(1.0, 20.0)
    Hm = K2 @ (R - np.outer(t, n) / d) @ np.linalg.inv(K1)
    return (Hm / Hm[2, 2] * rng.choice([1.0, -1.0, 1e-3, 1e3])).astype(np.float32).ravel()


def test_unclamped_condition_is_sound():
    rng = np.random.default_rng(7)
    hits = checked = 0
    for i in range(1500):
        W, H = [(1600, 1200), (400, 300), (2688, 1792), (48, 40)][i % 4]
        h = plane_homography(rng, W, H) if i % 5 else rng.normal(0, 1, 9).astype(np.float32) * F(10.0 ** rng.uniform(-3, 3))
        # centres anywhere, with extra weight near the borders
        px = int(rng.choice([rng.integers(0, W), rng.integers(0, 12), W - 1 - rng.integers(0, 12)]))
        py = int(rng.choice([rng.integers(0, H), rng.integers(0, 12), H - 1 - rng.integers(0, 12)]))
        x0, x1, y0, y1 = F(px - 5), F(px + 5), F(py - 5), F(py + 5)
        if not rcp_range_ok(h, x0, x1, y0, y1):
            continue
        checked += 1
        if taps_unclamped(h, x0, x1, y0, y1, F(W - 1), F(H - 1)):
            hits += 1
            assert taps_inside(h, px, py, W, H), (i, W, H, px, py, h)
    # the condition is not vacuous: it admits a good share of the realistic patches
    assert checked > 800 and hits > 200, (checked, hits)


def test_unclamped_condition_rejects_border_and_outside():
    h = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1], np.float32)   # identity: s = x
    W, H = 100, 80
    assert taps_unclamped(h, F(45), F(55), F(35), F(45), F(W - 1), F(H - 1))
    assert not taps_unclamped(h, F(-1), F(9), F(35), F(45), F(W - 1), F(H - 1))   # a tap at x = -1
    assert not taps_unclamped(h, F(90), F(100), F(35), F(45), F(W - 1), F(H - 1))  # a tap at x = 100
    assert taps_unclamped(h, F(0), F(10), F(0), F(10), F(W - 1), F(H - 1))         # exactly on the edge
    assert taps_unclamped(-h, F(45), F(55), F(35), F(45), F(W - 1), F(H - 1))      # qz < 0: the same coordinates
