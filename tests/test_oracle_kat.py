"""Known-answer / invariant tests of the CPU restatement's primitives (oracle/oracle_math.h).

The reference ships no tests or golden vectors; these pin the restatement's
building blocks independently of the GPU: Philox4x32-10 against the published Random123 KAT
vectors, the exp/sin/cos restatements against numpy, CUDA texture semantics of the bilinear
sampler, and NCC invariants (identical views -> cost 0, flat patch -> cost 2).
"""
import math

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, synthetic


# Random123 philox4x32-10 known-answer vectors (kat_vectors: ctr, key -> output)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expect", PHILOX_KAT)
def test_philox_kat(ctr, key, expect):
    assert tuple(oracle.philox(ctr, key)) == expect


def test_expf_accuracy():
    xs = np.concatenate([np.linspace(-87, 88, 20001), np.linspace(-1, 1, 2001), [-0.18, -1.0 / 90]]).astype(np.float32)
    got = np.array([oracle.lib().oracle_expf(float(x)) for x in xs], np.float64)
    ref = np.exp(xs.astype(np.float64))
    rel = np.abs(got - ref) / ref
    assert rel.max() < 4e-7
    assert oracle.lib().oracle_expf(-200.0) == 0.0
    assert math.isinf(oracle.lib().oracle_expf(100.0))


def test_sincos_accuracy():
    xs = np.linspace(-0.2, 0.2, 4001).astype(np.float32)
    s = np.array([oracle.lib().oracle_sinf(float(x)) for x in xs])
    c = np.array([oracle.lib().oracle_cosf(float(x)) for x in xs])
    assert np.abs(s - np.sin(xs.astype(np.float64))).max() < 2e-7
    assert np.abs(c - np.cos(xs.astype(np.float64))).max() < 2e-7


def test_exp_double_accuracy():
    for x in np.linspace(-16.25, 8.75, 501):
        got = oracle.lib().oracle_exp_d(float(x))
        assert abs(got - math.exp(x)) / math.exp(x) < 1e-14


def test_bilinear_texture_semantics():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(7, 9)).astype(np.float32)
    # texel centres (tex2D(x + 0.5, y + 0.5) at integer x, y) return the texel
    for y in range(7):
        for x in range(9):
            assert oracle.sample(img, x, y) == img[y, x]
    # half-way between two texels -> their mean (weights 128/256)
    assert oracle.sample(img, 2.5, 3.0) == pytest.approx((img[3, 2] + img[3, 3]) / 2, abs=1e-5)
    # clamp addressing outside the image
    assert oracle.sample(img, -5.0, -5.0) == img[0, 0]
    assert oracle.sample(img, 100.0, 3.0) == img[3, 8]
    assert oracle.sample(img, float("nan"), 2.0) == img[2, 0]
    # weights are quantised to 1/256
    v = oracle.sample(img, 4.0 + 1.0 / 1024, 1.0)
    assert v == img[1, 4]


@pytest.fixture(scope="module")
def scene():
    return synthetic.make_scene(64, 48, 3)


def test_ncc_identical_view_is_zero(scene):
    # a source camera identical to the reference: the homography is the identity for any plane
    cams = [scene["cams"][0], scene["cams"][0]]
    imgs = [scene["images"][0], scene["images"][0]]
    p = _abi.default_params()
    inp = dict(images=imgs, cams=cams, params=p)
    c = oracle.ncc_old(inp, 30, 20, 1, (0.0, 0.0, -1.0, 5.0))
    assert c == pytest.approx(0.0, abs=1e-5)


def test_ncc_flat_patch_is_max(scene):
    cams = [scene["cams"][0], scene["cams"][1]]
    flat = np.full_like(scene["images"][0], 140.0)
    inp = dict(images=[flat, scene["images"][1]], cams=cams, params=_abi.default_params())
    assert oracle.ncc_old(inp, 30, 20, 1, (0.0, 0.0, -1.0, 5.0)) == 2.0


def test_ncc_true_plane_beats_wrong_plane(scene):
    # at a textured pixel the ground-truth plane must score better than a plane at 0.7x depth
    v0 = scene["views"][0]
    inp = dict(images=scene["images"][:2], cams=scene["cams"][:2], params=_abi.default_params())
    cam = scene["cams"][0]
    wins = 0
    pts = [(20, 30), (40, 30), (50, 20), (15, 15), (45, 40)]
    for x, y in pts:
        d = float(v0["depth"][y, x])
        n_world = v0["normals"][y, x]
        R = np.array(cam.R[:]).reshape(3, 3)
        n = R @ n_world
        K = np.array(cam.K[:]).reshape(3, 3)
        X = d * np.linalg.inv(K) @ np.array([x, y, 1.0])
        good = (*n, -float(n @ X))
        bad = (*n, -float(n @ (0.7 * X)))
        if oracle.ncc_old(inp, x, y, 1, good) < oracle.ncc_old(inp, x, y, 1, bad):
            wins += 1
    assert wins >= 4
