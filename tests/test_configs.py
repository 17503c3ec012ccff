"""Every BASELINE.json config at its own shape (shapes table; BASELINE.json "configs").

Each config is exercised on the passes its schedule actually runs (ComputeRoundNum and the pass
parameters of main.cpp:390-408, 508-566, restated in `schedule_params` below):

  config 1  320x240, 2 views, max_iterations 1, CPU path   whole pipeline on the oracle (CPU test);
                                                           the same pipeline on HIP is bit-identical
  config 2  1600x1200, 5 src views, photometric only       FIRST_INIT / REFINE_INIT / REFINE_ITER
                                                           (geom off) at full size, HIP == oracle
  config 3  1600x1200, 9 src views, + geometric passes     the full-size REFINE_ITER + geom pass
                                                           (the bench workload), HIP == oracle
  config 4  2688x1792, 16 src views (ETH3D pair.txt <= 20) round 0 (672x448, FIRST_INIT) and round 1
                                                           (1344x896, REFINE_ITER + geom) HIP == oracle;
                                                           the full-size pass by size-independent
                                                           properties
  config 5  1920x1080, 31 src views (the reference's       round 0 (480x270) REFINE_ITER + geom
            MAX_IMAGES = 32 limit; 32 src is rejected)     HIP == oracle; the full-size pass by
                                                           properties; fusion's projection tests at
                                                           full size HIP == oracle

Tolerance: 0 (bit-identical planes, costs, weak_info, selected_views) against the scalar CPU
restatement (oracle/), whose own parity vs the CUDA reference is unpinned.
Properties at full size where the oracle would take minutes: overlapped and sequential schedules
agree bit for bit, execute is idempotent, the 6-pixel border is UNKNOWN (DepthToWeak :2599-2603),
view masks only name existing views, and the depths reconstruct the synthetic ground truth.
"""
import os
import shutil

import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, pipeline, synthetic
from golden_io import bits_equal

_SCENES = {}


def scene(W, H, N):
    """Synthetic scenes are expensive at these sizes: build each once per session; a scene with
    fewer views is the prefix of a larger one at the same size (same reference image)."""
    for (w, h, n), sc in _SCENES.items():
        if (w, h) == (W, H) and n >= N:
            return subset(sc, N)
    sc = synthetic.make_scene(W, H, N)
    _SCENES[(W, H, N)] = sc
    return sc


def subset(sc, N):
    if sc["N"] == N:
        return sc
    out = dict(sc)
    out.update(N=N, cams=sc["cams"][:N], views=sc["views"][:N], images=sc["images"][:N])
    return out


def schedule_params(i, j, photometric=False, max_iterations=3):
    """Per-pass parameters of RunDPEPipeline (main.cpp:508-566): round i, pass j (-1 = first)."""
    p = _abi.default_params()
    p.max_iterations = max_iterations
    if j < 0:
        if i == 0:
            p.state = _abi.FIRST_INIT; p.use_APD = False; p.use_edge = False
        else:
            p.state = _abi.REFINE_INIT; p.use_APD = True; p.use_edge = True
            p.ransac_threshold = 0.01 - i * 0.00125
            p.rotate_time = min(2 ** i, 4)
        p.geom_consistency = False
        p.weak_peak_radius = 6
    else:
        p.state = _abi.REFINE_ITER
        p.use_APD = i != 0; p.use_edge = i != 0
        p.ransac_threshold = 0.01 - i * 0.00125
        p.rotate_time = min(2 ** i, 4)
        p.geom_consistency = not photometric
        p.weak_peak_radius = max(4 - 2 * j, 2)
    return p


def round_num(W, H):   # ComputeRoundNum (main.cpp:390-408)
    m, r = max(W, H), 1
    while m > 800:
        m //= 2
        r += 1
    return max(r, 2)


def pass_case(W, H, N, i, j, photometric=False, seed=1):
    sc = scene(W, H, N)
    p = schedule_params(i, j, photometric)
    p.max_scale_size = 2 ** (round_num(W, H) - 1)
    p.scale_size = 1
    st = synthetic.first_init_state(sc) if p.state == _abi.FIRST_INIT else synthetic.gt_state(sc)
    depths = synthetic.src_depths(sc) if p.geom_consistency else None
    return sc, synthetic.pass_input(sc, p, depths=depths, seed=seed), st


def assert_same(g, o, what):
    for k in ("planes", "weak", "sel", "costs"):
        if not bits_equal(g[k], o[k]):
            a, b = g[k], o[k]
            neq = (a.view(np.uint32) != b.view(np.uint32)) if a.dtype == np.float32 else (a != b)
            if neq.ndim == 3:
                neq = neq.any(-1)
            ys, xs = np.nonzero(neq)
            pytest.fail(f"{what}: {k} differs at {len(ys)} pixels, first ({ys[0]}, {xs[0]})")


def check_properties(out, sc, what, n_views):
    H, W = sc["H"], sc["W"]
    planes, weak, sel = out["planes"], out["weak"], out["sel"]
    assert np.isfinite(planes).all(), what
    assert set(np.unique(weak)) <= {_abi.WEAK, _abi.STRONG, _abi.UNKNOWN}, what
    m = 6                                             # DepthToWeak's min_margin (DPE.cu:2599-2603)
    border = np.ones((H, W), bool)
    border[m:H - m, m:W - m] = False
    assert (weak[border] == _abi.UNKNOWN).all(), what
    if n_views < 32:
        assert (sel >> np.uint32(n_views) == 0).all(), what       # only existing views are selected
    gt = sc["views"][0]["depth"]
    d = planes[..., 3]
    ok = (weak == _abi.STRONG) & np.isfinite(gt)
    assert ok.mean() > 0.3, what
    rel = np.abs(d[ok] - gt[ok]) / gt[ok]
    assert np.median(rel) < 0.01, (what, float(np.median(rel)))


@pytest.fixture(scope="module")
def ctx():
    from DPE_MVS import native
    c = native.PatchMatchContext(0)
    yield c
    c.close()


def run_both(ctx, inp, st):
    return ctx.run(inp, st), oracle.run_pass(inp, st)


# ------------------------------------------------------------------------------ config 1 (CPU)
def _config1_folder(tmp_path):
    d = str(tmp_path / "cfg1")
    synthetic.write_dense_folder(d, 320, 240, 2, max_src=1)
    return d


def _oracle_runner():
    import ctypes as C
    t = C.c_int(oracle.host_threads())
    _oracle_runner.keep = t
    return (C.cast(oracle.lib().oracle_pass_runner, C.c_void_p), C.addressof(t))


def test_config1_cpu_plumbing(tmp_path):
    """Config 1: 2-view 320x240, 1 PatchMatch iteration, the whole schedule on the scalar CPU path:
    2 rounds (ComputeRoundNum's minimum) at 160x120 then 320x240, 4 passes each."""
    d = _config1_folder(tmp_path)
    assert pipeline.run_dpe_pipeline(d, runner=_oracle_runner(), normal=True, weak=True, verbose=False,
                                     max_iterations=1, keep_intermediate=True) == 0
    sc = synthetic.make_scene(320, 240, 2)
    for i in range(2):
        dep = np.load(os.path.join(d, "DPE", f"{i:08d}", "depth.npy"))
        wk = np.load(os.path.join(d, "DPE", f"{i:08d}", "weak.npy"))
        assert dep.shape == (240, 320) and dep.dtype == np.float32
        assert np.all(dep[wk == 0] == 0)
        gt = sc["views"][i]["depth"]
        m = dep > 0
        assert m.mean() > 0.3
        assert np.median(np.abs(dep[m] - gt[m]) / gt[m]) < 0.05


@pytest.mark.gpu
def test_config1_hip_pipeline_matches_cpu(tmp_path):
    a = _config1_folder(tmp_path)
    b = str(tmp_path / "cfg1_cpu")
    shutil.copytree(a, b)
    assert pipeline.run_dpe_pipeline(a, normal=True, weak=True, verbose=False, max_iterations=1) == 0
    assert pipeline.run_dpe_pipeline(b, runner=_oracle_runner(), normal=True, weak=True, verbose=False,
                                     max_iterations=1) == 0
    for i in range(2):
        for f in ("depth.npy", "normal.npy", "weak.npy"):
            x = np.load(os.path.join(a, "DPE", f"{i:08d}", f))
            y = np.load(os.path.join(b, "DPE", f"{i:08d}", f))
            assert x.tobytes() == y.tobytes(), (i, f)


# ------------------------------------------------------------------------------ config 2
@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["first_init", "refine_init", "refine_iter"])
def test_config2_photometric_full_size(ctx, kind):
    """Config 2: 5 source views, 1600x1200, photometric only (geom off on every pass)."""
    i, j = {"first_init": (0, -1), "refine_init": (1, -1), "refine_iter": (1, 0)}[kind]
    sc, inp, st = pass_case(1600, 1200, 6, i, j, photometric=True, seed=3 + j)
    assert not inp["params"].geom_consistency
    g, o = run_both(ctx, inp, st)
    assert_same(g, o, f"config2 {kind}")


# ------------------------------------------------------------------------------ config 3
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config3_full_size_geom_pass(ctx):
    """Config 3: 9 source views, 1600x1200, the full-size REFINE_ITER + geometric pass."""
    sc, inp, st = pass_case(1600, 1200, 10, 1, 0)
    g, o = run_both(ctx, inp, st)
    assert_same(g, o, "config3 refine_iter+geom")
    check_properties(g, sc, "config3", 9)


# ------------------------------------------------------------------------------ config 4
@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("W,H,i,j", [(672, 448, 0, -1), (1344, 896, 1, 0)])
def test_config4_pyramid_levels_vs_oracle(ctx, W, H, i, j):
    """Config 4 (ETH3D 2688x1792, 3 rounds): its round-0 and round-1 passes with 16 source views."""
    sc, inp, st = pass_case(W, H, 17, i, j)
    inp["params"].max_scale_size = 4
    g, o = run_both(ctx, inp, st)
    assert_same(g, o, f"config4 {W}x{H}")


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config4_full_size_properties(ctx):
    """Config 4 at 2688x1792 with 16 source views (round 2, REFINE_ITER + geom)."""
    sc, inp, st = pass_case(2688, 1792, 17, 2, 0)
    inp["params"].max_scale_size = 4
    ctx.stage(inp, st)
    ctx.set_timing(True)
    ctx.execute(); seq = ctx.fetch()          # one stream, per-class events
    ctx.set_timing(False)
    ctx.execute(); ovl = ctx.fetch()          # GenNeighbours on the second stream
    ctx.execute(); again = ctx.fetch()        # idempotent
    for k in seq:
        assert bits_equal(seq[k], ovl[k]) and bits_equal(ovl[k], again[k]), k
    check_properties(ovl, sc, "config4 full", 16)


# ------------------------------------------------------------------------------ config 5
@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config5_coarse_level_31_views_vs_oracle(ctx):
    """Config 5 (TaT 1920x1080, 3 rounds): round 0 at 480x270 with 31 source views (32 images, the
    reference's MAX_IMAGES: all 32 bits of the view masks in use)."""
    sc, inp, st = pass_case(480, 270, 32, 0, 0)
    inp["params"].max_scale_size = 4
    g, o = run_both(ctx, inp, st)
    assert_same(g, o, "config5 480x270x31")


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config5_full_size_properties_and_fusion(ctx):
    """Config 5 at 1920x1080 with 31 source views: the full-size pass by properties, and fusion's
    per-(pixel, view) projection tests (RunFusion DPE.cpp:1303-1343) HIP == oracle at full size."""
    sc, inp, st = pass_case(1920, 1080, 32, 2, 0)
    inp["params"].max_scale_size = 4
    ctx.stage(inp, st)
    ctx.execute(); a = ctx.fetch()
    ctx.execute(); b = ctx.fetch()
    for k in a:
        assert bits_equal(a[k], b[k]), k
    check_properties(a, sc, "config5 full", 31)
    # fusion projection tests over the 32 views' ground-truth depth / normal maps
    views = [(np.where(np.isfinite(v["depth"]), v["depth"], 0).astype(np.float32), v["normals"], cam)
             for v, cam in zip(sc["views"], sc["cams"])]
    src = list(range(1, 32))
    gi, gv = ctx.fusion_candidates(views, 0, src)
    oi, ov = oracle.fusion_candidates(views, 0, src)
    assert np.array_equal(gi, oi)
    m = np.repeat(gi >= 0, 3)
    assert np.array_equal(gv[m].view(np.uint32), ov[m].view(np.uint32))
    assert (gi >= 0).mean() > 0.3
