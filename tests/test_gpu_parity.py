"""GPU parity: the HIP path (through the C-ABI) is bit-exact against the CPU restatement.

Tolerance: 0 — planes (depth + normal), costs, weak_info and selected_views must be
bit-identical (the north star asks depth within 1e-3 relative and weak/edge maps bit-exact;
the shared IEEE arithmetic makes every output exact).
"""
import numpy as np
import pytest

import oracle
from DPE_MVS import _abi, synthetic
from golden_io import bits_equal, load, names

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from DPE_MVS import native
    c = native.PatchMatchContext(0)
    yield c
    c.close()


def assert_same(g, o, what=""):
    for k in ("planes", "weak", "sel", "costs"):
        if not bits_equal(g[k], o[k]):
            a, b = g[k], o[k]
            neq = (a.view(np.uint32) != b.view(np.uint32)) if a.dtype == np.float32 else (a != b)
            if neq.ndim == 3:
                neq = neq.any(-1)
            ys, xs = np.nonzero(neq)
            pytest.fail(f"{what}: {k} differs at {len(ys)} pixels, first ({ys[0]}, {xs[0]})")


@pytest.mark.parametrize("name", names())
def test_gpu_matches_golden(ctx, name):
    inp, st, exp = load(name)
    assert_same(ctx.run(inp, st), exp, name)


def _params(kind, iters=3):
    p = _abi.default_params()
    p.max_iterations = iters
    if kind == "first":
        p.state = _abi.FIRST_INIT; p.use_APD = False; p.use_edge = False
    elif kind == "refine_init":
        p.state = _abi.REFINE_INIT; p.rotate_time = 4; p.ransac_threshold = 0.0075; p.max_scale_size = 4
        p.weak_peak_radius = 6
    elif kind == "refine_iter":
        p.state = _abi.REFINE_ITER; p.geom_consistency = True; p.rotate_time = 2; p.ransac_threshold = 0.00875
        p.max_scale_size = 2; p.weak_peak_radius = 2
    elif kind == "refine_iter_lowres":
        p.state = _abi.REFINE_ITER; p.geom_consistency = True; p.rotate_time = 1; p.ransac_threshold = 0.01
        p.high_res_img = False; p.use_label = True; p.weak_peak_radius = 4
    elif kind == "acmh_geom":            # ACMH candidate scheme (no APD / edges) with geometric consistency
        p.state = _abi.REFINE_ITER; p.use_APD = False; p.use_edge = False; p.geom_consistency = True
        p.rotate_time = 2; p.ransac_threshold = 0.00875
    elif kind == "no_limit":             # no edge limit, labels or radius map (DPE.cu:2116-2124, 1690-1700)
        p.state = _abi.REFINE_INIT; p.use_limit = False; p.use_label = False; p.use_radius = False
        p.rotate_time = 2; p.ransac_threshold = 0.0075
    elif kind == "weak_generic":         # 5x5 neighbour patches: the untabulated NCC-New path
        p.state = _abi.REFINE_ITER; p.geom_consistency = True; p.rotate_time = 2; p.ransac_threshold = 0.00875
        p.weak_radius = 6; p.weak_increment = 3; p.sigma_spatial = 4.0; p.sigma_color = 6.0
    return p


CASES = [
    # W, H, views, kind
    (96, 72, 4, "first"),
    (96, 72, 4, "refine_init"),
    (128, 96, 6, "refine_iter"),
    (77, 33, 3, "refine_iter"),          # odd H with (H/2) % 16 == 0: last row outside the red/black grid
    (64, 48, 2, "first"),                # 1 source view
    (72, 54, 5, "refine_iter_lowres"),
    (80, 60, 4, "acmh_geom"),
    (88, 66, 4, "no_limit"),
    (72, 56, 3, "weak_generic"),
    (23, 131, 3, "refine_iter"),         # tall, narrow: W < one block, ragged in both axes
    (193, 29, 3, "first"),               # W = 3*64+1: one pixel into a fourth wave-width column
    (12, 40, 3, "refine_iter"),          # no DepthToWeak interior: LocalRefine over every pixel (border kernel)
    (40, 13, 3, "refine_iter"),          # one interior row: fused DepthToWeak+LocalRefine beside the border kernel
]


@pytest.mark.parametrize("W,H,N,kind", CASES)
def test_gpu_matches_oracle(ctx, W, H, N, kind):
    sc = synthetic.make_scene(W, H, N)
    p = _params(kind)
    geom = p.geom_consistency
    st = synthetic.first_init_state(sc) if kind == "first" else synthetic.gt_state(sc, seed=W + H)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc) if geom else None, seed=W * 7 + N)
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), f"{W}x{H}x{N} {kind}")


@pytest.mark.parametrize("W,H,N,kind", [(128, 96, 6, "refine_iter"), (96, 72, 4, "refine_init"), (88, 66, 4, "no_limit")])
def test_gpu_gen_neighbours_overflow_path(W, H, N, kind):
    # GenNeighbours' deferral path (DPE.cu:2281-2307 point collection, :2367-2449 sorts): with 8
    # support-point slots (DPE_OPT_GN_SLOTS) the scratch-free kernel hands every pixel with more points
    # to the scratch kernel (k_gen_neighbours over the overflow list).  The neighbours, weak_reliable
    # and complex it writes feed NeigbourUpdate and every NCC-New of the weak sweep, so the pass
    # outputs must stay the oracle's bit for bit; the deferred count must be > 0.  With the default
    # slots nothing is deferred at these sizes.
    from DPE_MVS import native
    sc = synthetic.make_scene(W, H, N)
    p = _params(kind)
    st = synthetic.gt_state(sc, seed=W + H)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc) if p.geom_consistency else None, seed=W * 7 + N)
    want = oracle.run_pass(inp, st)
    c = native.PatchMatchContext(0)
    try:
        got_default = c.run(inp, st)
        assert c.last_stat(_abi.DPE_STAT_GN_DEFERRED) == 0
        c.set_option(_abi.DPE_OPT_GN_SLOTS, 8)
        got = c.run(inp, st)
        deferred = c.last_stat(_abi.DPE_STAT_GN_DEFERRED)
    finally:
        c.close()
    assert deferred > 0, deferred
    assert_same(got_default, want, f"{W}x{H}x{N} {kind} default slots")
    assert_same(got, want, f"{W}x{H}x{N} {kind} 8 slots ({deferred} pixels deferred)")


def test_gpu_many_views(ctx):
    # 32 images = the reference's MAX_IMAGES (31 source views, 32-bit view masks)
    sc = synthetic.make_scene(48, 36, 32)
    p = _params("refine_iter", iters=1)
    st = synthetic.gt_state(sc)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), "32 views")


def test_gpu_nondefault_patch(ctx):
    # strong_radius / increment other than 5 / 2 take the generic (per-tap weight) NCC path
    sc = synthetic.make_scene(64, 48, 3)
    p = _params("first", iters=1)
    p.strong_radius = 4; p.strong_increment = 1
    inp = synthetic.pass_input(sc, p)
    st = synthetic.first_init_state(sc)
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), "radius 4 / increment 1")


def test_execute_idempotent_and_deterministic(ctx):
    sc = synthetic.make_scene(160, 120, 5)
    p = _params("refine_iter")
    st = synthetic.gt_state(sc)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    ctx.stage(inp, st)
    ctx.execute(); a = ctx.fetch()
    ctx.execute(); b = ctx.fetch()
    for k in a:
        assert bits_equal(a[k], b[k]), k


@pytest.mark.parametrize("kind", ["refine_iter", "refine_init", "first"])
def test_overlapped_and_sequential_schedules_agree(ctx, kind):
    # untimed executes fork the setup chain (GenEdgeInform .. NeigbourUpdate) to the aux stream beside
    # RandomInitialization and the first strong half-sweep; timed executes keep one stream.  Both
    # must give the oracle's bits in every output (planes, weak, sel, costs), so a launch that reads a
    # setup output before the join is caught (include/dpe_mvs.h, dpe_pm_execute).
    sc = synthetic.make_scene(128, 96, 6)
    p = _params(kind)
    st = synthetic.gt_state(sc, seed=11)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc) if p.geom_consistency else None, seed=5)
    ctx.stage(inp, st)
    ctx.set_timing(True)
    ctx.execute(); seq = ctx.fetch()
    ctx.set_timing(False)
    ctx.execute(); ovl = ctx.fetch()
    for k in seq:
        assert bits_equal(seq[k], ovl[k]), k
    assert_same(ovl, oracle.run_pass(inp, st), "overlapped schedule")


def test_error_paths(ctx):
    from DPE_MVS import native
    sc = synthetic.make_scene(32, 24, 2)
    p = _params("refine_iter")
    inp = synthetic.pass_input(sc, p, depths=None)          # geom without depth maps
    with pytest.raises(native.DpeError):
        ctx.run(inp, synthetic.gt_state(sc))
    fresh = native.PatchMatchContext(0)
    with pytest.raises(native.DpeError):
        fresh.execute()                                      # execute before stage
    fresh.close()


def test_gpu_non_integer_images(ctx):
    # grey levels that are not multiples of 1/4: exercises the f32 quad-texel layout
    sc = synthetic.make_scene(96, 72, 4)
    sc["images"] = [(im * np.float32(0.73) + np.float32(0.31)).astype(np.float32) for im in sc["images"]]
    p = _params("refine_iter")
    st = synthetic.gt_state(sc)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), "f32 images")
    assert ctx.last_stat(_abi.DPE_STAT_TEX_CLASS) == 0


@pytest.mark.parametrize("kind", ["refine_iter", "refine_init", "first"])
def test_gpu_quarter_integer_images(ctx, kind):
    """A coarse pyramid level: the host pipeline's INTER_LINEAR 1/2 downscale (DPE.cpp:798-809) of 8-bit
    images has grey levels in multiples of 1/4, which the f16 texel layouts hold exactly (strong sweep
    P16, DepthToWeak / LocalRefine / init F16, weak sweep F16 instead of U8): bit-exact vs the oracle."""
    from DPE_MVS import pipeline
    full = synthetic.make_scene(192, 144, 4)
    sc = synthetic.make_scene(96, 72, 4)
    sc["images"] = [pipeline.resize_linear(im.astype(np.float32), 96, 72) for im in full["images"]]
    q = np.concatenate([im.ravel() for im in sc["images"]])
    assert np.all(q * 4 == np.round(q * 4)) and not np.all(q == np.round(q))   # quarter-integers, not 8-bit
    p = _params(kind)
    st = synthetic.first_init_state(sc) if kind == "first" else synthetic.gt_state(sc)
    depths = synthetic.src_depths(sc) if p.geom_consistency else None
    inp = synthetic.pass_input(sc, p, depths=depths)
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), f"quarter-integer images ({kind})")
    assert ctx.last_stat(_abi.DPE_STAT_TEX_CLASS) == 1


def test_image_ids_keep_images_resident(ctx):
    """DpePassInput.image_ids: images uploaded once per (id, size); later passes reuse the HBM copies
    and give the same bits as uploading every time."""
    sc = synthetic.make_scene(96, 72, 4)
    p = _abi.default_params()
    p.state = _abi.REFINE_ITER
    p.geom_consistency = True
    p.rotate_time = 2
    p.ransac_threshold = 0.00875
    p.max_scale_size = 2
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    st = synthetic.gt_state(sc)
    plain = ctx.run(inp, st)
    inp_ids = dict(inp, image_ids=[7, 3, 9, 11])
    first = ctx.run(inp_ids, st)
    again = ctx.run(inp_ids, st)                                   # all four from the cache
    for k in ("planes", "weak", "sel", "costs"):
        assert plain[k].tobytes() == first[k].tobytes() == again[k].tobytes(), k
    other = synthetic.make_scene(96, 72, 4, seed=synthetic.SCENE_SEED + 5)
    inp2 = dict(synthetic.pass_input(other, p, depths=synthetic.src_depths(other)), image_ids=[21, 22, 23, 24])
    ref2 = ctx.run(dict(inp2, image_ids=None), synthetic.gt_state(other))
    got2 = ctx.run(inp2, synthetic.gt_state(other))
    assert ref2["planes"].tobytes() == got2["planes"].tobytes()


def test_stage_waits_for_execute_on_a_foreign_stream(ctx):
    """dpe_pm_stage host-waits for the previous execute even when it was enqueued on a caller stream:
    stage(A); execute(A, s); stage(B) must not overwrite inputs pass A is still reading.  The caller
    stream comes from the HIP runtime the library itself links (torch's HIP runtime is a second copy
    that cannot open the device once the library has)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
    sa, sb = synthetic.make_scene(160, 120, 5), synthetic.make_scene(160, 120, 5, seed=synthetic.SCENE_SEED + 9)
    p = _params("refine_iter")
    ia, sta = synthetic.pass_input(sa, p, depths=synthetic.src_depths(sa)), synthetic.gt_state(sa)
    ib, stb = synthetic.pass_input(sb, p, depths=synthetic.src_depths(sb), seed=4), synthetic.gt_state(sb, seed=3)
    want = ctx.run(ia, sta)
    s = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0          # hipStreamNonBlocking
    try:
        ctx.stage(ia, sta)
        ctx.execute(s.value)
        ctx.stage(ib, stb)                  # returns only after pass A is done
        got = ctx.fetch()                   # the working buffers still hold pass A's result
        for k in want:
            assert bits_equal(want[k], got[k]), k
    finally:
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0


def test_zero_iterations_joins_the_aux_stream(ctx):
    # max_iterations = 0: no sweep joins the GenNeighbours stream, so the pass keeps one stream
    sc = synthetic.make_scene(96, 72, 4)
    p = _params("refine_iter", iters=0)
    st = synthetic.gt_state(sc)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), "max_iterations 0")


def _random_case(seed):
    """A seeded random pass configuration: size, views, pass type and the schedule's switches
    (rotate_time, labels, edge limit, radius map, resolution class, iterations, peak radius,
    RANSAC threshold, candidate scheme, geometric consistency, NCC-New patch)."""
    r = np.random.default_rng(1000 + seed)
    W, H, N = int(r.integers(24, 161)), int(r.integers(24, 121)), int(r.integers(2, 11))
    p = _abi.default_params()
    p.max_iterations = int(r.integers(1, 4))
    kind = ("first", "refine_init", "refine_iter")[int(r.integers(0, 3))]
    if kind == "first":
        p.state = _abi.FIRST_INIT; p.use_APD = False; p.use_edge = False; p.geom_consistency = False
    else:
        p.state = _abi.REFINE_INIT if kind == "refine_init" else _abi.REFINE_ITER
        p.geom_consistency = kind == "refine_iter" and bool(r.integers(0, 2))
        apd = bool(r.integers(0, 4))                      # 1 in 4: the ACMH scheme
        p.use_APD = apd; p.use_edge = apd
        p.rotate_time = int((1, 2, 4)[int(r.integers(0, 3))])
        p.ransac_threshold = float(np.float32(r.uniform(0.005, 0.01)))
        p.weak_peak_radius = int(r.integers(2, 7))
        p.use_label = bool(r.integers(0, 2)); p.use_limit = bool(r.integers(0, 4))
        p.use_radius = bool(r.integers(0, 4)); p.high_res_img = bool(r.integers(0, 2))
        if r.integers(0, 4) == 0:                         # untabulated NCC-New neighbour patches
            p.weak_radius = int(r.integers(3, 7)); p.weak_increment = int(r.integers(2, 4))
    return W, H, N, kind, p


@pytest.mark.parametrize("seed", range(24))
def test_gpu_matches_oracle_random_configs(ctx, seed):
    W, H, N, kind, p = _random_case(seed)
    sc = synthetic.make_scene(W, H, N, seed=synthetic.SCENE_SEED + seed)
    st = synthetic.first_init_state(sc) if kind == "first" else synthetic.gt_state(sc, seed=seed)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc) if p.geom_consistency else None, seed=seed + 3)
    what = f"seed {seed}: {W}x{H}x{N} {kind} it={p.max_iterations} rot={p.rotate_time} apd={p.use_APD} " \
           f"geom={p.geom_consistency} label={p.use_label} limit={p.use_limit} radius={p.use_radius} " \
           f"hires={p.high_res_img} weak={p.weak_radius}/{p.weak_increment}"
    assert_same(ctx.run(inp, st), oracle.run_pass(inp, st), what)
