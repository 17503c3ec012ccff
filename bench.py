#!/usr/bin/env python3
"""Benchmark of the MI355X PatchMatch pass (BASELINE.json metric: depth-map Mpix/s).

Workload (BASELINE.json configs[2], the headline of SURVEY.md §8d): one full-resolution
REFINE_ITER pass with geometric consistency at 1600x1200, 9 source views (num_images = 10),
round-1 parameters of the reference schedule (main.cpp:536-557: use_APD, use_edge,
rotate_time 2, ransac_threshold 0.00875, weak_peak_radius 4, max_iterations 3).
Inputs are a synthetic scene (DPE_MVS.synthetic, no datasets reachable) with ground-truth-derived
priors and source depth maps, resident in HBM before the timed region (dpe_pm_stage).

A step = one dpe_pm_execute (all 26+ launches of DPE::RunPatchMatch) on each rank's own reference
image; at N > 1 each step also all-gathers the depth maps over RCCL (the exchange between
geometric-consistency passes).  Reference images shard one per rank, so per-GPU
work is fixed as N grows ("scaling": "weak"); value = all ranks' pixels / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 either under a launcher (WORLD_SIZE must equal N):
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
  or directly: `python bench.py --gpus N` starts the N ranks itself as a child torch.distributed.run
  (before anything touches the GPU) and relays rank 0's JSON line and exit code.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))

W_, H_, NV_ = 1600, 1200, 10
METRIC = "depth-map Mpixels/sec (9-view 1600x1200 PatchMatch) at 1/2/4/8 GPUs; L1 vs ref"
FP32_PEAK_TFLOPS = 157.3        # MI355X vector/matrix FP32 peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FLOP_PER_TAP = 32               # algorithmic model: 36-tap NCC = 36*32 + 120
FLOP_PER_HOMOGRAPHY = 120
FLOP_PER_GEOM = 60
MODEL_FLOP_PER_PX = (36 * FLOP_PER_TAP + FLOP_PER_HOMOGRAPHY) * (42 * (NV_ - 1) + 75 * 4)   # 0.86 MFLOP
# per-dispatch HBM bytes from the committed PMC passes (tools/pmc.sh + tools/prof_summary.py)
PMC_JSON = next((os.path.join(ROOT, "profiles", f) for f in ("r06g_pmc.json", "r06f_pmc.json", "r06_pmc.json", "r05_pmc.json", "r04f_pmc.json", "r04_pmc.json", "r03s2_pmc.json", "r03_pmc.json", "r02_pmc.json")
                 if os.path.exists(os.path.join(ROOT, "profiles", f))), os.path.join(ROOT, "profiles", "r04_pmc.json"))
# secondary roof (the on-chip gather rate): a 64-lane texel gather costs the texture
# path at least one CU-cycle per lane quad = 16 CU-cycles (profiles/r03_td_probe2.md), so at the
# ~2.4 GHz the chip holds a CU serves at most 64 taps per 16 cycles; bytes per tap of each class's layout
GATHER_CU = 256
GATHER_GHZ = 2.4
GATHER_CYCLES_PER_WAVE = 16
TAP_BYTES = {"strong": 8, "depth_to_weak": 8, "local_refine": 8, "init": 8, "weak": 4}   # P16 / F16 / U8 texels
CLASS_KERNEL = {"strong": "k_strong_coop", "weak": "k_weak_coop", "depth_to_weak": "k_depth_to_weak",
                "local_refine": "k_local_refine_jobs", "init": "k_random_init", "ransac": "k_ransac_fit",
                "setup": "k_gen_neighbours_lds"}


def workload_params(abi, N):
    p = abi.default_params()
    p.state = abi.REFINE_ITER
    p.use_APD = True
    p.use_edge = True
    p.geom_consistency = True
    p.max_iterations = 3
    p.rotate_time = 2                 # min(2^i, 4), i = 1 (main.cpp:552)
    p.ransac_threshold = 0.01 - 1 * 0.00125
    p.weak_peak_radius = 4            # max(4 - 2j, 2), j = 0 (main.cpp:555)
    p.max_scale_size = 2
    p.scale_size = 1
    p.num_images = N
    return p


def algorithmic_flops(cnt: dict) -> float:
    return FLOP_PER_HOMOGRAPHY * cnt["ncc"] + FLOP_PER_TAP * cnt["taps"] + FLOP_PER_GEOM * cnt["geom"]


def pmc_traffic(cls: str):
    """HBM bytes per launch of the class's kernel from the committed PMC summary, or None."""
    if not os.path.exists(PMC_JSON):
        return None
    tr = json.load(open(PMC_JSON)).get("traffic", {})
    vals = [v["hbm_bytes_per_dispatch"] for k, v in tr.items() if k.split("<")[0] == CLASS_KERNEL.get(cls)]
    return sum(vals) / len(vals) if vals else None


def crop_rows(sc: dict, y0: int, y1: int) -> dict:
    """The scene restricted to reference-image rows [y0, y1) of every view: images, depths, edges and
    labels cropped, principal point and height of every camera moved with the crop.  A valid pass of
    the same workload on a full-width band (a 256-row crop, extrapolated in rows)."""
    import copy
    out = dict(sc)
    out["H"] = y1 - y0
    cams = []
    for c in sc["cams"]:
        c2 = copy.deepcopy(c)
        c2.K[5] = float(np.float32(c.K[5]) - np.float32(y0))
        c2.height = y1 - y0
        cams.append(c2)
    out["cams"] = cams
    out["images"] = [np.ascontiguousarray(im[y0:y1]) for im in sc["images"]]
    out["views"] = [dict(v, depth=np.ascontiguousarray(v["depth"][y0:y1]), normals=np.ascontiguousarray(v["normals"][y0:y1]),
                         sid=v["sid"][y0:y1], image=out["images"][k]) for k, v in enumerate(sc["views"])]
    out["edge"] = np.ascontiguousarray(sc["edge"][y0:y1])
    out["label"] = np.ascontiguousarray(sc["label"][y0:y1])
    lo = (y0 // 2, (y1 + 1) // 2)
    out["edge_low"] = np.ascontiguousarray(sc["edge_low"][lo[0]:lo[1]])
    out["weak_gt"] = sc["weak_gt"][y0:y1]
    return out


def cpu_baseline(abi, synthetic, sc: dict) -> tuple:
    """Scalar C++ restatement (oracle/) timed on this host's cores: the headline pass
    (same parameters, 9 source views) on full-width row bands of the 1600x1200 scene, extrapolated
    linearly in rows -- all host threads on a 256-row band, 1 thread on a 32-row band (bounded:
    about 10-30 s of CPU work each on the GPU box)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / baseline only
    W, H = sc["W"], sc["H"]
    p = workload_params(abi, NV_)
    res = {}
    sample = None
    for threads, rows in ((oracle.host_threads(), 256), (1, 32)):
        y0 = (H - rows) // 2
        band = crop_rows(sc, y0, y0 + rows)
        inp = synthetic.pass_input(band, p, depths=synthetic.src_depths(band))
        st = synthetic.gt_state(band)
        t0 = time.perf_counter()
        ref = oracle.run_pass(inp, st, threads=threads)
        dt = time.perf_counter() - t0
        res[threads] = (dt, rows, dt * H / rows)
        if sample is None:
            sample = (inp, st, ref, f"{W}x{rows} band (rows {y0}..{y0 + rows - 1})")
    nt = max(res)
    dt, rows, full = res[nt]
    dt1, rows1, full1 = res[1]
    base = {"value": round(W * H / full / 1e6, 6), "unit": "Mpix/s", "cores": nt, "kind": "port",
            "sample": f"the headline REFINE_ITER+geom pass (9 source views) on a full-width {rows}-row band "
                      f"({W}x{rows}), oracle/ scalar C++ restatement, {nt} threads, {dt:.1f} s, extrapolated "
                      f"x{H / rows:.2f} in rows to {full:.1f} s per {W}x{H} pass",
            "single_thread": {"value": round(W * H / full1 / 1e6, 6), "unit": "Mpix/s", "cores": 1,
                              "sample": f"{W}x{rows1} band, 1 thread, {dt1:.1f} s, extrapolated to {full1:.1f} s per pass"},
            "host_cpus": os.cpu_count(), "threads_note": "threads = OMP_NUM_THREADS (the GPU box's CPU share) "
                                                          "or the affinity mask; host_cpus = the whole machine"}
    return base, sample


def end_to_end(local_rank: int, n_images: int, W: int, H: int, scene=None) -> dict:
    """SURVEY.md §8d end-to-end rate: n_images * W * H / wall time of DPE_MVS.dpe_mvs() on a synthetic
    dense_folder (JPEG images, cams, pair.txt; no edge/label maps, so EdgeSegment runs as in the
    reference): decode, pyramid, EdgeSegment, the whole coarse-to-fine schedule (8 passes per image),
    the .npy outputs."""
    import shutil
    import tempfile
    from DPE_MVS import synthetic, dpe_mvs
    d = tempfile.mkdtemp(prefix="dpe_e2e_")
    try:
        synthetic.write_dense_folder(d, W, H, n_images, max_src=min(9, n_images - 1), with_edges=False,
                                     scene=scene if scene is not None and len(scene["views"]) == n_images else None)
        t0 = time.perf_counter()
        dpe_mvs(d, local_rank, False, False, False, True, False, False, False)
        dt = time.perf_counter() - t0
        import ctypes
        from DPE_MVS import pipeline
        phases = (ctypes.c_double * 5)()
        pipeline.lib().dpe_pipeline_last_timings(phases, 5)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"images": n_images, "width": W, "height": H, "src_views": min(9, n_images - 1), "passes_per_image": 8,
            "wall_s": round(dt, 3), "mpix_s": round(n_images * W * H / dt / 1e6, 4),
            "phases_s": {"decode": round(phases[1], 3), "edge_segment_prepass": round(phases[2], 3),
                         "passes": round(phases[3], 3), "outputs": round(phases[4], 3)},
            "note": "dpe_mvs() wall clock incl. JPEG decode, EdgeSegment, host I/O; value is per-pass HBM-resident"}


def coarse_level_pass(native, _abi, synthetic, local_rank: int, sp, W: int, H: int, nv: int = 10, reps: int = 3) -> dict:
    """A coarse pyramid level of the schedule (main.cpp:494-501): the REFINE_ITER + geom pass at
    (W/2) x (H/2), its images the host pipeline's INTER_LINEAR 1/2 downscale (DPE.cpp:798-809) of an
    8-bit W x H rendering -- quarter-integer grey levels, i.e. the f16 texel layouts
    (DPE_STAT_TEX_CLASS 1) -- with the cameras, priors and source depths of the same synthetic scene
    rendered at (W/2) x (H/2).  Rate = pixels / wall time of one execute (timed after a warm-up)."""
    import torch
    from DPE_MVS import pipeline
    w, h = W // 2, H // 2
    full = synthetic.make_scene(W, H, nv)
    sc = synthetic.make_scene(w, h, nv)
    sc["images"] = [pipeline.resize_linear(im.astype(np.float32), w, h) for im in full["images"]]
    del full
    p = workload_params(_abi, nv)
    p.max_scale_size = 2
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    st = synthetic.gt_state(sc)
    c = native.PatchMatchContext(local_rank)
    try:
        c.stage(inp, st)
        cls = c.last_stat(_abi.DPE_STAT_TEX_CLASS)
        c.execute(sp)                                   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):                           # each execute restarts from the staged state
            c.execute(sp)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
    finally:
        c.close()
    return {"mpix_s": round(w * h / dt / 1e6, 4), "ms": round(dt * 1e3, 3), "tex_class": int(cls)}


PIPELINE_CONFIGS = {
    # BASELINE configs[3]: ETH3D high-res size, 16 reference images, 9 source views each
    "config4": dict(n=16, W=2688, H=1792, max_src=9, fusion=False,
                    label="BASELINE configs[3]: ETH3D-size 2688x1792, 16 reference images, 9 source views each, "
                          "full 3-round schedule, images sharded over the ranks (synthetic scene)"),
    # BASELINE configs[4]: Tanks&Temples Intermediate size, 32 images, 31 source views each (the most the
    # 32-bit view masks hold, main.h MAX_IMAGES), edge-guided deformable patches, fusion
    "config5": dict(n=32, W=1920, H=1080, max_src=31, fusion=True,
                    label="BASELINE configs[4]: TaT-size 1920x1080, 32 reference images, 31 source views each, "
                          "edge-guided deformable patches, full 3-round schedule + RunFusion, images sharded "
                          "over the ranks (synthetic scene)"),
}


def pipeline_config(dist, rank: int, world: int, local_rank: int, name: str) -> dict:
    """A BASELINE multi-image config at the pipeline level (PIPELINE_CONFIGS[name]) through
    DPE_MVS.run_dpe_pipeline: decode, EdgeSegment, the full coarse-to-fine schedule of RunDPEPipeline
    (main.cpp:508-566: 3 resolution rounds x 4 passes, geometric consistency from the second pass on),
    the outputs and, for config 5, RunFusion on rank 0 (main.cpp:578-580 -> DPE.cpp:1220-1370) -- with
    the images sharded in contiguous blocks over the ranks and the depth maps all-gathered between
    passes (RCCL device hook under "nccl").  Wall time = max over ranks; rate = n * W * H / wall."""
    import shutil
    from DPE_MVS import pipeline, synthetic
    cfg = PIPELINE_CONFIGS[name]
    n, W, H = cfg["n"], cfg["W"], cfg["H"]
    tag = os.environ.get("TORCHELASTIC_RUN_ID") or os.environ.get("MASTER_PORT") or str(os.getpid())
    folder = os.path.join("/tmp", f"dpe_{name}_{tag}")
    if rank == 0:
        shutil.rmtree(folder, ignore_errors=True)
        sc = synthetic.make_scene(W, H, n)
        synthetic.write_dense_folder(folder, W, H, n, max_src=min(cfg["max_src"], n - 1), with_edges=False, scene=sc)
        del sc
    if dist:
        dist.barrier()
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    error = None
    try:   # a failed run is reported in the line (the pipeline fails every rank at the same exchange);
        # every rank still joins the timing all-gather below, so the ranks stay in step
        pipeline.run_dpe_pipeline(folder, gpu_index=local_rank, verbose=False, fusion=cfg["fusion"],
                                  dist=dist if world > 1 else None)
    except Exception as e:  # noqa: BLE001
        error = f"{type(e).__name__}: {e}"[:400]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    import ctypes
    ph = (ctypes.c_double * 8)()
    pipeline.lib().dpe_pipeline_last_timings(ph, 8)
    # per rank: wall, pass work, depth exchanges (status + export + all-gather + import), EdgeSegment, fusion
    mine = [float("nan") if error else dt, ph[6], ph[5], ph[2], ph[7]]
    per_rank = [mine]
    if dist:
        t = torch.tensor(mine, dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        allr = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        per_rank = [[float(v) for v in a.tolist()] for a in allr]
        dist.barrier()
    if rank == 0:
        shutil.rmtree(folder, ignore_errors=True)
    if error or any(p[0] != p[0] for p in per_rank):
        return {"config": cfg["label"], "ranks": world, "error": error or "failed on another rank",
                "measured_on_hardware": False}
    dt = max(p[0] for p in per_rank)
    passes = [round(p[1], 3) for p in per_rank]
    rehearsal = bool(dist) and dist.get_backend() != "nccl"
    out = {"config": cfg["label"], "images": n, "width": W, "height": H, "src_views": min(cfg["max_src"], n - 1),
           "ranks": world, "ranks_in_group": world,
           "images_per_rank": [((r + 1) * n) // world - (r * n) // world for r in range(world)],
           "wall_s": round(dt, 3), "mpix_s": round(n * W * H / dt / 1e6, 4),
           "passes_s": max(passes), "passes_s_per_rank": passes,
           "exchange_s": round(max(p[2] for p in per_rank), 3),
           "edge_segment_s": round(max(p[3] for p in per_rank), 3)}
    if cfg["fusion"]:
        out["fusion_s"] = round(per_rank[0][4], 3)
    out["note"] = ("pipeline wall incl. JPEG decode, EdgeSegment, 12 passes per image, depth all-gathers, .npy outputs" +
                   ("; fusion_s: RunFusion on rank 0 (dpe_pipeline_last_timings [7], incl. the normal / state "
                    "gather at N > 1)" if cfg["fusion"] else "") +
                   "; passes_s / exchange_s: max over ranks of the pass work and of the depth exchanges "
                   "(dpe_pipeline_last_timings [6] / [5]); passes_s_per_rank shows the load balance" +
                   ("" if world > 1 else "; one rank: no exchange") +
                   ("; REHEARSAL over gloo (ranks may share one GPU): unmeasured on hardware, the RCCL/xGMI numbers "
                    "come only from the driver's multi-GPU node" if rehearsal else ""))
    out["measured_on_hardware"] = not rehearsal
    return out


def parity_on_sample(native, local_rank: int, sample) -> dict:
    """The metric's "L1 vs ref": the HIP pass on the cpu_baseline sample against the oracle's output
    of the same run (depth = plane .w; weak/selected-view maps compared exactly)."""
    import numpy as np
    inp, st, ref, size = sample
    c = native.PatchMatchContext(local_rank)
    try:
        out = c.run(inp, st)
    finally:
        c.close()
    dg, do = out["planes"][..., 3].astype(np.float64), ref["planes"][..., 3].astype(np.float64)
    ok = np.abs(do) > 0
    rel = np.abs(dg - do)[ok] / np.abs(do)[ok]
    bits = {k: bool(np.array_equal(out[k].view(np.uint8), ref[k].view(np.uint8))) for k in ("planes", "weak", "sel", "costs")}
    return {"sample": f"{size} REFINE_ITER+geom pass (the cpu_baseline sample), HIP vs oracle",
            "depth_l1_rel": float(rel.mean()) if rel.size else 0.0,
            "depth_max_rel": float(rel.max()) if rel.size else 0.0,
            "weak_mismatch_px": int((out["weak"] != ref["weak"]).sum()),
            "bit_exact": bits}


def spawn_ranks(n: int) -> int:
    """`--gpus N` (N > 1) without a launcher: one rank per GPU through a CHILD torch.distributed.run
    on 127.0.0.1 (never an exec; nothing has initialised the GPU in this process), its stdout (rank
    0's JSON line) and stderr inherited; returns the child's exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def launch_check(world: int, rank: int) -> None:
    """--launch-check: the rank layout alone (no GPU, gloo), so the --gpus N launch path is testable
    on CPU: every rank joins one all-reduce, rank 0 prints the line's n_gpus and the ranks seen."""
    seen = 1
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "launch_check": True, "n_gpus": world, "ranks_joined": seen}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-instrument", action="store_true", help="skip the hipEvent / work-counter runs (PMC profiling)")
    ap.add_argument("--no-pass-types", action="store_true", help="skip the FIRST_INIT / REFINE_INIT passes (kernel traces)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end dpe_mvs() run")
    ap.add_argument("--e2e-images", type=int, default=10)
    ap.add_argument("--no-pipeline", action="store_true", help="skip the BASELINE configs[3] / [4] pipeline lines")
    ap.add_argument("--no-config5", action="store_true", help="skip the BASELINE configs[4] pipeline line")
    ap.add_argument("--launch-check", action="store_true", help="only check the rank layout (CPU, gloo)")
    ap.add_argument("--width", type=int, default=W_)
    ap.add_argument("--height", type=int, default=H_)
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus}: need at least 1")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                 f"(--nproc-per-node {args.gpus}) or drop the launcher and let --gpus start the ranks")
    rank = int(os.environ.get("RANK", "0"))
    if args.launch_check:
        launch_check(world, rank)
        return
    import torch
    # one rank per GPU; the modulo only matters for a rehearsal of several ranks on one card
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = None
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist
        # "nccl" = RCCL over xGMI; DPE_BENCH_BACKEND=gloo rehearses the N > 1 control flow on one GPU
        backend = os.environ.get("DPE_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    from DPE_MVS import _abi, native, synthetic

    Wd, Hd = args.width, args.height
    # each rank owns a different reference image (different scene seed)
    sc = synthetic.make_scene(Wd, Hd, NV_, seed=synthetic.SCENE_SEED + rank)
    p = workload_params(_abi, NV_)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    inp["image_ids"] = list(range(NV_))          # images stay resident in HBM across passes
    st = synthetic.gt_state(sc)
    ctx = native.PatchMatchContext(local_rank)
    ctx.stage(inp, st)
    torch.cuda.synchronize()
    ts = time.perf_counter()
    ctx.stage(inp, st)            # second staging: the steady-state host->HBM cost of one pass (images cached)
    stage_ms = (time.perf_counter() - ts) * 1e3
    # a dedicated (non-default) stream, made current: the pass, export_depth, the all-gather and the
    # step events are then ordered on one stream.  torch's default stream is the null stream (handle
    # 0), which the library would read as "use my own stream", leaving the collective and the events
    # unordered with the pass.  torch is imported before DPE_MVS, so the library's libamdhip64.so.7
    # resolves to torch's already-loaded copy (same SONAME): one HIP runtime, and torch's stream
    # handle is valid in the library
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp, "bench stream handle must be non-null"
    depth_local = torch.empty((Hd, Wd), dtype=torch.float32, device="cuda")
    gathered = [torch.empty_like(depth_local) for _ in range(world)] if world > 1 else None

    # at N > 1 the step's exchange (export_depth + the all-gather) is bracketed by stream events so
    # that its share of the step is reported beside the pass (events on the pass stream: the
    # all-gather's completion is ordered into it before the next step)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)] if world > 1 else None

    def step(k=None):
        if evs is not None and k is not None:
            evs[k][0].record(stream)
        ctx.execute(sp)
        if world > 1:
            if k is not None:
                evs[k][1].record(stream)
            ctx.export_depth(depth_local.data_ptr(), sp)
            dist.all_gather(gathered, depth_local)
            if k is not None:
                evs[k][2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    value = world * args.steps * Wd * Hd / dt / 1e6
    exchange = None
    if world > 1:   # per-step means on this rank, then the max over ranks
        ex_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
        pass_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
        t = torch.tensor([ex_ms, pass_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ex_ms, pass_ms = float(t[0]), float(t[1])
        exchange = {"allgather_ms": round(ex_ms, 4), "execute_ms": round(pass_ms, 3),
                    "comm_share": round(ex_ms / ms_per_step, 5), "world": world, "backend": dist.get_backend(),
                    "ranks_in_group": dist.get_world_size(),
                    "bytes_per_rank": Wd * Hd * 4, "bytes_gathered": world * Wd * Hd * 4,
                    "scope": "per step, max over ranks: export_depth + all_gather of the f32 depth maps (stream "
                             "events on the pass stream); execute_ms = the pass",
                    "measured_on_hardware": dist.get_backend() == "nccl"}

    if args.no_instrument:
        if rank == 0:
            line = {"metric": METRIC, "value": round(value, 4), "unit": "Mpix/s", "ms_per_step": round(ms_per_step, 3)}
            if exchange is not None:
                line["exchange"] = exchange
            print(json.dumps(line))
        ctx.close()
        return
    # instrumented (untimed) runs: per-class kernel time (hipEvents on the pass stream) and
    # algorithmic work counters (separate run; atomics are never in a timed run)
    ctx.set_timing(True)
    ctx.execute(sp)
    torch.cuda.synchronize()
    tim = ctx.timings()
    ctx.set_timing(False)
    ctx.set_counting(True)
    ctx.execute(sp)
    torch.cuda.synchronize()
    cnt = ctx.counts()
    ctx.set_counting(False)

    # the other pass types of the schedule at the same size (reported per pass type)
    per_type = {"refine_iter": round(value / world, 4)}
    for kind in (() if args.no_pass_types else ("first_init", "refine_init")):
        pk = workload_params(_abi, NV_)
        if kind == "first_init":
            pk.state = _abi.FIRST_INIT; pk.use_APD = False; pk.use_edge = False; pk.geom_consistency = False
            stk = synthetic.first_init_state(sc)
        else:
            pk.state = _abi.REFINE_INIT; pk.geom_consistency = False; pk.rotate_time = 4
            pk.ransac_threshold = 0.0075; pk.max_scale_size = 4; pk.weak_peak_radius = 6
            stk = st
        ik = synthetic.pass_input(sc, pk, depths=None)
        ck = native.PatchMatchContext(local_rank)
        ck.stage(ik, stk)
        ck.execute(sp)                                   # warm-up
        exec_s = 0.0
        for _ in range(2):                               # each pass starts from the staged state
            ck.stage(ik, stk)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ck.execute(sp)
            torch.cuda.synchronize()
            exec_s += time.perf_counter() - t1
        ck.close()
        per_type[kind] = round(2 * Wd * Hd / exec_s / 1e6, 4)
    # the coarse pyramid levels (configs 2/3 at 800x600, config 4 at 1344x896), f16 texel layouts
    levels = {}
    if not args.no_pass_types:
        for (Wl, Hl) in ((Wd, Hd), (2688, 1792)):
            levels[f"{Wl // 2}x{Hl // 2}"] = coarse_level_pass(native, _abi, synthetic, local_rank, sp, Wl, Hl)
    dom = max(("strong", "weak", "depth_to_weak", "local_refine", "init", "ransac", "setup"), key=lambda k: tim.get(k, 0.0))
    launches = max(1, cnt[dom]["launches"])
    flop_per_launch = algorithmic_flops(cnt[dom]) / launches
    avg_launch_ms = tim[dom] / launches
    achieved_tflops = flop_per_launch / (avg_launch_ms * 1e-3) / 1e12
    pass_flops = sum(algorithmic_flops(v) for v in cnt.values())
    # algorithmic HBM bytes of the whole pass (~1.5 KB/px/pass compulsory)
    L = Wd * Hd
    pass_bytes = L * (4 * NV_ + 4 * NV_ + 16 * 2 + 4 + 5 + 32 + 32 + 36) * 1.0
    result = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (DPE_MVS.synthetic pinhole scene, ground-truth-derived priors; no datasets reachable)",
        "config": {"workload": f"DTU-like {Wd}x{Hd}, 9 src views, full-res REFINE_ITER pass + geometric consistency "
                               "(BASELINE configs[2])",
                   "width": Wd, "height": Hd, "num_images": NV_, "max_iterations": 3,
                   "parallelism": f"reference-image sharding x{world}" + (
                       (" + RCCL depth all-gather" if dist.get_backend() == "nccl" else f" + {dist.get_backend()} depth "
                        "all-gather (rehearsal)") if world > 1 else "")},
        "roofline": {
            "bound": "valu",
            "kernel": f"k_{dom}",
            "achieved": round(achieved_tflops, 3),
            "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved_tflops / FP32_PEAK_TFLOPS, 4),
            "traffic": pmc_traffic(dom),
            "traffic_source": os.path.relpath(PMC_JSON, ROOT) + " (FETCH_SIZE x2 x1024 + WRITE_SIZE x1024, per launch)",
            "note": "no MFMA-shaped work: priced against the f32 vector peak.  The tap loops keep the VALU "
                    "occupied ~100 % of the time (~70 % in throughput terms, the rest dependency stalls); making "
                    "every texel gather free moves the strong sweep by nothing and DepthToWeak by 5.7 % "
                    "(profiles/r06a_ab_fake_gather.log, DESIGN.md s3), so HBM / gather bandwidth does not bound "
                    "them. achieved = "
                    "algorithmic FLOP per launch (120/homography + 32/bilinear tap + 60/geom term, counted on "
                    "device) / avg launch time (hipEvents on the pass stream)",
            "avg_launch_ms": round(avg_launch_ms, 3),
            "flop_per_launch": flop_per_launch,
            # SURVEY.md §8(d)'s fixed model for the whole pass, independent of the device counters (and so of
            # any work the implementation skips): F = (36*32 + 120) * S per px, S = 42*Ns + 75*4 NCCs
            "model": {"flop_per_px": MODEL_FLOP_PER_PX, "pass_flop": MODEL_FLOP_PER_PX * L,
                      "achieved": round(MODEL_FLOP_PER_PX * L / (ms_per_step * 1e-3) / 1e12, 3),
                      "frac": round(MODEL_FLOP_PER_PX * L / (ms_per_step * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4),
                      "scope": "whole pass wall time (ms_per_step)"},
            "device_counted": {"pass_flop": pass_flops,
                               "frac": round(pass_flops / (ms_per_step * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4),
                               "vs_model": round(pass_flops / (MODEL_FLOP_PER_PX * L), 3),
                               "scope": "whole pass wall time; the device counts every NCC the pass evaluates "
                                        "(vs_model x the fixed model: DepthToWeak's 61 hypotheses x selected views, "
                                        "LocalRefine, the refinement and final-cost NCCs exceed the model's count; "
                                        "bitwise-identical candidate planes sharing one NCC lowers it)"},
        },
        "gather_roof": {
            "kernel": f"k_{dom}",
            "achieved_taps_per_s": round(cnt[dom]["taps"] / launches / (avg_launch_ms * 1e-3), -6),
            "peak_taps_per_s": GATHER_CU * GATHER_GHZ * 1e9 * 64 / GATHER_CYCLES_PER_WAVE,
            "frac": round(cnt[dom]["taps"] / launches / (avg_launch_ms * 1e-3)
                          / (GATHER_CU * GATHER_GHZ * 1e9 * 64 / GATHER_CYCLES_PER_WAVE), 4),
            "achieved_GBps": round(cnt[dom]["taps"] / launches / (avg_launch_ms * 1e-3) * TAP_BYTES.get(dom, 8) / 1e9, 1),
            "bytes_per_tap": TAP_BYTES.get(dom, 8),
            "note": "SURVEY.md §8d's secondary roof: device-counted bilinear taps per launch / avg launch time against "
                    "the texture path's best case of 16 CU-cycles per 64-lane gather (one 128-B line per lane quad, "
                    "profiles/r03_td_probe2.md); making every gather free does not speed the strong sweep "
                    "(profiles/r06a_ab_fake_gather.log), so this roof is not the bound either"},
        "hbm": {"pass_algorithmic_bytes": pass_bytes,
                "achieved_GBps": round(pass_bytes / (ms_per_step * 1e-3) / 1e9, 2), "peak_GBps": HBM_PEAK_GBS},
        "pass_tflops": round(pass_flops / (ms_per_step * 1e-3) / 1e12, 3),
        "stage_ms": round(stage_ms, 3),
        "pcie_inclusive_mpix_s": round(Wd * Hd / ((stage_ms + ms_per_step) * 1e-3) / 1e6, 4),
        "pass_types_mpix_s": per_type,
        "pass_levels": levels,
        "kernel_ms": {k: round(v, 3) for k, v in tim.items()},
        "work": {k: v for k, v in cnt.items() if v["launches"]},
    }
    if exchange is not None:
        result["exchange"] = exchange
    if not args.no_pipeline:   # every rank joins (the pipeline all-gathers depth maps between passes)
        ctx.close()
        ctx = None
        result["pipeline_config4"] = pipeline_config(dist, rank, world, local_rank, "config4")
        if not args.no_config5:
            result["pipeline_config5"] = pipeline_config(dist, rank, world, local_rank, "config5")
    if rank == 0 and world == 1 and not args.no_e2e:
        if ctx is not None:
            ctx.close()
        ctx = None
        result["end_to_end"] = end_to_end(local_rank, args.e2e_images, Wd, Hd, scene=sc)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], sample = cpu_baseline(_abi, synthetic, sc)
        result["parity"] = parity_on_sample(native, local_rank, sample)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if ctx is not None:
        ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
