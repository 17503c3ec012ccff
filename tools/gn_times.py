"""Per-pixel / per-wave durations of the scratch-free GenNeighbours on the bench workload (a
-DDPE_DIAG=8 build of libdpe_mvs.so): how long each WEAK pixel's probes and whole job take
(shader clocks), and how long each wave lives (its slowest lane), to tell a few stragglers from a
uniform load.  One timed, one-stream execute; prints quantiles.
Usage: python tools/gn_times.py lib/variants/gntimes.so"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
torch.cuda.set_device(0)
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
st = synthetic.gt_state(sc)
lib = native.load_library(sys.argv[1])
ctx = lib.dpe_create(0)
bufs = _abi.PassBuffers(inp, st)
assert lib.dpe_pm_stage(ctx, C.byref(bufs.inp), C.byref(bufs.st)) == 0
lib.dpe_set_timing(ctx, 1)
assert lib.dpe_pm_execute(ctx, None) == 0
assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0
tm = (C.c_float * 9)()
lib.dpe_pm_last_timings(ctx, tm, 9)
n = 2 << 20
buf = (C.c_uint * n)()
lib.dpe_dbg_gn_times(buf, n)
a = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 2).astype(np.float64)
used = np.nonzero(a[:, 1])[0]
m = int(used.max()) + 1 if used.size else 0
a = a[:m]
probe, total = a[:, 0], a[:, 1]
waves = total[: (m // 64) * 64].reshape(-1, 64)
wmax, wmean = waves.max(1), waves.mean(1)
q = lambda v: " ".join(f"p{k}={np.percentile(v, k):.3g}" for k in (10, 50, 90, 99, 100))  # noqa: E731
print(f"setup class {tm[1]:.3f} ms (one stream); WEAK pixels {m}, waves {waves.shape[0]}")
print("pixel total cycles  ", f"mean={total.mean():.3g}", q(total))
print("pixel probe cycles  ", f"mean={probe.mean():.3g}", q(probe))
print("wave max (lifetime) ", f"mean={wmax.mean():.3g}", q(wmax))
print("wave mean / wave max", f"{(wmean / np.maximum(wmax, 1)).mean():.3f}")
print("lane utilisation (sum of pixel cycles / (64 x sum of wave lifetimes))", f"{waves.sum() / (64 * wmax.sum()):.3f}")
srt = np.sort(wmax)[::-1]
for k in (1, 10, 100, 1000):
    if k <= srt.size:
        print(f"slowest {k:5d}-th wave: {srt[k - 1]:.3g} cycles")
cb = (C.c_uint * (6 << 20))()
lib.dpe_dbg_gn_counts(cb, 6 << 20)
cnt = np.frombuffer(cb, dtype=np.uint32).reshape(-1, 6)[:m].astype(np.float64)
names = ["radius steps", "probe Bresenham walks", "RANSAC tries", "RANSAC Bresenham walks",
         "probe Bresenham clocks", "RANSAC Bresenham clocks"]
nw = (m // 64) * 64
for k, nm in enumerate(names):
    v = cnt[:, k]
    w = v[:nw].reshape(-1, 64)
    util = w.sum() / max(1.0, 64 * w.max(1).sum())
    print(f"{nm:24s} per pixel mean={v.mean():.1f}", q(v), f"| per wave max mean={w.max(1).mean():.1f} lane utilisation={util:.3f}")
# the slowest waves: their slowest lane's time and work counts (what the kernel's tail is made of)
order = np.argsort(wmax)[::-1][:20]
print("slowest waves (a lane's time is its wave's: lanes wait for each other at every reconvergence):")
print("  wave: cycles | probe cycles | max over lanes of: radius steps, probe walks, RANSAC tries, RANSAC walks, probe walk clocks, RANSAC walk clocks")
for wi in order:
    lanes = np.arange(wi * 64, wi * 64 + 64)
    mx = cnt[lanes].max(axis=0)
    print(f"  wave {wi:5d}: {wmax[wi]:.3g} | {probe[lanes].max():.3g} | " + " ".join(f"{mx[k]:.0f}" for k in range(6)))
lib.dpe_destroy(ctx)
