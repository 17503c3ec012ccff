"""Job-pool utilisation of the cooperative kernels (a -DDPE_DIAG=16 build of libdpe_mvs.so) over one
timed bench-workload pass: per pool the jobs, the 64-lane rounds they take and the waves, i.e. the
share of lanes a pool round keeps busy (before any divergence inside the jobs).
Usage: python tools/pool_stats.py lib/variants/pstat.so"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
torch.cuda.set_device(0)
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

NAMES = ["strong cost vectors", "strong refinement", "weak candidates", "weak current/fit plane",
         "weak refinement", "weak final Old NCC", "-", "-"]
sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
st = synthetic.gt_state(sc)
lib = native.load_library(sys.argv[1])
ctx = lib.dpe_create(0)
bufs = _abi.PassBuffers(inp, st)
assert lib.dpe_pm_stage(ctx, C.byref(bufs.inp), C.byref(bufs.st)) == 0
lib.dpe_set_timing(ctx, 1)
buf = (C.c_ulonglong * 24)()
for fn in ("dpe_dbg_pool_stats_main", "dpe_dbg_pool_stats_tap", "dpe_dbg_pool_stats_f32"):
    getattr(lib, fn)(buf, 1)
assert lib.dpe_pm_execute(ctx, None) == 0, lib.dpe_last_error()
assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0, lib.dpe_last_error()
tot = [0] * 24
for fn in ("dpe_dbg_pool_stats_main", "dpe_dbg_pool_stats_tap", "dpe_dbg_pool_stats_f32"):
    getattr(lib, fn)(buf, 1)
    for k in range(24):
        tot[k] += buf[k]
print(f"Old NCC patches from LDS {tot[18]:12d}  slow (reciprocal range check failed) {tot[19]:12d} "
      f"= {100.0 * tot[19] / max(tot[18], 1):.2f}%", flush=True)
print(f"fast Old NCC lanes {tot[21]:12d}  failing taps_unclamped {tot[20]:12d} = {100.0 * tot[20] / max(tot[21], 1):.2f}%  "
      f"on the clamp-free path {tot[22]:12d} = {100.0 * tot[22] / max(tot[21], 1):.2f}%", flush=True)
for k in range(6):
    jobs, rounds, waves = tot[3 * k: 3 * k + 3]
    if waves:
        print(f"{NAMES[k]:26s} waves {waves:10d}  jobs/wave {jobs / waves:7.1f}  rounds/wave {rounds / waves:5.2f}  "
              f"lanes busy per round {jobs / max(rounds, 1):5.1f} of 64", flush=True)
lib.dpe_destroy(ctx)
