"""Gather locality of the tap kernels (a -DDPE_DIAG=2 build of libdpe_mvs.so): distinct 128-B
lines per wave gather and the sum over lane quads of the lines each quad touches (the TA cost, tools/td_probe2.hip), per texel layout (P16: strong sweep; F16: DepthToWeak +
LocalRefine + RandomInitialization; U8: weak sweep), one timed bench-workload pass.
Usage: python tools/line_stats.py lib/variants/lstat.so"""
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

sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
st = synthetic.gt_state(sc)
lib = native.load_library(sys.argv[1])
ctx = lib.dpe_create(0)
bufs = _abi.PassBuffers(inp, st)
assert lib.dpe_pm_stage(ctx, C.byref(bufs.inp), C.byref(bufs.st)) == 0
lib.dpe_set_timing(ctx, 1)
buf = (C.c_ulonglong * 16)()
for fn in ("dpe_dbg_line_stats_main", "dpe_dbg_line_stats_tap", "dpe_dbg_line_stats_f32"):
    getattr(lib, fn)(buf, 1)
rc = lib.dpe_pm_execute(ctx, None)
assert rc == 0, (rc, lib.dpe_last_error())
assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0, lib.dpe_last_error()
tot = [0] * 16
for fn in ("dpe_dbg_line_stats_main", "dpe_dbg_line_stats_tap", "dpe_dbg_line_stats_f32"):
    getattr(lib, fn)(buf, 1)
    if buf[1]:   # row 0: the clamp-free choice of ELIDE builds, per translation unit
        print(f"{fn}: clamp-free choice: wave calls {buf[1]:.3e}, all lanes inside {buf[0] / buf[1]:.3f}, "
              f"lanes inside {buf[2] / max(buf[3], 1):.3f}", flush=True)
    for k in range(16):
        tot[k] += buf[k]
for t, name in ((1, "U8 (weak sweep)"), (2, "F16 (DepthToWeak, LocalRefine, init)"), (3, "P16 (strong sweep)")):
    n, nl, ns, act = tot[4 * t: 4 * t + 4]
    if n:
        print(f"{name:40s} wave gathers {n:.3e}  lines/gather {nl / n:6.2f}  quad lines/gather (TA cycles) {ns / n:6.2f}  "
              f"active lanes {act / n:5.1f}", flush=True)
lib.dpe_destroy(ctx)
