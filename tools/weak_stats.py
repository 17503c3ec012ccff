"""Weak-sweep path statistics (a -DDPE_DIAG=4 build of libdpe_mvs.so) over one bench-workload
pass: centre-patch sides and paths of the NCC-New jobs, neighbour-patch paths, and the distinct
centre-patch variants a wave executes one after another.
Usage: python tools/weak_stats.py lib/variants/wstat.so"""
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
buf = (C.c_ulonglong * 24)()
lib.dpe_dbg_weak_stats(buf, 1)
rc = lib.dpe_pm_execute(ctx, None)
assert rc == 0, (rc, lib.dpe_last_error())
assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0, lib.dpe_last_error()   # joins the pass's streams
lib.dpe_dbg_weak_stats(buf, 1)
s = list(buf)
jobs = max(1, s[0])
print(f"NCC-New jobs {s[0]}  centre outside {s[1] / jobs:.3f}")
cen = sum(s[2:12])
print("centre patch side n_c: " + "  ".join(f"{n}:{s[2 + n] / max(1, cen):.3f}" for n in range(10) if s[2 + n]))
print(f"centre untabulated {s[12] / max(1, cen):.3f}  tabulated with the slow reciprocal {s[13] / max(1, cen):.3f}")
print(f"neighbour box fast {s[14] / jobs:.3f} of jobs  neighbour patches/job {s[15] / jobs:.2f}  generic {s[16] / max(1, s[15]):.3f}")
print(f"centre variants per wave call {s[17] / max(1, s[18]):.2f}  active lanes per wave call {s[19] / max(1, s[18]):.1f}", flush=True)
lib.dpe_destroy(ctx)
