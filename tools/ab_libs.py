"""A/B of several builds of libdpe_mvs.so on the bench workload, interleaved in one process (the
scene is generated once).  Usage: python tools/ab_libs.py lib/variants/*.so"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402  (initialised before the libraries, as in bench.py)
torch.cuda.set_device(0)
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
st = synthetic.gt_state(sc)
libs = sys.argv[1:]
NOCHECK = os.environ.get("AB_NOCHECK") == "1"   # timing-only variants (e.g. stubbed phases)
ctxs = []
for path in libs:
    lib = native.load_library(path)
    ctx = lib.dpe_create(0)
    bufs = _abi.PassBuffers(inp, st)
    assert lib.dpe_pm_stage(ctx, C.byref(bufs.inp), C.byref(bufs.st)) == 0, lib.dpe_last_error()
    lib.dpe_set_timing(ctx, 1)
    ctxs.append((path, lib, ctx, bufs))
res = {path: [] for path in libs}
ref = None
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for path, lib, ctx, bufs in ctxs:
        assert lib.dpe_pm_execute(ctx, None) == 0, (path, lib.dpe_last_error())
        assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0
        out = b''.join(a.tobytes() for a in (bufs.planes, bufs.weak, bufs.sel, bufs.costs))
        if ref is None:
            ref = out
        if not NOCHECK:
            assert out == ref, f"{path}: output differs from {libs[0]}"
        buf = (C.c_float * 9)()
        lib.dpe_pm_last_timings(ctx, buf, 9)
        res[path].append([float(x) for x in buf])
# wall clock of untimed executes (per-class events off: the pass may then overlap streams)
import time  # noqa: E402
wall = {path: [] for path in libs}
for path, lib, ctx, bufs in ctxs:
    lib.dpe_set_timing(ctx, 0)
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for path, lib, ctx, bufs in ctxs:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            assert lib.dpe_pm_execute(ctx, None) == 0, (path, lib.dpe_last_error())
        assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0
        torch.cuda.synchronize()
        wall[path].append((time.perf_counter() - t0) / 5 * 1e3)
        if not NOCHECK:
            assert b''.join(a.tobytes() for a in (bufs.planes, bufs.weak, bufs.sel, bufs.costs)) == ref, f"{path}: untimed output differs from {libs[0]}"
names = ["total"] + native.CLASSES
for path in libs:
    best = min(res[path], key=lambda t: t[0])
    d = {k: round(v, 2) for k, v in zip(names, best)}
    d["wall_ms"] = round(min(wall[path]), 2)
    print(os.path.basename(path), json.dumps(d), flush=True)
