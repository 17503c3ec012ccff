"""Timing experiment: the pass without GenNeighbours on its critical path (DPE_DBG_GN_ONCE=1).

With the knob, the first execute after a stage runs GenNeighbours and keeps its outputs; later
executes of the same staged state skip it.  This script checks that a skipped execute gives the same
bits as the first one (GenNeighbours depends only on the staged state), then prints the mean wall
time of the skipped executes.  Run it once with and once without the knob (separate processes: the
knob is read once per process).  Usage: [DPE_DBG_GN_ONCE=1] python tools/gn_ceiling.py [reps]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
torch.cuda.set_device(0)
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
st = synthetic.gt_state(sc)
lib = native.load_library()
ctx = lib.dpe_create(0)
bufs = _abi.PassBuffers(inp, st)
assert lib.dpe_pm_stage(ctx, C.byref(bufs.inp), C.byref(bufs.st)) == 0, lib.dpe_last_error()


def run():
    assert lib.dpe_pm_execute(ctx, None) == 0, lib.dpe_last_error()
    assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0, lib.dpe_last_error()
    return b''.join(a.tobytes() for a in (bufs.planes, bufs.weak, bufs.sel, bufs.costs))


first = run()
second = run()
assert first == second, "an execute after the first gives different bits"
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    assert lib.dpe_pm_execute(ctx, None) == 0, lib.dpe_last_error()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps * 1e3
print(f"DPE_DBG_GN_ONCE={os.environ.get('DPE_DBG_GN_ONCE', '0')}: {dt:.3f} ms per execute ({reps} reps), "
      "bits of execute 2 == execute 1", flush=True)
lib.dpe_destroy(ctx)
