"""Shader-clock phase sums of the cooperative kernels (a -DDPE_DIAG=1 build of libdpe_mvs.so):
one bench-workload pass, the library prints 'PHASE kernel.phase cycles share' lines to stderr.
Usage: python tools/phase_prof.py lib/variants/phase.so"""
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
assert lib.dpe_pm_execute(ctx, None) == 0
assert lib.dpe_pm_fetch(ctx, C.byref(bufs.st)) == 0
