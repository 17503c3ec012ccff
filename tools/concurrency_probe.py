"""Throughput of K independent PatchMatch passes (different reference images) in flight at once on one
GPU, each on its own stream and context, vs one at a time.  Usage: python tools/concurrency_probe.py [K]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from DPE_MVS import _abi, native, synthetic  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
W, H, NV = 1600, 1200, 10
ctxs, streams = [], []
for k in range(K):
    sc = synthetic.make_scene(W, H, NV, seed=synthetic.SCENE_SEED + k)
    p = bench.workload_params(_abi, NV)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
    c = native.PatchMatchContext(0)
    c.stage(inp, synthetic.gt_state(sc))
    ctxs.append(c)
    streams.append(torch.cuda.Stream())
for c, s in zip(ctxs, streams):
    c.execute(s.cuda_stream)
torch.cuda.synchronize()
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    for c, s in zip(ctxs, streams):
        c.execute(s.cuda_stream)
        s.synchronize()
serial = (time.perf_counter() - t0) / (reps * K)
t0 = time.perf_counter()
for _ in range(reps):
    for c, s in zip(ctxs, streams):
        c.execute(s.cuda_stream)
    torch.cuda.synchronize()
conc = (time.perf_counter() - t0) / (reps * K)
print(f"K={K}: serial {serial*1e3:.1f} ms/pass ({W*H/serial/1e6:.2f} Mpix/s), concurrent {conc*1e3:.1f} ms/pass "
      f"({W*H/conc/1e6:.2f} Mpix/s)", flush=True)
