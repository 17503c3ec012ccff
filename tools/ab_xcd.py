"""A/B of the XCD chunk knob (DPE_XCD_ROWS) on the bench workload, interleaved in one process."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
import bench
from DPE_MVS import _abi, native, synthetic
sc = synthetic.make_scene(1600, 1200, 10)
p = bench.workload_params(_abi, 10)
inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc))
ctx = native.PatchMatchContext(0)
ctx.stage(inp, synthetic.gt_state(sc))
ctx.set_timing(True)
variants = [int(v) for v in (sys.argv[1:] or ["0", "1", "4", "16"])]
res = {v: [] for v in variants}
for rnd in range(3):
    for v in variants:
        os.environ["DPE_XCD_ROWS"] = str(v)
        ctx.execute(); ctx.fetch()
        res[v].append(ctx.timings())
for v in variants:
    best = min(res[v], key=lambda t: t["total"])
    print("xcd_rows", v, json.dumps({k: round(x, 2) for k, x in best.items()}))
