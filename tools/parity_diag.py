"""Diagnostic: runs a matrix of pass configurations through the HIP library and the CPU oracle
and prints per-output mismatch counts (localises a parity break to a pass stage)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from DPE_MVS import _abi, native, synthetic  # noqa: E402
import oracle  # noqa: E402


def configs():
    out = []
    for iters in (0, 1, 3):
        p = _abi.default_params(); p.state = _abi.FIRST_INIT; p.use_APD = False; p.use_edge = False
        p.max_iterations = iters
        out.append(("first_init_it%d" % iters, p, "first", False))
    for iters in (0, 1, 3):
        p = _abi.default_params(); p.state = _abi.REFINE_INIT; p.use_APD = True; p.use_edge = True
        p.max_iterations = iters; p.rotate_time = 2; p.ransac_threshold = 0.00875; p.max_scale_size = 2; p.weak_peak_radius = 6
        out.append(("refine_init_it%d" % iters, p, "gt", False))
    for iters in (0, 1, 3):
        p = _abi.default_params(); p.state = _abi.REFINE_ITER; p.use_APD = True; p.use_edge = True
        p.geom_consistency = True; p.max_iterations = iters; p.rotate_time = 2; p.ransac_threshold = 0.00875
        p.max_scale_size = 2; p.weak_peak_radius = 4
        out.append(("refine_iter_geom_it%d" % iters, p, "gt", True))
    return out


def main():
    W, H, N = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (96, 72, 4)))
    sc = synthetic.make_scene(W, H, N)
    depths = synthetic.src_depths(sc)
    ctx = native.PatchMatchContext(0)
    report = {}
    for name, p, init, geom in configs():
        st = synthetic.first_init_state(sc) if init == "first" else synthetic.gt_state(sc)
        inp = synthetic.pass_input(sc, p, depths=depths if geom else None)
        t0 = time.time(); g = ctx.run(inp, st); tg = time.time() - t0
        t0 = time.time(); o = oracle.run_pass(inp, st); to = time.time() - t0
        r = {}
        for k in ("planes", "weak", "sel", "costs"):
            a, b = g[k], o[k]
            if k in ("planes", "costs"):
                neq = ~((a.view(np.uint32) == b.view(np.uint32)))
            else:
                neq = a != b
            if neq.ndim == 3:
                neq = neq.any(-1)
            r[k] = int(neq.sum())
            if neq.any():
                ys, xs = np.nonzero(neq)
                r[k + "_first"] = [int(ys[0]), int(xs[0])]
        d = g["planes"][..., 3]; do = o["planes"][..., 3]
        r["max_rel_depth"] = float(np.nanmax(np.abs(d - do) / np.maximum(np.abs(do), 1e-6)))
        r["t_gpu"] = round(tg, 3); r["t_cpu"] = round(to, 3)
        report[name] = r
        print(name, json.dumps(r), flush=True)
    ctx.close()
    return report


if __name__ == "__main__":
    main()
