"""Generates the golden fixtures in this directory from the CPU restatement (oracle/).

Fixtures = inputs + expected outputs of complete PatchMatch passes on small synthetic scenes.
They pin the restatement against accidental change (tests/test_oracle_pass.py) and are the
expected values of the GPU parity tests (tests/test_gpu_parity.py).  Re-run only after a
deliberate, documented change of the restated semantics:
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from DPE_MVS import _abi, synthetic  # noqa: E402
import oracle  # noqa: E402

# v5 (round 5): restatement choice 8, the tap reciprocal as gfx950's v_rcp_f32 (oracle_math.h)
CASES = {
    # name: (W, H, num_images, pass kind)
    "first_init_64x48_v5": (64, 48, 3, "first"),
    "refine_init_64x48_v5": (64, 48, 3, "refine_init"),
    "refine_iter_geom_80x60_v5": (80, 60, 4, "refine_iter"),
}


def case_params(kind):
    p = _abi.default_params()
    if kind == "first":
        p.state = _abi.FIRST_INIT; p.use_APD = False; p.use_edge = False
    elif kind == "refine_init":
        p.state = _abi.REFINE_INIT; p.rotate_time = 2; p.ransac_threshold = 0.00875; p.max_scale_size = 2
        p.weak_peak_radius = 6
    else:
        p.state = _abi.REFINE_ITER; p.geom_consistency = True; p.rotate_time = 2; p.ransac_threshold = 0.00875
        p.max_scale_size = 2; p.weak_peak_radius = 4
    return p


def build_case(name):
    W, H, N, kind = CASES[name]
    sc = synthetic.make_scene(W, H, N)
    p = case_params(kind)
    depths = synthetic.src_depths(sc) if kind == "refine_iter" else None
    st = synthetic.first_init_state(sc) if kind == "first" else synthetic.gt_state(sc)
    inp = synthetic.pass_input(sc, p, depths=depths, seed=1234, pass_salt=7)
    return sc, inp, st


def params_to_dict(p):
    return {n: getattr(p, n) for n, _ in _abi.DpePatchMatchParams._fields_}


def cams_to_array(cams):
    out = []
    for c in cams:
        out.append(list(c.K) + list(c.R) + list(c.t) + list(c.c) + [c.height, c.width, c.depth_min, c.depth_max])
    return np.array(out, np.float64)


def main():
    for name in CASES:
        sc, inp, st = build_case(name)
        out = oracle.run_pass(inp, st)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            images=np.stack(inp["images"]).astype(np.uint8),
            cams=cams_to_array(inp["cams"]),
            depths=np.stack([np.zeros_like(inp["images"][0])] + list(inp["depths"][1:])) if inp["depths"] else np.zeros(0),
            edge=inp["edge"], edge_low=inp["edge_low"], label=inp["label"],
            params=np.array([repr(params_to_dict(inp["params"]))]), seed=inp["seed"], pass_salt=inp["pass_salt"],
            in_planes=st["planes"], in_weak=st["weak"], in_sel=st["sel"],
            out_planes=out["planes"], out_weak=out["weak"], out_sel=out["sel"], out_costs=out["costs"],
        )
        print("wrote", name)


if __name__ == "__main__":
    main()
