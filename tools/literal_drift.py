"""How far the oracle's restatement choices 3, 7 and 8 (oracle/dpe_oracle.cpp header) move whole
passes and the whole 8-pass schedule, measured on the CPU against the ORACLE_LITERAL builds, which
evaluate ComputeHomography / ComputeCorrespondingPoint (DPE.cu:453-522) and tex2D(pt + 0.5f)
(DPE.cu:734-736, DPE.cpp:927-933) as the reference writes them (literal 1: IEEE division; literal 2:
a * (1 / b), a model of --use_fast_math's approximate division; both with choices 3, 7 and 8 off),
and against the ORACLE_RCP_IEEE build (choice 8 alone off: the tap reciprocal IEEE 1.0f / z instead of
the gfx950 v_rcp_f32 table).  Same inputs, same Philox seeds.

TEST INFRASTRUCTURE (uses the oracle only).  Usage:
    python tools/literal_drift.py [--threads T] [--out profiles/r04_literal_drift.json] [--sizes 160x120x3,320x240x5]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpe-mvs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from DPE_MVS import _abi, pipeline, synthetic  # noqa: E402

MODES = {"restated": None, "literal_ieee": 1, "literal_fastdiv": 2, "rcp_ieee": "rcp"}
COMPARED = ("literal_ieee", "literal_fastdiv", "rcp_ieee")
SEED = 0x5EED   # run_dpe_pipeline's default base_seed


def _lib(mode):
    if MODES[mode] is None:
        return oracle.lib()
    return oracle.rcp_ieee_lib() if MODES[mode] == "rcp" else oracle.literal_lib(MODES[mode])


def compare(depth_a, depth_b, normal_a=None, normal_b=None, weak_a=None, weak_b=None) -> dict:
    """Relative depth difference of b against a over pixels where both depths are > 0, the
    normal-angle difference there, and the weak-class agreement over all pixels."""
    da, db = np.asarray(depth_a, np.float64).ravel(), np.asarray(depth_b, np.float64).ravel()
    m = (da > 0) & (db > 0) & np.isfinite(da) & np.isfinite(db)
    rel = np.abs(db[m] - da[m]) / da[m]
    r = {"pixels": int(da.size), "compared": int(m.sum()),
         "rel_mean": float(rel.mean()) if rel.size else 0.0,
         "rel_median": float(np.median(rel)) if rel.size else 0.0,
         "rel_p90": float(np.percentile(rel, 90)) if rel.size else 0.0,
         "frac_rel_gt_1e-3": float((rel > 1e-3).mean()) if rel.size else 0.0,
         "frac_bit_identical": float((da == db).mean())}
    if normal_a is not None:
        na = np.asarray(normal_a, np.float64).reshape(-1, 3)[m]
        nb = np.asarray(normal_b, np.float64).reshape(-1, 3)[m]
        den = np.linalg.norm(na, axis=1) * np.linalg.norm(nb, axis=1)
        ok = den > 0
        cosang = np.clip((na[ok] * nb[ok]).sum(1) / den[ok], -1.0, 1.0)
        ang = np.degrees(np.arccos(cosang))
        r["normal_deg_mean"] = float(ang.mean()) if ang.size else 0.0
        r["normal_deg_median"] = float(np.median(ang)) if ang.size else 0.0
    if weak_a is not None:
        r["weak_agreement"] = float((np.asarray(weak_a).ravel() == np.asarray(weak_b).ravel()).mean())
    return r


def single_pass(W: int, H: int, n: int, threads: int) -> dict:
    """One REFINE_ITER + geom pass (BASELINE configs[2]'s pass type) from the same state."""
    sc = synthetic.make_scene(W, H, n)
    p = _abi.default_params()
    p.state = _abi.REFINE_ITER; p.geom_consistency = True; p.rotate_time = 2; p.ransac_threshold = 0.00875
    p.max_scale_size = 2; p.weak_peak_radius = 4
    st = synthetic.gt_state(sc, seed=W + H)
    inp = synthetic.pass_input(sc, p, depths=synthetic.src_depths(sc), seed=W * 7 + n)
    out = {m: oracle.run_pass(inp, st, threads, library=_lib(m)) for m in MODES}
    res = {}
    for m in COMPARED:
        a, b = out["restated"], out[m]
        # depth along the pixel ray is what the plane's w holds after the pass (GetDepthandNormal)
        res[m] = compare(a["planes"][..., 3], b["planes"][..., 3], a["planes"][..., :3], b["planes"][..., :3],
                         a["weak"], b["weak"])
    return res


def schedule(W: int, H: int, n: int, threads: int) -> dict:
    """The full coarse-to-fine schedule (main.cpp:474-600: 8 passes per reference image) through the
    host pipeline, the pass runner being each oracle build."""
    th = C.c_int(threads)
    tmp = tempfile.mkdtemp(prefix="litdrift_")
    try:
        base = os.path.join(tmp, "base")
        sc = synthetic.write_dense_folder(base, W, H, n)
        outs = {}
        # the control: the restatement itself under another base seed (PatchMatch's own spread)
        runs = [(m, m, SEED) for m in MODES] + [("restated_seed+1", "restated", SEED + 1)]
        for name, m, seed in runs:
            d = os.path.join(tmp, name)
            shutil.copytree(base, d)
            fn = _lib(m).oracle_pass_runner
            pipeline.run_dpe_pipeline(d, runner=(C.cast(fn, C.c_void_p), C.addressof(th)), normal=True, weak=True,
                                      verbose=False, base_seed=seed)
            outs[name] = {i: {f: np.load(os.path.join(d, "DPE", f"{i:08d}", f + ".npy")) for f in ("depth", "normal", "weak")}
                          for i in range(n)}
        cat = lambda o, f: np.concatenate([o[i][f].reshape(-1, *o[i][f].shape[2:]) for i in range(n)])  # noqa: E731
        res = {}
        for m in COMPARED + ("restated_seed+1",):
            a = outs["restated"]; b = outs[m]
            res[m] = compare(cat(a, "depth"), cat(b, "depth"), cat(a, "normal"), cat(b, "normal"), cat(a, "weak"),
                             cat(b, "weak"))
        # accuracy against the rendered ground truth (z depth of every reference image)
        gt = np.concatenate([np.asarray(v["depth"], np.float64).ravel() for v in sc["views"][:n]])
        acc = {}
        for m in outs:
            d = cat(outs[m], "depth").astype(np.float64).ravel()
            ok = np.isfinite(gt) & (gt > 0) & (d > 0)
            rel = np.abs(d[ok] - gt[ok]) / gt[ok]
            acc[m] = {"rel_median": float(np.median(rel)), "frac_within_1pct": float((rel < 1e-2).mean()),
                      "frac_within_1e-3": float((rel < 1e-3).mean()), "pixels": int(ok.sum())}
        res["vs_ground_truth"] = acc
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=oracle.host_threads())
    ap.add_argument("--sizes", default="160x120x3,320x240x5")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    report = {"what": "restated oracle vs the ORACLE_LITERAL builds (restatement choices 3, 7 and 8 off) and the "
                      "ORACLE_RCP_IEEE build (choice 8 alone off: IEEE tap reciprocal)", "cases": []}
    for spec in a.sizes.split(","):
        W, H, n = (int(v) for v in spec.split("x"))
        t0 = time.time()
        case = {"W": W, "H": H, "images": n, "single_pass": single_pass(W, H, n, a.threads),
                "schedule_8_pass": schedule(W, H, n, a.threads)}
        case["seconds"] = round(time.time() - t0, 1)
        report["cases"].append(case)
        print(json.dumps(case), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
