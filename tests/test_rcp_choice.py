"""Which parity claims rest on device-derived semantics (restatement choice 8).

The oracle's tap reciprocal is the gfx950 v_rcp_f32 itself: a table dumped from the MI355X
(oracle/make_rcp_table.py, oracle/rcp_gfx950.bin.xz), a characterisation of the device, not a
restatement of the reference (which divides under --use_fast_math, DPE.cu:515-522,
CMakeLists.txt:72, with NVIDIA's own approximate reciprocal).  Every GPU == oracle bit-exact claim
therefore includes "the oracle's reciprocal is the device's" by construction.  This test runs the
ORACLE_RCP_IEEE build (choice 8 alone off: IEEE 1.0f / z, every other choice on) over the committed
golden inputs and checks that
  * the default build reproduces every golden fixture bit for bit (the fixtures are choice-8 outputs),
  * choice 8 really changes results on them (so the bit-exact GPU tests do depend on the table), and
  * what it changes stays inside the single-pass drift bounds of the literal builds
    (tests/test_literal_drift.py), i.e. PatchMatch's own seed-to-seed spread.
The whole-schedule numbers are in profiles/r06_rcp_choice8_drift.json (tools/literal_drift.py).
"""
import numpy as np
import pytest

import golden_io
import oracle

sys_names = golden_io.names()


def _drift(a, b):
    da = a["planes"][..., 3].astype(np.float64).ravel()
    db = b["planes"][..., 3].astype(np.float64).ravel()
    m = (da > 0) & (db > 0) & np.isfinite(da) & np.isfinite(db)
    rel = np.abs(db[m] - da[m]) / da[m]
    return {"frac_bit_identical": float((a["planes"].view(np.uint32) == b["planes"].view(np.uint32)).all(-1).mean()),
            "frac_rel_gt_1e-3": float((rel > 1e-3).mean()) if rel.size else 0.0,
            "weak_agreement": float((a["weak"] == b["weak"]).mean()),
            "sel_agreement": float((a["sel"] == b["sel"]).mean())}


@pytest.fixture(scope="module")
def runs():
    out = {}
    for name in sys_names:
        inp, st, exp = golden_io.load(name)
        on = oracle.run_pass(inp, st, threads=4)
        off = oracle.run_pass(inp, st, threads=4, library=oracle.rcp_ieee_lib())
        out[name] = (exp, on, off)
    return out


def test_goldens_are_choice8_outputs(runs):
    assert sys_names
    for name, (exp, on, _off) in runs.items():
        for k in ("planes", "weak", "sel", "costs"):
            assert golden_io.bits_equal(on[k], exp[k]), (name, k)


def test_choice8_changes_results(runs):
    # the device-derived table is load-bearing: with the IEEE reciprocal some output bits move
    changed = [name for name, (_e, on, off) in runs.items()
               if not all(golden_io.bits_equal(on[k], off[k]) for k in ("planes", "costs"))]
    assert changed, "choice 8 changed nothing on the goldens: the device table would not be load-bearing"


def test_choice8_drift_within_literal_bounds(runs):
    for name, (_e, on, off) in runs.items():
        d = _drift(on, off)
        # the literal builds' single-pass bounds (test_literal_drift.py::test_single_pass_drift)
        assert d["frac_bit_identical"] > 0.85, (name, d)
        assert d["frac_rel_gt_1e-3"] < 0.01, (name, d)
        assert d["weak_agreement"] > 0.995, (name, d)
