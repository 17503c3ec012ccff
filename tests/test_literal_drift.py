"""What the oracle's restatement choices cost: the restated oracle against its ORACLE_LITERAL builds
(oracle/dpe_oracle.cpp: ComputeHomography / ComputeCorrespondingPoint / tex2D(pt + 0.5f) evaluated as
DPE.cu:453-522, 734-736 write them; literal 1 with IEEE division, literal 2 with a * (1 / b) as a
model of --use_fast_math; choices 3, 7 and 8 off) and against the ORACLE_RCP_IEEE build (choice 8
alone off), same inputs and Philox seeds, through one pass and through the 8-pass coarse-to-fine
schedule (tools/literal_drift.py, numbers in DESIGN.md §4 and profiles/r06_rcp_choice8_drift.json).

Parity stays unpinned (no reference vectors): this measures the distance between the restatement
and the reference's literal float32 semantics, and sets it beside PatchMatch's own spread (the
restatement under another base seed) and beside the accuracy against the rendered ground truth.
The bounds are the measured levels at 160x120 (3 images) with headroom.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import literal_drift  # noqa: E402


@pytest.fixture(scope="module")
def threads():
    import oracle
    return min(8, oracle.host_threads())


def test_single_pass_drift(threads):
    # one REFINE_ITER + geom pass: ~93 % of the depths bit-identical, ~0.5 % beyond 1e-3 relative
    r = literal_drift.single_pass(160, 120, 3, threads)
    for m in literal_drift.COMPARED:
        d = r[m]
        assert d["frac_bit_identical"] > 0.85, (m, d)
        assert d["frac_rel_gt_1e-3"] < 0.01, (m, d)
        assert d["rel_median"] == 0.0, (m, d)
        assert d["weak_agreement"] > 0.995, (m, d)


def test_schedule_drift_within_patchmatch_spread(threads):
    # 8 passes per image: the flips compound (about a third of the depths end beyond 1e-3), but no
    # more than a change of the random seed moves the restatement itself, and the accuracy against
    # ground truth is the same
    r = literal_drift.schedule(160, 120, 3, threads)
    ctl = r["restated_seed+1"]
    for m in literal_drift.COMPARED:
        d = r[m]
        assert d["frac_rel_gt_1e-3"] <= 1.1 * ctl["frac_rel_gt_1e-3"], (m, d, ctl)
        assert d["rel_median"] <= 1.1 * ctl["rel_median"], (m, d, ctl)
        assert d["normal_deg_median"] <= 1.1 * ctl["normal_deg_median"], (m, d, ctl)
        assert d["weak_agreement"] >= ctl["weak_agreement"] - 0.005, (m, d, ctl)
    gt = r["vs_ground_truth"]
    base = gt["restated"]
    for m in literal_drift.COMPARED:
        assert abs(gt[m]["frac_within_1pct"] - base["frac_within_1pct"]) < 0.01, (m, gt)
        assert abs(gt[m]["rel_median"] - base["rel_median"]) < 0.05 * base["rel_median"], (m, gt)
