"""Per-kernel derived PMC metrics from tools/pmc.sh output (VALU busy, lane utilisation, HBM bytes).
Usage: python tools/pmc_table.py gpurun_out/pmcTAG"""
import collections
import csv
import glob
import re
import sys

res = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("dpe::", "").replace("void ", "")
        res[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
print(f"{'kernel':34s} {'VALU/SIMD-cyc':>13s} {'lanes/64':>8s} {'VALUinst':>10s} {'waitany%':>8s} {'HBM MB':>8s} {'TA busy':>7s}")
for k, d in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if d.get("SQ_WAVE_CYCLES", 0) == 0 and d.get("FETCH_SIZE", 0) == 0:
        continue
    gui = d.get("GRBM_GUI_ACTIVE", 0) / 8.0       # cycles per XCD, summed over dispatches
    busy = 4 * d.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * gui) if gui else float("nan")
    lanes = d.get("SQ_THREAD_CYCLES_VALU", 0) / d["SQ_ACTIVE_INST_VALU"] if d.get("SQ_ACTIVE_INST_VALU") else float("nan")
    wait = d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"] * 100 if d.get("SQ_WAVE_CYCLES") else float("nan")
    hbm = (2 * 1024 * d.get("FETCH_SIZE", 0) + 1024 * d.get("WRITE_SIZE", 0)) / 1e6
    ta = d.get("TA_BUSY_avr", 0) / gui if gui and "TA_BUSY_avr" in d else float("nan")
    print(f"{k[:34]:34s} {busy:13.2f} {lanes:8.1f} {d.get('SQ_INSTS_VALU', 0):10.3g} {wait:8.1f} {hbm:8.1f} {ta:7.2f}")
