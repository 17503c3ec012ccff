#!/usr/bin/env python3
"""Summarise rocprofv3 output of bench.py into profiles/ (markdown + JSON).

  kernel trace:  rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- python3 bench.py ...
  PMC traffic:   tools/pmc.sh TAG  (one rocprofv3 --pmc pass per counter group over one bench step)

Kernel durations: bench.py runs W warmup + K timed executes, then one hipEvent-timed execute and one
work-counting execute (device atomics).  The counting execute's dispatches are dropped (they are
slowed by the atomics), so the averages here are the ones bench.py's roofline uses.

HBM traffic (MI355X_MICROARCH.md § HBM): FETCH_SIZE and WRITE_SIZE are in KiB per dispatch; on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so bytes_read = 2 * 1024 * FETCH_SIZE and
bytes_written = 1024 * WRITE_SIZE.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re
import statistics


def short_name(name: str) -> str:
    name = name.strip('"')
    m = re.match(r"^(.*?)\(", name)
    base = m.group(1) if m else name
    base = base.replace("dpe::", "")
    return base[5:] if base.startswith("void ") else base


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def kernel_trace(dirname: str, execs: int, drop_last: int):
    paths = glob.glob(os.path.join(dirname, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no kernel_trace.csv under {dirname}")
    rows = read_csv(paths[0])
    per = collections.OrderedDict()
    meta = {}
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        k = short_name(r["Kernel_Name"])
        per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
        meta[k] = {"vgpr": r.get("VGPR_Count") or r.get("Arch_VGPR_Count"), "agpr": r.get("Accum_VGPR_Count"),
                   "scratch": r.get("Scratch_Size") or r.get("Private_Segment_Size"),
                   "lds": r.get("LDS_Block_Size") or r.get("Group_Segment_Size")}
    out = {}
    for k, d in per.items():
        kept = d
        if execs and len(d) % execs == 0 and drop_last:
            g = len(d) // execs
            kept = d[: len(d) - g * drop_last]
        out[k] = {"dispatches": len(kept), "mean_ms": statistics.fmean(kept), "median_ms": statistics.median(kept),
                  "min_ms": min(kept), "total_ms": sum(kept),
                  "per_execute_ms": sum(kept) / max(1, execs - drop_last) if execs and len(d) % execs == 0 else None,
                  **meta[k]}
    return out


def pmc_traffic(pmc_dir: str):
    res = collections.defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0, "dispatches": set()})
    for path in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in read_csv(path):
            name = r["Counter_Name"]
            if name not in ("FETCH_SIZE", "WRITE_SIZE"):
                continue
            k = short_name(r["Kernel_Name"])
            e = res[k]
            e["dispatches"].add((path, r["Dispatch_Id"]))
            e["fetch_kib" if name == "FETCH_SIZE" else "write_kib"] += float(r["Counter_Value"])
    out = {}
    for k, e in res.items():
        # FETCH and WRITE come from separate passes over the same single execute: dispatch count per pass
        n = max(1, len(e["dispatches"]) // 2)
        rd = 2 * 1024 * e["fetch_kib"] / n
        wr = 1024 * e["write_kib"] / n
        out[k] = {"dispatches_per_pass": n, "read_bytes_per_dispatch": rd, "write_bytes_per_dispatch": wr,
                  "hbm_bytes_per_dispatch": rd + wr}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--execs", type=int, required=True, help="total dpe_pm_execute calls in the traced bench run")
    ap.add_argument("--drop-last", type=int, default=1)
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--bench-json", default=None, help="the bench.py JSON line of the same run")
    ap.add_argument("--title", default="")
    ap.add_argument("--out-md", required=True)
    ap.add_argument("--out-json", required=True)
    a = ap.parse_args()
    kt = kernel_trace(a.trace, a.execs, a.drop_last)
    tr = pmc_traffic(a.pmc) if a.pmc else {}
    bench = None
    if a.bench_json and os.path.exists(a.bench_json):
        for line in open(a.bench_json):
            line = line.strip()
            if line.startswith("{"):
                bench = json.loads(line)
    lines = [f"# {a.title}", "",
             "Per-kernel dispatch durations from `rocprofv3 --kernel-trace --stats` (the work-counting execute dropped).",
             "HBM bytes from separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes over one execute, "
             "read = 2 x 1024 x FETCH_SIZE (gfx950 correction), write = 1024 x WRITE_SIZE.", "",
             "| kernel | dispatches | mean ms | median ms | min ms | ms / execute | trace VGPR field (x2 = VGPRs per lane, tools/ru.py) | scratch B | LDS B | HBM MB / dispatch |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for k, v in sorted(kt.items(), key=lambda kv: -kv[1]["total_ms"]):
        t = tr.get(k)
        hb = f"{t['hbm_bytes_per_dispatch'] / 1e6:.1f}" if t else "-"
        pe = f"{v['per_execute_ms']:.3f}" if v["per_execute_ms"] is not None else "-"
        lines.append(f"| {k} | {v['dispatches']} | {v['mean_ms']:.3f} | {v['median_ms']:.3f} | {v['min_ms']:.3f} | {pe} | "
                     f"{v['vgpr']} | {v['scratch']} | {v['lds']} | {hb} |")
    if bench:
        lines += ["", "bench.py line of the same run:", "", "```", json.dumps(bench), "```"]
    open(a.out_md, "w").write("\n".join(lines) + "\n")
    json.dump({"kernels": kt, "traffic": tr, "bench": bench}, open(a.out_json, "w"), indent=1)
    print(f"wrote {a.out_md}, {a.out_json}")


if __name__ == "__main__":
    main()
