"""Timeline of one overlapped pass from a rocprofv3 --kernel-trace CSV (tools/gpu_run.sh TAG timeline): every
dispatch of the last pass with its start offset, duration and queue, then the busy time of each
queue and the span of the setup chain on the aux stream.

usage: python tools/timeline.py gpurun_out/<tag>_tl [pass_index_from_end=1]"""
import csv
import glob
import re
import sys


def short(n):
    n = n.strip('"')
    m = re.match(r"^(?:void )?(.*?)(\(|$)", n)
    return m.group(1).replace("dpe::", "")


def main():
    d = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
           r.get("Queue_Id") or r.get("Stream_Id") or "?") for r in rows]
    ks.sort()
        # (since round 6 a pass begins with k_pass_init, the initial state in one launch)
    pass_starts = [i for i, k in enumerate(ks) if k[2].startswith("k_pass_init")]
    if not pass_starts:   # older builds: the first k_list_count<0> of a pass precedes k_gen_edge_inform
        starts = [i for i, k in enumerate(ks) if k[2].startswith("k_list_count<0>")]
        pass_starts = [i for i in starts if i + 3 < len(ks) and any(ks[j][2].startswith("k_gen_edge_inform") for j in range(i, min(i + 6, len(ks))))]
    if len(pass_starts) < back:
        print("passes found:", len(pass_starts))
        return
    a = pass_starts[-back]
    b = pass_starts[-back + 1] if back > 1 else len(ks)
    seg = ks[a:b]
    t0 = seg[0][0]
    t1 = max(k[1] for k in seg)
    print(f"pass span {(t1 - t0) / 1e6:.3f} ms, {len(seg)} dispatches")
    busy = {}
    for s, e, n, q in seg:
        print(f"{(s - t0) / 1e6:8.3f} {(e - s) / 1e6:8.3f}  q{q:>3}  {n}")
        busy.setdefault(q, 0)
        busy[q] += e - s
    for q, v in busy.items():
        print(f"queue {q}: busy {v / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
