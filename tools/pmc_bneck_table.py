"""Per-kernel bottleneck table from tools/pmc_bottleneck.sh output.
Usage: python tools/pmc_bneck_table.py gpurun_out/pmcbTAG"""
import collections
import csv
import glob
import re
import sys

res = collections.defaultdict(lambda: collections.defaultdict(float))
for path in glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv"):
    g = path.split("/")[-2]
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("dpe::", "").replace("void ", "")
        name = r["Counter_Name"]
        res[k][name if name != "GRBM_GUI_ACTIVE" else "GUI_" + g] += float(r["Counter_Value"])
keys = ["k_strong_coop<3, true>", "k_strong_coop<2, true>", "k_depth_to_weak<2>", "k_depth_to_weak<2, true>", "k_depth_to_weak_cols<2>",
        "k_weak_coop<1, 16>", "k_local_refine_jobs<2>", "k_gen_neighbours_lds<32>", "k_gen_neighbours",
        "k_random_init<2>", "k_ransac_fit", "k_gen_edge_inform"]
for k in keys:
    d = res.get(k)
    if not d:
        continue
    g0 = d["GUI_g0"] / 8; g1 = d["GUI_g1"] / 8; g2 = d["GUI_g2"] / 8; g3 = d["GUI_g3"] / 8
    cu_cyc = g0 * 256            # CU-cycles of the dispatch(es)
    print(f"== {k}  GUI/XCD {g0:.3g} cyc")
    print(f"  VALU issue/SIMD-cyc {4 * d['SQ_ACTIVE_INST_VALU'] / (1024 * g0):.2f} (SQ quad-cycles x4)  insts VALU {d['SQ_INSTS_VALU']:.3g}  VMEM_RD {d['SQ_INSTS_VMEM_RD']:.3g}  LDS {d['SQ_INSTS_LDS']:.3g}")
    print(f"  lanes/VALU {d['SQ_THREAD_CYCLES_VALU'] / max(1, d['SQ_ACTIVE_INST_VALU']):.1f}  wait_any {d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES'] * 100:.1f}%  wait_inst_any {d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES'] * 100:.1f}%  waves/SIMD {d['SQ_WAVE_CYCLES'] / (1024 * g0):.2f}")
    print(f"  TA_ADDR_FIFO_FULL/CU-cyc {d['SQ_VMEM_TA_ADDR_FIFO_FULL'] / (256 * g1):.3f}  TA_CMD_FIFO_FULL/CU-cyc {d['SQ_VMEM_TA_CMD_FIFO_FULL'] / (256 * g1):.3f}  VMEM level {d['SQ_INST_LEVEL_VMEM'] / max(1, d['SQ_INSTS_VMEM_RD']):.0f} cyc/inst")
    print(f"  TA busy {d['TA_BUSY_avr'] / g2:.2f}  TA addr stalled by TC/CU {d['TA_ADDR_STALLED_BY_TC_CYCLES_sum'] / (256 * g2):.2f}  TD busy/CU {d['TD_TD_BUSY_sum'] / (256 * g2):.2f}  TD_TC_STALL/CU {d['TD_TC_STALL_sum'] / (256 * g2):.2f}")
    print(f"  TCP: TA data stall/CU {d['TCP_TCP_TA_DATA_STALL_CYCLES_sum'] / (256 * g2):.2f}  pending stall/CU {d['TCP_PENDING_STALL_CYCLES_sum'] / (256 * g2):.2f}  TCR stall/CU {d['TCP_TCR_TCP_STALL_CYCLES_sum'] / (256 * g2):.2f}  tagconflict/CU {d['TCP_READ_TAGCONFLICT_STALL_CYCLES_sum'] / (256 * g2):.2f}")
    acc = d['TCP_TOTAL_CACHE_ACCESSES_sum']
    print(f"  TCP accesses/CU-cyc {acc / (256 * g3):.2f}  L1 miss->L2 {d['TCP_TCC_READ_REQ_sum'] / max(1, acc) * 100:.1f}%  L2 lat {d['TCP_TCC_READ_REQ_LATENCY_sum'] / max(1, d['TCP_TCC_READ_REQ_sum']):.0f} cyc  TA waves/CU-cyc {d['TA_TOTAL_WAVEFRONTS_sum'] / (256 * g3):.3f} flat-rd {d['TA_FLAT_READ_WAVEFRONTS_sum']:.3g}  TD load {d['TD_LOAD_WAVEFRONT_sum']:.3g} coalescable {d['TD_COALESCABLE_WAVEFRONT_sum']:.3g}")
