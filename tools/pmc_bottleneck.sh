#!/bin/bash
# Bottleneck PMC passes (issue, TA/TD/TCP stalls, LDS) over one bench step, one rocprofv3 run per group.
# Run on the GPU box from the repo root: bash tools/pmc_bottleneck.sh TAG
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/pmcb${1:-}; mkdir -p $OUT; export TMPDIR=/tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_READ_sum TA_FLAT_READ_WAVEFRONTS_sum TA_TOTAL_WAVEFRONTS_sum TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum GRBM_GUI_ACTIVE"
)
i=0
for g in "${groups[@]}"; do
  DPE_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $OUT/g$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-instrument --no-e2e --no-pass-types --no-pipeline > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo PMC_DONE
