#!/bin/bash
# PMC passes over one bench step (run on the GPU box from the repo root): one rocprofv3
# invocation per counter group (never combined with trace domains).
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/pmc${1:-}; mkdir -p $OUT; export TMPDIR=/tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE SQ_LEVEL_WAVES"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
)
i=0
for g in "${groups[@]}"; do
  if [ -n "$PMC_GROUPS" ] && [[ " $PMC_GROUPS " != *" $i "* ]]; then i=$((i+1)); continue; fi
  DPE_OVERLAP=0 timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d $OUT/g$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-instrument --no-e2e --no-pass-types --no-pipeline > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo PMC_DONE
