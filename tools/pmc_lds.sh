#!/bin/bash
# LDS / issue PMC passes over one bench step (GPU box, repo root): bash tools/pmc_lds.sh TAG
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/pmcl${1:-}; mkdir -p $OUT; export TMPDIR=/tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "TA_BUSY_avr TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TOTAL_WAVEFRONTS_sum SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
)
i=0
for g in "${groups[@]}"; do
  DPE_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $OUT/g$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-instrument > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo PMC_DONE
