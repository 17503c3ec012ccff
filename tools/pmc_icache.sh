#!/bin/bash
# Instruction-cache PMC pass over one bench step (DPE_OVERLAP=0): SQC I-cache hits/misses and
# instruction fetches per kernel.  Run on the GPU box from the repo root: bash tools/pmc_icache.sh TAG
set -o pipefail
R=$PWD; OUT=$R/gpurun_out/pmci${1:-}; mkdir -p $OUT; export TMPDIR=/tmp
g="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
DPE_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $OUT/g0 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-instrument --no-e2e --no-pass-types > $OUT/g0.log 2>&1 || { echo "pass failed"; exit 1; }
echo PMC_DONE
