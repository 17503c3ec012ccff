#!/bin/bash
# round 4, call J: bottleneck PMC passes of the default build (one bench step, one stream), then the
# 2-rank gloo rehearsal of bench.py's N > 1 line (exchange decomposition)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/pmc_bottleneck.sh r04 > gpurun_out/r4j_pmcb.log 2>&1 || exit $?
python tools/pmc_bneck_table.py gpurun_out/pmcbr04 > gpurun_out/r4j_pmcb_table.txt 2>&1
bash tools/gpu_multirank_rehearsal.sh r04
