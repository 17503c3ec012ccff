#!/bin/bash
# round 5, call P: coarse pyramid levels on the F32 path (quarter-integer class off) and on the
# half-precision layouts, then the 2-rank gloo rehearsal of the N > 1 bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
DPE_MVS_LIB=$V/noq.so timeout -k 10 300 python -u tools/levels.py > gpurun_out/r05p_levels.log 2>&1 || exit $?
DPE_MVS_LIB=$V/withq.so timeout -k 10 300 python -u tools/levels.py >> gpurun_out/r05p_levels.log 2>&1 || exit $?
DPE_MVS_LIB=$V/noq.so timeout -k 10 300 python -u tools/levels.py >> gpurun_out/r05p_levels.log 2>&1 || exit $?
DPE_MVS_LIB=$V/withq.so timeout -k 10 300 python -u tools/levels.py >> gpurun_out/r05p_levels.log 2>&1 || exit $?
bash tools/gpu_multirank_rehearsal.sh r05
