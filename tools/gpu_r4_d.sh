#!/bin/bash
# round 4, call D: GenNeighbours per-pixel / per-wave durations (-DDPE_GN_TIMES=1 build), an A/B of
# the default build against the lane-0 refinement draws (nopre) and the early geometric gather in
# DepthToWeak (gearly), then the one-stream kernel trace + stats of the bench and the PMC passes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 300 python -u tools/gn_times.py $V/gntimes.so > gpurun_out/r04d_gn_times.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/nopre.so $V/gearly.so > gpurun_out/r04d_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04d_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$GRAFT_REPO_ROOT/gpurun_out/r04d_prof_bench.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/pmc.sh r04d > gpurun_out/r04d_pmc.log 2>&1
