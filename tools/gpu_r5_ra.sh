#!/bin/bash
# round 5, call RA: the build's phase profile, one-stream kernel trace + stats, overlapped timeline,
# and the bottleneck PMC passes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
tag=r05r
timeout -k 10 200 python -u tools/phase_prof.py dpe-mvs_amd/lib/variants/phase.so > gpurun_out/${tag}_phase.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${tag}_tl" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-instrument > "$R/gpurun_out/${tag}_tl_bench.log" 2>&1 || exit $?
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${tag}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types --no-pipeline > "$R/gpurun_out/${tag}_prof_bench.log" 2>&1 || exit $?
cd "$R" && bash tools/pmc_bottleneck.sh $tag
