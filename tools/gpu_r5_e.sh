#!/bin/bash
# round 5, call E: the generic slow-patch form (restatement choice 8) -- full -m gpu suite, smoke,
# bench and the kernel-trace summary of the bench command
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_round2_a.sh r05e || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r05e_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05e_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05e_prof -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r05e_prof.log 2>&1
