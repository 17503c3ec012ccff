#!/bin/bash
# round 5, call A: the knob clean-up build -- full -m gpu suite, smoke, bench
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_round2_a.sh r05a || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r05a_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05a_bench.log 2>&1
