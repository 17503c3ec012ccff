#!/bin/bash
# round 5, call C: restatement choice 8 (tap reciprocal = v_rcp_f32) + the quarter-integer texel
# layouts -- interleaved timing A/B of the Newton / row-wise slow-loop variants, pool / line
# statistics, phase profile, then the full -m gpu suite, smoke and bench
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
AB_NOCHECK=1 AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/variants/newton.so dpe-mvs_amd/lib/variants/newton_row1.so dpe-mvs_amd/lib/variants/rcp_row1.so > gpurun_out/r05c_ab_rcp.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/pool_stats.py dpe-mvs_amd/lib/variants/pstat.so > gpurun_out/r05c_pool_stats.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/line_stats.py dpe-mvs_amd/lib/variants/pstat.so >> gpurun_out/r05c_pool_stats.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/phase_prof.py dpe-mvs_amd/lib/variants/phase.so > gpurun_out/r05c_phase.log 2>&1 || exit $?
bash tools/gpu_round2_a.sh r05c || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r05c_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05c_bench.log 2>&1
