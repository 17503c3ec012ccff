#!/bin/bash
# round 4, call C: A/B of the refinement-draw variants, the resident exchange tests after the
# export/collective sync fix, the phase profile, an overlapped timeline and the bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 400 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/spre.so $V/wpre.so $V/swpre.so > gpurun_out/r04c_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_resident.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04c_resident.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/phase_prof.py $V/phase.so > gpurun_out/r04c_phase.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04c_tl" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-instrument > "$GRAFT_REPO_ROOT/gpurun_out/r04c_tl_bench.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04c_bench.log 2>&1
