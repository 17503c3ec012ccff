#!/bin/bash
# round 4, call R: GenNeighbours forked after RandomInitialization as well as the setup chain
# (DPE_GN_AFTER_RI) -- interleaved A/B of the overlapped wall time, then its timeline
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/gnri.so $V/gnric2.so > gpurun_out/r4r_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
DPE_MVS_LIB=$GRAFT_REPO_ROOT/$V/gnri.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04r_tl" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-instrument > "$GRAFT_REPO_ROOT/gpurun_out/r04r_tl_bench.log" 2>&1
