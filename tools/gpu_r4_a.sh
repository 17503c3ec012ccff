#!/bin/bash
# round 4, call A: interleaved A/B of the fused DepthToWeak + LocalRefine against the unfused build
# (bit-identical outputs asserted), the -m gpu suite on the in-tree (fused) build, then the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_libs.py dpe-mvs_amd/lib/variants/nofuse.so dpe-mvs_amd/lib/libdpe_mvs.so dpe-mvs_amd/lib/variants/spre.so > gpurun_out/r04_ab_fuse_lr.log 2>&1 || exit $?
bash tools/gpu_round2_a.sh r04a || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-e2e --no-pipeline > gpurun_out/r04a_bench.log 2>&1
