#!/bin/bash
# round 4, call S: with GenNeighbours sharing the GPU with the first strong half-sweep (pixel-first
# walks), its instruction cuts again: 64-bit-product Philox, direction tables + fast angle test
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 500 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/ph64.so $V/gnopt.so $V/gnopt64.so > gpurun_out/r4s_ab.log 2>&1
