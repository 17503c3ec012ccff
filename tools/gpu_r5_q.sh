#!/bin/bash
# round 5, call Q: GenNeighbours held to fewer resident waves (dynamic LDS padding: 5 / 4 / 3 / 2 waves
# per SIMD) so that the first strong half-sweep shares the CUs in the pre-join window
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=5 timeout -k 10 600 python -u tools/ab_libs.py $V/gnp0.so $V/gnp4.so $V/gnp3.so $V/gnp2.so > gpurun_out/r05q_ab_gnpad.log 2>&1
