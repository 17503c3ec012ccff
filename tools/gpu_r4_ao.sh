#!/bin/bash
# round 4, call AO: GenNeighbours' direction table and fast angle test again, now that the pre-join
# window is throughput-bound (they measured nothing while GenNeighbours' tail was critical) -- A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=6 timeout -k 10 600 python -u tools/ab_libs.py dpe-mvs_amd/lib/libdpe_mvs.so $V/dirtab.so $V/fastangle.so $V/dirfast.so > gpurun_out/r4ao_ab.log 2>&1
