#!/bin/bash
# round 5, call V: the weak sweep's texel layout for 8-bit images (U8 / F16 / P16) after the round-5
# weak changes -- interleaved A/B with output check
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/wu8.so $V/wf16.so $V/wp16.so > gpurun_out/r05v_ab_weaktex.log 2>&1
