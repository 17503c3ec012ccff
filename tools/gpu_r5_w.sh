#!/bin/bash
# round 5, call W: the strong sweep's texel layout for 8-bit images (P16 / U8) -- interleaved A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 500 python -u tools/ab_libs.py $V/sp16.so $V/su8.so > gpurun_out/r05w_ab_strongtex.log 2>&1
