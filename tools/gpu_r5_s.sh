#!/bin/bash
# round 5, call S: v_cvt_i32_f32 against f2i on the device; weak neighbour loop unrolled x2 / x4 and
# the hardware f2i in an interleaved A/B (outputs checked)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/f2i_check > gpurun_out/r05s_f2i_check.log 2>&1 || exit $?
V=dpe-mvs_amd/lib/variants
AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_libs.py $V/nb1.so $V/nb2.so $V/nb4.so $V/f2ihw.so > gpurun_out/r05s_ab.log 2>&1
