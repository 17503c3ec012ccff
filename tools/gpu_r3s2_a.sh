# round 3 session 2, A: bit-exact A/B of the fract-weight taps and the scratch-free GenNeighbours
# against the round-3 build, then the parity suite on the scratch-free build
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 400 python -u tools/ab_libs.py $V/base.so $V/fract.so $V/pool.so $V/gnlds.so $V/d2w5.so > gpurun_out/r4a_ab.log 2>&1 || exit $?
cp $V/gnlds.so dpe-mvs_amd/lib/libdpe_mvs.so
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4a_parity.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4a_parity.log
exit $rc
