# round 3 session 2, F: GenNeighbours with flattened direction walks against the nested walks (bit-exact
# A/B), then the parity suite on the in-tree (flattened) build
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 400 python -u tools/ab_libs.py $V/ec0.so $V/ec.so $V/ec5.so > gpurun_out/r4f_ab.log 2>&1 || exit $?
[ -n "$NOPAR" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_resident.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4f_parity.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4f_parity.log
exit $rc
