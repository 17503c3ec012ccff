# GPU run: a subset of the -m gpu suite given as pytest node ids / files (log under gpurun_out/)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread --durations=10 > gpurun_out/${tag}.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${tag}.log
exit $rc
