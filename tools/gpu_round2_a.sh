# GPU run: the -m gpu suite (every BASELINE config at its own shape), log under gpurun_out/
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 1140 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread --durations=0 > gpurun_out/${1:-r2}_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${1:-r2}_gputest.log
exit $rc
