# GPU run: the -m gpu suite, then the 1-GPU bench unless the suite crashed or timed out
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2_gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-e2e > gpurun_out/r2_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r2_bench.log
