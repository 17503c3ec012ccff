# GPU run: the 1-GPU bench line, then a one-stream rocprofv3 kernel-trace summary of the same command
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${1:-r02}
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
DPE_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-pass-types > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_bench.log" 2>&1
