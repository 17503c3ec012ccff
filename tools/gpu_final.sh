# GPU run: A/B of two variant libraries, then the full -m gpu suite, smoke and the bench line +
# one-stream kernel trace of the in-tree build (logs under gpurun_out/)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=$1; shift
if [ $# -ge 2 ]; then AB_ROUNDS=6 bash tools/gpu_ab.sh ab_$tag "$@" || exit $?; fi
bash tools/gpu_round2_a.sh $tag || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
bash tools/gpu_bench.sh $tag
