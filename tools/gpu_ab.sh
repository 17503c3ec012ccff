# GPU run: A/B of the variant libraries on the bench workload (+ optional window statistics)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tag=${1:-ab}
shift
stats=""
libs=()
for a in "$@"; do case $a in *s_stats*) stats=$a;; *) libs+=($a);; esac; done
timeout -k 10 500 python -u tools/ab_libs.py "${libs[@]}" > gpurun_out/${tag}.log 2>&1 || exit $?
if [ -n "$stats" ]; then timeout -k 10 200 python -u tools/win_stats.py $stats >> gpurun_out/${tag}.log 2>&1; fi
