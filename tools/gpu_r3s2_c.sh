# round 3 session 2, C: how often the clamp-free tap loop's wave-uniform choice holds (strong sweep,
# DepthToWeak; DPE_LINE_STATS builds)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 200 python -u tools/line_stats.py $V/selst.so > gpurun_out/r4c_stats.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/line_stats.py $V/d2wst.so >> gpurun_out/r4c_stats.log 2>&1
