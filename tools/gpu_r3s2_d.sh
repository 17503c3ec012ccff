# round 3 session 2, D: the scratch-free GenNeighbours variants against the default build (bit-exact A/B)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 500 python -u tools/ab_libs.py $V/lr.so $V/gnl_nsdp.so $V/gnl_s.so $V/gnl_s6.so $V/gnl_s128.so > gpurun_out/r4d_ab.log 2>&1
