# round 3 session 2, B: bit-exact A/B of LocalRefine coordinates from LDS, F16 texels for the strong
# sweep and the clamp-free tap loops (strong / LocalRefine) on the fract-weight build
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 500 python -u tools/ab_libs.py $V/fract.so $V/lr.so $V/sf16.so $V/se.so $V/lre.so > gpurun_out/r4b_ab.log 2>&1
