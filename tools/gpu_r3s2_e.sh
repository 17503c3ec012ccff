# round 3 session 2, E: phase sums of the scratch-free GenNeighbours, probe batch sizes (bit-exact A/B)
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
V=dpe-mvs_amd/lib/variants
timeout -k 10 200 python -u tools/phase_prof.py $V/gnphase.so > gpurun_out/r4e_phase.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab_libs.py $V/gnl_s.so $V/gspec2.so $V/gspec1.so > gpurun_out/r4e_ab.log 2>&1
