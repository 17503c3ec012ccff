#!/bin/bash
# round 4, call M: the full -m gpu suite, smoke, the bench line and its one-stream kernel trace on the
# current default build, then GenNeighbours' slowest waves (timing build)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/gpu_final.sh r04m || exit $?
timeout -k 10 300 python -u tools/gn_times.py dpe-mvs_amd/lib/variants/gntimes3.so > gpurun_out/r04m_gn_times.log 2>&1
