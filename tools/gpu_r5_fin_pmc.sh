#!/bin/bash
# round 5: PMC traffic and bottleneck passes of the final build
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
bash tools/pmc.sh ${1:-r05f} && bash tools/pmc_bottleneck.sh ${1:-r05f}
