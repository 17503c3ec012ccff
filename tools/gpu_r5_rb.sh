#!/bin/bash
# round 5, call RB: the PMC traffic / issue passes of the build (tools/pmc.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
bash tools/pmc.sh r05r
