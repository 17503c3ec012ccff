#!/bin/bash
# Run a command and print its wall time (for gpu_run.sh's run: step, whose argument is split on
# whitespace without shell quoting): bash tools/timed.sh python -u bench.py
t0=$(date +%s%N)
"$@"; rc=$?
echo "wall_ms $(( ($(date +%s%N) - t0) / 1000000 )) rc $rc"
exit $rc
