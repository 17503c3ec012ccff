#!/bin/bash
# Build A/B variants of lib/libdpe_mvs.so into dpe-mvs_amd/lib/variants/<name>.so (in parallel).
# Usage: tools/build_variants.sh "name:-DFLAG=1 -DOTHER=2" "base:" ...
cd "$(dirname "$0")/../dpe-mvs_amd" || exit 1
mkdir -p lib/variants
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w $flags -shared \
    -o lib/variants/$name.so csrc/dpe_mvs.hip -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
