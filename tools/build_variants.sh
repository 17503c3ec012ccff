#!/bin/bash
# Build A/B variants of lib/libdpe_mvs.so into dpe-mvs_amd/lib/variants/<name>.so (in parallel).
# Usage: tools/build_variants.sh "name:-DFLAG=1 -DOTHER=2" "base:" ...
# The flags apply to all three translation units; TAP_SCHED / F32_SCHED (env) override the
# schedulers of csrc/tap_launch.hip / csrc/tap_f32.hip (defaults: the Makefile's); flags after a
# second colon ("name:all flags:main-unit flags") apply to csrc/dpe_mvs.hip only, which always gets
# the Makefile's MAIN_FLAGS (-fno-slp-vectorize; MAIN_FLAGS in the environment overrides).
cd "$(dirname "$0")/../dpe-mvs_amd" || exit 1
mkdir -p lib/variants obj/variants
TAP_SCHED=${TAP_SCHED-}
F32_SCHED=${F32_SCHED--mllvm -amdgpu-sched-strategy=iterative-maxocc}
MAIN_FLAGS=${MAIN_FLAGS--fno-slp-vectorize}
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w"
build() {
  local name=$1 flags=${2%%:*} mflags=
  [[ $2 == *:* ]] && mflags=${2#*:}
  /opt/rocm/bin/hipcc $HF $MAIN_FLAGS $flags $mflags -c -o obj/variants/$name.main.o csrc/dpe_mvs.hip &
  local a=$!
  /opt/rocm/bin/hipcc $HF $flags $TAP_SCHED -c -o obj/variants/$name.tap.o csrc/tap_launch.hip &
  local b=$!
  /opt/rocm/bin/hipcc $HF $flags $F32_SCHED -c -o obj/variants/$name.f32.o csrc/tap_f32.hip &
  local c=$!
  wait $a && wait $b && wait $c || return 1
  /opt/rocm/bin/hipcc $HF -shared -o lib/variants/$name.so obj/variants/$name.main.o obj/variants/$name.tap.o \
    obj/variants/$name.f32.o \
    -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
}
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build "$name" "$flags" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
