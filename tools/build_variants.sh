#!/bin/bash
# Builds tick-kernel variants as tools/variants/libmraft_hip_<tag>.so (same
# sources, different compile-time knobs); tools/ab_tick_pmc.sh and tools/ab_message_path.py time them.
# Each argument is  tag[@SRCDIR]=DEFINES  e.g.  "w6=-DMRAFT_TICK_MINW=6 -DMRAFT_TICK_CMP_EPL=2"
# or "head@/tmp/head/multiraft_amd/csrc=" (another source tree, e.g. git archive HEAD).
# TICK_ONLY=1: recompile only mraft_tick.hip per variant (the rest from build/).
set -e
cd "$(dirname "$0")/../multiraft_amd/csrc"
OUT=$(cd ../../tools && pwd)/variants
HERE=$(pwd)
mkdir -p "$OUT"
[ -n "$KEEP" ] || rm -f "$OUT"/*.so
build_one() {
  local spec="$1"
  cd "$HERE"
  tag=${spec%%=*}
  defs=${spec#*=}
  case "$tag" in *@*) cd "${tag#*@}"; tag=${tag%%@*};; esac
  mkdir -p build_$tag
  srcs="mraft_abi mraft_kernels mraft_tick mraft_elect"
  if [ -n "$TICK_ONLY" ] && [ "$(pwd)" = "$HERE" ]; then
    # only the tick differs: the other objects come from the in-tree build
    srcs="mraft_tick"
    for f in mraft_abi mraft_kernels mraft_elect; do cp build/$f.o build_$tag/; done
  fi
  for f in $srcs; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 \
      $defs -c $f.hip -o build_$tag/$f.o 2>/dev/null &
  done
  g++ -O3 -std=c++17 -fPIC -c mraft_persist.cpp -o build_$tag/mraft_persist.o &
  g++ -O3 -std=c++17 -fPIC -c mraft_router.cpp -o build_$tag/mraft_router.o &
  wait
  for f in mraft_abi mraft_kernels mraft_tick mraft_elect mraft_persist mraft_router; do
    [ -f build_$tag/$f.o ] || { echo "variant $tag: $f did not compile" >&2; rm -rf build_$tag; return 1; }
  done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT"/libmraft_hip_$tag.so build_$tag/*.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined || return 1
  rm -rf build_$tag
  printf "%s " "$tag"; /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 \
      $defs -Rpass-analysis=kernel-resource-usage -c mraft_tick.hip -o /dev/null 2>&1 | \
      grep -A9 "k_tick_groupILi5ELb0" | grep -E "VGPRs:|Scratch|Occupancy" | sed -E "s/.*(VGPRs|ScratchSize|Occupancy)[^:]*: ([0-9]+).*/\1=\2/" | tr "\n" " "; echo
}
# variants build in parallel (one compiler process per source file each)
for spec in "$@"; do build_one "$spec" > "$OUT/.log_${spec%%[=@]*}" 2>&1 & done
wait
cat "$OUT"/.log_*; rm -f "$OUT"/.log_*
