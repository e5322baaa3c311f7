#!/bin/bash
# Register / scratch / occupancy of the kernels in one .hip file (device-only
# compile with -Rpass-analysis=kernel-resource-usage). Usage: tools/kres.sh FILE [name-filter] [extra hipcc flags]
f=$1; flt=${2:-.}; shift; shift
cd "$(dirname "$0")/../multiraft_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 --offload-device-only "$@" \
  -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep remark |
  awk '/Function Name/ {n=$(NF-1)} / VGPRs:/ {v=$(NF-1)} /TotalSGPRs/ {s=$(NF-1)} /ScratchSize/ {sc=$(NF-1)} /Occupancy/ {print n, "vgpr", v, "sgpr", s, "scratch", sc, "occ", $(NF-1)}' |
  grep -E "$flt"
