#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for lib in ${LIBS:-in-tree nodesc}; do
  if [ "$lib" = in-tree ]; then unset MRAFT_LIB; else export MRAFT_LIB=$PWD/tools/variants/libmraft_hip_$lib.so; fi
  echo "== $lib"
  timeout -k 10 200 python3 tools/dbg/ring2b.py 2>&1 | grep -E "trial|row" | head -12 || exit 1
done
