#!/bin/bash
# Round 3, call F: the -m gpu suite, the default bench line, then the ramp
# experiments at 32,768 groups (tools/gpu_r3e.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r3d.sh || exit 1
bash tools/gpu_r3e.sh || exit 1
