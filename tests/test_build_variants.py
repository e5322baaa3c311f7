"""The numeric knobs kept in the kernel sources (the losing code variants were
removed in round 5; git history keeps them) still compile for gfx950 at other
values: the tick at 6 waves per SIMD, dwordx2 compare chunks and 256-term
ConflictIndex scans, and its s_memrealtime trace build (tools/trace_tick.py);
the message path's grids at their smallest (one workgroup for the fold, the
deferred launch and each half of the fold's tail: every loop grid-strides).
CPU only (device-only compile, no GPU)."""
import os
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multiraft_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

VARIANTS = {
    "mraft_tick.hip": ["-DMRAFT_TICK_MINW=6", "-DMRAFT_TICK_CMP_EPL=2", "-DMRAFT_TICK_SCANU=4", "-DMRAFT_TICK_TRACE=1"],
    "mraft_kernels.hip": ["-DMRAFT_FOLD_GRID=1", "-DMRAFT_FOLD_TAIL_NL=1",
                          "-DMRAFT_FOLD_TAIL_NS=1"],
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("src", list(VARIANTS))
def test_alternatives_compile(src):
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c",
                        *VARIANTS[src], os.path.join(CSRC, src), "-o", os.devnull],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
