"""The compile-time alternatives kept in the kernel sources still compile for
gfx950. The tick's (each was measured against the default and
lost, and stays selectable for A/B runs, tools/build_variants.sh): the
unpipelined compare / copy loops, plain (temporal) loads and stores, two
dwordx4 per lane per compare chunk, the state pointers held across the pass,
linear group order, four groups per workgroup. The message path's grid knobs
at their smallest (one workgroup for the fold, the deferred launch and each
half of the fold's tail: every loop grid-strides). CPU only (device-only
compile, no GPU)."""
import os
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multiraft_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

VARIANTS = {
    "mraft_tick.hip": ["-DMRAFT_PASS_PIPE=0", "-DMRAFT_TICK_NT=0", "-DMRAFT_TICK_V=2", "-DMRAFT_TICK_RELOAD=0",
                       "-DMRAFT_TICK_XCD=0", "-DMRAFT_TICK_WPB=4", "-DMRAFT_TICK_MINW=6", "-DMRAFT_COPY_DEPTH=3"],
    "mraft_kernels.hip": ["-DMRAFT_TICK_NT=1", "-DMRAFT_FOLD_GRID=1", "-DMRAFT_AE_DGRID=1", "-DMRAFT_FOLD_TAIL_NL=1",
                          "-DMRAFT_FOLD_TAIL_NS=1"],
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("src", list(VARIANTS))
def test_alternatives_compile(src):
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c",
                        *VARIANTS[src], os.path.join(CSRC, src), "-o", os.devnull],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
