"""The bounds-checking build (MRAFT_DEBUG_BOUNDS, multiraft_amd/libmraft_hip_dbg.so,
built by __graft_entry__.build()): every dereference the streaming pass makes
through a source's or a follower row's 32-bit ring offset (mraft_pass.h at_u)
is counted when the offset is outside [-32, 2^30 - 32) — where it would wrap —
instead of trusting the construction (flat sources relative to their first
entry, the pass on rebased Indexes, capacities below MRAFT_MAX_LOG_CAPACITY).
A subprocess runs every Index-domain case (tests/index_domain_cases.py: the
tick and the message path through host buffers, in place, deferred, staged
and the ordered fallback, at the top of the Index domain and at ordinary
Indexes) on that library, GPU == oracle, and must report no violation."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(ROOT, "multiraft_amd", "libmraft_hip_dbg.so")


def test_no_ring_offset_out_of_range_gpu():
    assert os.path.exists(DBG), "build() makes the bounds-checking library"
    env = dict(os.environ, MRAFT_LIB=DBG)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "index_domain_cases.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(out["cases"]) >= 12 and all(c[-1] > 0 for c in out["cases"]), out["cases"]
    assert out["violations"] == {"mraft_debug_bounds_kernels": 0, "mraft_debug_bounds_tick": 0}, out
