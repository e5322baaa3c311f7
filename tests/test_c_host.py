"""The boundary from a plain C host: tests/c_host/
mraft_host_tick.c includes only include/mraft.h (C11, -Wall -Wextra -Werror
-pedantic, no C++, no HIP header) and links libmraft_hip.so as a cgo binding
does. On each seeded tick vector it runs one replication
round four ways, each on a fresh engine: the fused tick
(set_tick_shards(2) -> replicate_tick_export), the same with
set_tick_mode(MRAFT_TICK_LIGHT) (ABI 6), the per-message sequence a Go
host drives (gather_append_args -> handle_append_entries_ex by reference ->
process_append_replies -> export_group_status), and the same with the entries
passed by value; every path's flags, GetState words and state are compared
with tests/golden/tick_vectors.bin — the committed tick_vectors.npz (expected
outputs from the pure-Python restatement of src/raft/raft_append_entry.go:
20-162) as a flat int32 file."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHOST = os.path.join(ROOT, "tests", "c_host")
BIN = os.path.join(CHOST, "mraft_host_tick")
FIXTURE = os.path.join(ROOT, "tests", "golden", "tick_vectors.bin")


def _build():
    r = subprocess.run(["make", "-s", "-C", CHOST], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_fixture_is_the_npz_vectors():
    """tick_vectors.bin is exactly tick_vectors_bin(tick_vectors.npz): the C
    host checks the same expected values as the Python tests."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden
    z = np.load(os.path.join(ROOT, "tests", "golden", "tick_vectors.npz"))
    assert open(FIXTURE, "rb").read() == make_golden.tick_vectors_bin(z)


def test_c_host_builds_pedantic():
    """The C11 host compiles with -Werror -pedantic against the header alone
    and links the in-tree library (no GPU needed to build)."""
    _build()
    assert os.access(BIN, os.X_OK)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "usage" in r.stderr  # argument check runs before any engine call


@pytest.mark.gpu
def test_c_host_tick_vectors_gpu():
    _build()
    r = subprocess.run([BIN, FIXTURE, "0"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 3 vectors" in r.stdout
    assert r.stdout.count("tick (2 shards), messages and by value") == 3 and r.stdout.count("bit-exact") == 3
