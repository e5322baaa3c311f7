"""Shard router: key2shard and the shard controller's
ReAllocGID (src/shardkv/client.go:22-29, src/shardctrler/common.go:53-132) in
the library's host code, against hand-derived answers, the Python
restatement (oracle/pyoracle.py) and the assertions of
src/shardctrler/test_test.go (check(): every shard on a live group, loads
within one; minimal transfers after joins and leaves). CPU only."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyoracle as po  # noqa: E402

from multiraft_amd.router import NSHARDS, ShardCtrlerState, key2shard, realloc_gid  # noqa: E402


def test_key2shard():
    assert key2shard("hello") == ord("h") % 10
    assert key2shard("") == 0
    assert key2shard(b"\xff") == 255 % 10
    assert key2shard("a", 7) == ord("a") % 7


def test_realloc_kats():
    """Hand-derived from common.go:87-132 (ties break to the smallest gid;
    the join loop moves the FIRST shard of the most-loaded group)."""
    s = ShardCtrlerState()
    s.join({1: ["a"]})
    assert s.query().shards.tolist() == [1] * 10
    s.join({2: ["b"]})        # 1 -> 2 moves shards 0..4
    assert s.query().shards.tolist() == [2, 2, 2, 2, 2, 1, 1, 1, 1, 1]
    s.join({3: ["c"]})        # 5 (from 1), 0 (from 2), 6 (from 1) -> 3
    assert s.query().shards.tolist() == [3, 2, 2, 2, 2, 3, 3, 1, 1, 1]
    s.leave([2])              # 1,2,3,4 -> 1,3,1,3 (least loaded, smallest gid first)
    assert s.query().shards.tolist() == [3, 1, 3, 1, 3, 3, 3, 1, 1, 1]
    s.move(0, 1)              # server.go:144-147: no rebalance
    assert s.query().shards.tolist() == [1, 1, 3, 1, 3, 3, 3, 1, 1, 1]
    s.leave([1, 3])
    assert s.query().shards.tolist() == [0] * 10 and s.query().num == 6


def test_realloc_matches_restatement_random():
    rng = np.random.default_rng(7)
    for _ in range(2000):
        n = int(rng.integers(1, 16))
        pool = list(range(1, 20))
        gids = sorted(rng.choice(pool, size=int(rng.integers(1, 12)), replace=False).tolist())
        shards = rng.integers(0, 20, n).tolist()
        assert realloc_gid(shards, gids).tolist() == po.realloc_gid(shards, gids, n)


def _check(cfg, groups):
    """shardctrler/test_test.go:12-54."""
    assert sorted(cfg.groups) == sorted(groups)
    if groups:
        assert all(int(g) in cfg.groups for g in cfg.shards)
    counts = {g: int((cfg.shards == g).sum()) for g in cfg.groups}
    if counts:
        assert max(counts.values()) <= min(counts.values()) + 1


def test_reference_properties():
    """TestBasic / TestMulti's checks: balance after every op, and minimal
    transfers after joins and after leaves (test_test.go:211-250)."""
    npara = 10
    s = ShardCtrlerState()
    live = []
    for gid in range(1, npara + 1):
        s.join({gid: [f"s{gid}"]})
        live.append(gid)
        _check(s.query(), live)
    c1 = s.query()
    for i in range(5):
        gid = npara + 1 + i
        s.join({gid: [f"{gid}a"]})
        live.append(gid)
        _check(s.query(), live)
    c2 = s.query()
    for i in range(1, npara + 1):
        for j in range(NSHARDS):
            if c2.shards[j] == i:
                assert c1.shards[j] == i, "non-minimal transfer after Join()s"
    for i in range(5):
        s.leave([npara + 1 + i])
        live.remove(npara + 1 + i)
        _check(s.query(), live)
    c3 = s.query()
    for i in range(1, npara + 1):
        for j in range(NSHARDS):
            if c2.shards[j] == i:
                assert c3.shards[j] == i, "non-minimal transfer after Leave()s"


def test_only_invalid_group_is_rejected():
    with pytest.raises(ValueError):
        realloc_gid([0] * 10, [0])
