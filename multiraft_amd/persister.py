"""Host-side persistence driven by the engine's persist_dirty set
(SURVEY.md §5 "Checkpoint / resume", §8f #4).

`Persister` mirrors src/raft/persister.go:14-76 (one byte blob of raft state
and one of snapshot per replica). `flush_persist` is what the reference's
`persist()` / `SaveStateAndSnapshot()` call sites (raft.go:205-216,
raft_snapshot.go:12,47) do, batched: after a batch of engine calls it reads
every replica the engine marked (mraft_collect_persist), encodes its
currentTerm / votedFor / log terms (mraft_read_persistent +
mraft_encode_persistent) and stores the bytes. `restart` is crash + Make +
readPersist (raft.go:51-87,217-235) through mraft_restore. Commands are not
engine state: a host keeps them beside the bytes, index-aligned.
"""
from __future__ import annotations

import numpy as np

from ._abi import PERSIST_SNAPSHOT, PERSISTENT
from .engine import decode_persistent, encode_persistent


class Persister:
    """persister.go for G*P replicas: per slot a raftstate blob and a
    snapshot blob."""

    def __init__(self, n_slots: int):
        self.raftstate = [b""] * n_slots
        self.snapshot = [b""] * n_slots

    def copy(self) -> "Persister":                      # persister.go:30-37
        p = Persister(0)
        p.raftstate = list(self.raftstate)
        p.snapshot = list(self.snapshot)
        return p

    def save_raft_state(self, slot: int, state: bytes):  # :39-43
        self.raftstate[slot] = bytes(state)

    def save_state_and_snapshot(self, slot: int, state: bytes, snapshot: bytes):  # :58-63
        self.raftstate[slot] = bytes(state)
        self.snapshot[slot] = bytes(snapshot)

    def read_raft_state(self, slot: int) -> bytes:      # :45-49
        return self.raftstate[slot]

    def read_snapshot(self, slot: int) -> bytes:        # :65-69
        return self.snapshot[slot]

    def raft_state_size(self, slot: int) -> int:        # :51-55
        return len(self.raftstate[slot])


def flush_persist(engine, persister: Persister, snapshot_bytes=None) -> np.ndarray:
    """Saves every replica the engine marked since the last flush. For a
    MRAFT_PERSIST_SNAPSHOT mark the snapshot bytes come from
    snapshot_bytes(slot) (the service's bytes for Snapshot, the leader's for
    an installed InstallSnapshot). Returns the flushed slots."""
    bits = engine.collect_persist()
    slots = np.nonzero(bits)[0].astype(np.int32)
    if len(slots) == 0:
        return slots
    hdr, terms = engine.read_persistent(slots)
    for i, s in enumerate(slots):
        n = int(hdr["last_index"][i] - hdr["dummy_index"][i] + 1)
        off = int(hdr["terms_offset"][i])
        data = encode_persistent(hdr[i], terms[off:off + n])
        if bits[s] & PERSIST_SNAPSHOT:
            snap = snapshot_bytes(int(s)) if snapshot_bytes else b""
            persister.save_state_and_snapshot(int(s), data, snap)
        else:
            persister.save_raft_state(int(s), data)
    return slots


def restart(engine, persister: Persister, slots) -> np.ndarray:
    """Crash + restart of the given replicas from their persisted bytes
    (Make + readPersist). A replica with no persisted state restarts as
    Make leaves it (readPersist returns early on empty data, raft.go:218-220).
    Returns the per-slot item_err of mraft_restore."""
    slots = np.asarray(slots, dtype=np.int32)
    hdr = np.zeros(len(slots), dtype=PERSISTENT)
    parts, off = [], 0
    for i, s in enumerate(slots):
        data = persister.read_raft_state(int(s))
        if data:
            rec, t = decode_persistent(data)
            for f in ("current_term", "voted_for", "dummy_index", "last_index"):
                hdr[f][i] = rec[f]
        else:
            t = np.zeros(1, np.int32)                   # Make: term 0, votedFor -1, [dummy{0,0}]
            hdr["voted_for"][i] = -1
        hdr["slot"][i] = s
        hdr["terms_offset"][i] = off
        parts.append(t)
        off += len(t)
    return engine.restore(hdr, np.concatenate(parts) if parts else np.zeros(0, np.int32))
