"""multiraft_amd — MI355X-native batched Multi-Raft decision engine.

The product is libmraft_hip.so (hand-written gfx950 HIP kernels behind the C
ABI in include/mraft.h); this package is its host-side mirror:
  * `engine.Engine`  — one handle per GPU: HBM-resident replica state and the
    batched decision entry points (AppendEntries, replies/commit, RequestVote,
    vote tally, the fused replication tick);
  * `persister`      — persister.go for every replica, fed by the engine's
    persist_dirty set (flush after a batch; crash + restart via readPersist);
  * `router`         — the shard router's view of the all-gathered GetState
    words (one RCCL all-gather per tick on multi-GPU).
"""
from ._abi import (CANDIDATE, DEVICE, FOLLOWER, HOST, LEADER, TICK_AUTO, TICK_FULL, TICK_LIGHT, synth_seed)  # noqa: F401
from .engine import (Engine, MraftError, copy_state, decode_persistent, entry_positions,  # noqa: F401
                     encode_persistent, new_state, state_sizes, synth_election_state,
                     synth_fold_batch, synth_tick_state)

__all__ = ["Engine", "MraftError", "new_state", "copy_state", "state_sizes", "synth_tick_state",
           "synth_fold_batch", "synth_election_state", "encode_persistent", "decode_persistent", "synth_seed", "LEADER", "CANDIDATE", "FOLLOWER", "HOST", "DEVICE",
           "TICK_FULL", "TICK_LIGHT", "TICK_AUTO"]
