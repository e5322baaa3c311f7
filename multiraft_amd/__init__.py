"""multiraft_amd — MI355X-native batched Multi-Raft decision engine.

The product is libmraft_hip.so (hand-written gfx950 HIP kernels behind the C
ABI in include/mraft.h); this package is its host-side mirror:
  * `engine.Engine`  — one handle per GPU: HBM-resident replica state and the
    batched decision entry points (AppendEntries, replies/commit, RequestVote,
    vote tally, the fused replication tick);
  * `raft`           — the reference's per-instance API (Make / Start /
    GetState / handlers) for one group, driven through the same ABI, plus the
    deterministic 2B-scenario simulator.
"""
from ._abi import (CANDIDATE, DEVICE, FOLLOWER, HOST, LEADER, synth_seed)  # noqa: F401
from .engine import (Engine, MraftError, copy_state, new_state, state_sizes,  # noqa: F401
                     synth_election_state, synth_fold_batch, synth_tick_state)

__all__ = ["Engine", "MraftError", "new_state", "copy_state", "state_sizes", "synth_tick_state",
           "synth_fold_batch", "synth_election_state", "synth_seed", "LEADER", "CANDIDATE", "FOLLOWER", "HOST", "DEVICE"]
