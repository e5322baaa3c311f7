"""Host-side shard router view.

Each rank owns a contiguous range of groups; once per tick the GetState words
of every group (commitIndex, currentTerm<<1 | isLeader — mraft_export_group_status)
are all-gathered so every rank's router sees the whole deployment. This is the
replacement for polling GetState()/commit progress
(src/kvraft/server.go:114, src/shardkv/client.go:68-100). The collective is
torch.distributed's all_gather_into_tensor: RCCL over xGMI for device tensors
(backend "nccl"), gloo for host tensors (tests).
"""
from __future__ import annotations

import numpy as np

NSHARDS = 10  # src/shardctrler/common.go:23


def key2shard(key: str, nshards: int = NSHARDS) -> int:
    """src/shardkv/client.go:22-29: first byte of the key modulo NShards."""
    shard = ord(key[0]) if key else 0
    return shard % nshards


def allgather_status(commit_local, term_leader_local):
    """All-gather the per-group status words of this rank's groups (torch
    tensors, same length on every rank) into global [world * G] tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n = commit_local.numel()
    all_c = torch.empty(world * n, dtype=commit_local.dtype, device=commit_local.device)
    all_t = torch.empty(world * n, dtype=term_leader_local.dtype, device=term_leader_local.device)
    dist.all_gather_into_tensor(all_c, commit_local.contiguous())
    dist.all_gather_into_tensor(all_t, term_leader_local.contiguous())
    return all_c, all_t


class GroupStatusView:
    """Global view of every group's (commitIndex, term, isLeader) words."""

    def __init__(self, commit: np.ndarray, term_leader: np.ndarray):
        self.commit = np.asarray(commit, dtype=np.int32)
        tl = np.asarray(term_leader, dtype=np.int32).view(np.uint32)
        self.term = (tl >> 1).astype(np.int64)
        self.is_leader = (tl & 1).astype(bool)

    def route(self, key: str, shard_to_group) -> tuple:
        """Group serving `key` under a shard->group assignment (the
        shardctrler Config.Shards array, common.go:27-31) and its status."""
        g = int(shard_to_group[key2shard(key, len(shard_to_group))])
        return g, int(self.commit[g]), int(self.term[g]), bool(self.is_leader[g])
