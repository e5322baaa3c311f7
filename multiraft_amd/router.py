"""Host-side shard router.

Each rank owns a contiguous range of groups; once per tick the GetState words
of every group (commitIndex, currentTerm<<1 | isLeader — mraft_export_group_status)
are all-gathered so every rank's router sees the whole deployment. This is the
replacement for polling GetState()/commit progress
(src/kvraft/server.go:114, src/shardkv/client.go:68-100). On the data path
the collective is the library's own RCCL all-gather over xGMI through the C
ABI (RcclFanIn: mraft_comm_init + mraft_allgather_status); the
torch.distributed helpers below (allgather_status*) are the host-side
rehearsal used by the gloo tests and the bench's check of the RCCL words.

The shard -> group assignment is the shard controller's Config
(src/shardctrler/common.go:27-132), applied as its state machine does
(server.go:124-162: Join / Leave / Move), with ReAllocGID and key2shard in
the library's host code (mraft_realloc_gid, mraft_key2shard).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _abi

NSHARDS = 10  # src/shardctrler/common.go:23


def key2shard(key, nshards: int = NSHARDS) -> int:
    """src/shardkv/client.go:22-29: first byte of the key modulo NShards."""
    b = key.encode() if isinstance(key, str) else bytes(key)
    r = _abi.lib().mraft_key2shard(b, len(b), nshards)
    if r < 0:
        raise ValueError("nshards must be positive")
    return r


def realloc_gid(shards, gids):
    """Config.ReAllocGID (common.go:87-132) on a copy: the new shard -> gid array."""
    sh = np.ascontiguousarray(shards, dtype=np.int32).copy()
    g = np.ascontiguousarray(sorted(gids), dtype=np.int32)
    rc = _abi.lib().mraft_realloc_gid(sh.ctypes.data, len(sh), g.ctypes.data if len(g) else None, len(g))
    if rc != _abi.OK:
        raise ValueError("ReAllocGID has no valid group to assign (only gid 0 configured)")
    return sh


@dataclass
class Config:
    """shardctrler.Config (common.go:27-31)."""
    num: int = 0
    shards: np.ndarray = field(default_factory=lambda: np.zeros(NSHARDS, np.int32))
    groups: dict = field(default_factory=dict)

    def copy_next(self) -> "Config":                  # CopyConfig, common.go:33-44
        return Config(self.num + 1, self.shards.copy(), dict(self.groups))


class ShardCtrlerState:
    """The shard controller's applied state machine (server.go:124-162,
    StartServer :166-171): configs[0] has no groups, every shard on gid 0."""

    def __init__(self, nshards: int = NSHARDS):
        self.configs = [Config(0, np.zeros(nshards, np.int32), {})]

    def join(self, servers: dict):                     # server.go:130-136
        c = self.configs[-1].copy_next()
        c.groups.update(servers)
        c.shards = realloc_gid(c.shards, c.groups.keys())
        self.configs.append(c)

    def leave(self, gids):                             # :137-143
        c = self.configs[-1].copy_next()
        for g in gids:
            c.groups.pop(g, None)
        c.shards = realloc_gid(c.shards, c.groups.keys())
        self.configs.append(c)

    def move(self, shard: int, gid: int):              # :144-147
        c = self.configs[-1].copy_next()
        c.shards[shard] = gid
        self.configs.append(c)

    def query(self, num: int = -1) -> Config:          # Query(-1) = latest
        return self.configs[-1] if num < 0 or num >= len(self.configs) else self.configs[num]


class RcclFanIn:
    """The fan-in over the library's RCCL communicator (include/mraft.h
    §multi-GPU fan-in). Rank 0 makes the communicator's unique id and the host
    control plane (here any torch.distributed group, e.g. gloo) ships the 128
    bytes to the other ranks; every rank then joins with mraft_comm_init."""

    def __init__(self, eng, rank: int, world: int, broadcast_id=None):
        from .engine import comm_unique_id
        uid = comm_unique_id() if rank == 0 else bytes(128)
        if world > 1:
            if broadcast_id is None:
                import torch.distributed as dist

                def broadcast_id(b):
                    box = [b]
                    dist.broadcast_object_list(box, src=0)
                    return box[0]
            uid = broadcast_id(uid)
        self.eng, self.rank, self.world = eng, rank, world
        self.comm = eng.comm_init(world, rank, uid)

    def gather(self, local, out, overlap: bool = True, ordered: bool = False):
        """local: [2*G] device block of this rank; out: [world*2*G] device.
        ordered: the caller already ordered the fan-in stream after the tick."""
        return self.eng.allgather_status(self.comm, local, out, overlap=overlap, ordered=ordered)

    def close(self):
        from .engine import comm_destroy
        if self.comm:
            comm_destroy(self.comm)
            self.comm = None


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


def allgather_status_packed(status_local, out=None):
    """One collective for both words: `status_local` is this rank's [2 * n]
    block (commitIndex[0:n] then term<<1|leader[n:2n], the layout the fused
    tick exports into when handed two halves of one buffer); returns the
    [world * 2 * n] gather, rank-major. unpack_status() splits it."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if out is None:
        out = torch.empty(world * status_local.numel(), dtype=status_local.dtype,
                          device=status_local.device)
    dist.all_gather_into_tensor(out, status_local.contiguous())
    return out


def unpack_status(packed, world: int):
    """(commit[world * n], term_leader[world * n]) from a packed gather."""
    v = packed.reshape(world, 2, -1)
    return v[:, 0, :].reshape(-1), v[:, 1, :].reshape(-1)


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
