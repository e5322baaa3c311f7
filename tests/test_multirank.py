"""The N > 1 path on CPU: world-size-2 gloo. Each rank builds its shard of one
global seeded workload (by global group index), runs the tick (CPU oracle
stands in for the GPU here), exports GetState words and all-gathers them; the
gathered view must equal a single-process run over all groups, and the
router must answer from it."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, G, P, L, out_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from oracle_lib import Oracle

    from multiraft_amd import synth_tick_state
    from multiraft_amd.router import (GroupStatusView, allgather_status, allgather_status_packed,
                                      unpack_status)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st, lp, _ = synth_tick_state(G * world, P, L, seed=77, g_begin=rank * G, g_end=(rank + 1) * G)
    o = Oracle(G, P, L, st)
    o.replicate_tick(lp)
    c, tl = o.export_group_status(lp)
    all_c, all_t = allgather_status(torch.from_numpy(c), torch.from_numpy(tl))
    # the bench's single packed collective gives the same words
    pk_c, pk_t = unpack_status(allgather_status_packed(torch.from_numpy(np.concatenate([c, tl]))), world)
    assert torch.equal(pk_c, all_c) and torch.equal(pk_t, all_t)
    view = GroupStatusView(all_c.numpy(), all_t.numpy())
    shard_to_group = np.arange(10) * (G * world // 10)
    routed = view.route("k", shard_to_group)
    if rank == 0:
        out_q.put((all_c.numpy(), all_t.numpy(), routed))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_equal_single_process():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle

    from multiraft_amd import synth_tick_state
    from multiraft_amd.router import GroupStatusView
    G, P, L, world = 64, 5, 128, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, P, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    all_c, all_t, routed = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    st, lp, _ = synth_tick_state(G * world, P, L, seed=77)
    o = Oracle(G * world, P, L, st)
    o.replicate_tick(lp)
    c, tl = o.export_group_status(lp)
    assert np.array_equal(all_c, c) and np.array_equal(all_t, tl)
    view = GroupStatusView(c, tl)
    assert routed == view.route("k", np.arange(10) * (G * world // 10))


def test_key2shard():
    from multiraft_amd.router import key2shard
    assert key2shard("") == 0
    assert key2shard("a") == ord("a") % 10
    assert key2shard("zeta") == ord("z") % 10
