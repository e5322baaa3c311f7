"""The engine's N > 1 partition path on the GPU (VERDICT r4
item 6): two rank processes, spawned before this process makes any GPU call of
their own, each own a contiguous range of the groups of one seeded config-#3
shaped workload (`[rank*G, (rank+1)*G)` by global group index, as bench.py's
N > 1 lines shard config #4), create their own engine through the C ABI, split
their tick over two engine-owned shard queues (mraft_set_tick_shards(2)) and
run mraft_replicate_tick_export twice. They exchange the exported GetState
words over gloo (the host control plane; the RCCL all-gather needs one GPU
per rank, which this one-GPU box cannot give: profiles/r3_v11). The gathered
view must equal the oracle's GetState words over ALL groups (a single CPU
run of src/raft/raft_append_entry.go:20-162 on the unsharded workload), each
rank's state must equal the oracle's slice, and the shard router must answer
from the gathered view (src/shardkv/client.go:68-100,
src/shardkv/config.go:338-380: many groups at once, routed by the
shardctrler's Config)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD, G_RANK, P, L, TICKS, SEED = 2, 4096, 5, 4096, 2, 0xC0FFEE + 3

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import torch
        import torch.distributed as dist
        from oracle_lib import Oracle, assert_states_equal

        from multiraft_amd import DEVICE, Engine, synth_tick_state
        from multiraft_amd.router import GroupStatusView, allgather_status_packed, unpack_status
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        g0, g1 = rank * G_RANK, (rank + 1) * G_RANK
        st, lp, _ = synth_tick_state(WORLD * G_RANK, P, L, seed=SEED, g_begin=g0, g_end=g1)
        ora = Oracle(G_RANK, P, L, st)
        dev = torch.device("cuda", 0)
        lp_d = torch.from_numpy(lp).to(dev)
        status = torch.zeros(2 * G_RANK, dtype=torch.int32, device=dev)
        flags = torch.zeros(G_RANK, dtype=torch.int32, device=dev)
        words = []
        with Engine(G_RANK, P, L, device=0) as e:
            e.load_state(st)
            e.set_tick_shards(2)
            assert e.tick_shards() == 2
            for t in range(TICKS):
                e.replicate_tick_export(lp_d, flags, status[:G_RANK], status[G_RANK:], where=DEVICE)
                e.synchronize()
                ogf = ora.replicate_tick(lp)
                assert np.array_equal(flags.cpu().numpy(), ogf), (rank, t)
                local = status.cpu()
                gathered = allgather_status_packed(local)
                words.append(gathered.numpy().copy())
            assert_states_equal(e.store_state(), ora.state(), G_RANK, P, L, f"rank {rank} after {TICKS} ticks")
        c, tl = unpack_status(torch.from_numpy(words[-1]), WORLD)
        view = GroupStatusView(c.numpy(), tl.numpy())
        shard_to_group = np.arange(10) * (WORLD * G_RANK // 10) + 3
        routed = [view.route(k, shard_to_group) for k in ("", "a", "k17", "zz", "\x07x")]
        if rank == 0:
            q.put(("ok", words, routed))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:  # report, then fail the rank
        import traceback
        q.put(("error", rank, traceback.format_exc()))
        raise SystemExit(1) from ex


def test_two_rank_engine_partition_equals_oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle

    from multiraft_amd import synth_tick_state
    from multiraft_amd.router import GroupStatusView, unpack_status
    import torch

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        msg = q.get(timeout=300)
        assert msg[0] == "ok", f"rank {msg[1]} failed:\n{msg[2]}"
        _, words, routed = msg
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    # the oracle over all groups, unsharded
    st, lp, _ = synth_tick_state(WORLD * G_RANK, P, L, seed=SEED)
    ora = Oracle(WORLD * G_RANK, P, L, st)
    for t in range(TICKS):
        ora.replicate_tick(lp)
        c, tl = ora.export_group_status(lp)
        gc, gt = unpack_status(torch.from_numpy(words[t]), WORLD)
        assert np.array_equal(gc.numpy(), c), t
        assert np.array_equal(gt.numpy(), tl), t
    view = GroupStatusView(c, tl)
    shard_to_group = np.arange(10) * (WORLD * G_RANK // 10) + 3
    assert routed == [view.route(k, shard_to_group) for k in ("", "a", "k17", "zz", "\x07x")]
