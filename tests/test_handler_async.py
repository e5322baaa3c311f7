"""The message-level AppendEntries handler with no host round trip (VERDICT r4
item 1): mraft_handle_append_entries[_ex] by reference enqueues its three
launches and returns, whatever the batch; items that must run after others
are ordered on the device (include/mraft.h, mraft_kernels.hip "a4").

* K message steps (gather -> HandleAppendEntries -> reply fold,
  src/raft/raft_append_entry.go:20-162) enqueued back to back on one engine
  behind a device spin, with no host synchronisation: the calls return while
  the stream is still busy, and every step's outputs equal K oracle steps.
* Batches whose items read rows other items write, in rings of 2 and 3 stale
  leaders and with crafted self-references (cycles of deferred items), with
  the default stage, a stage too small for the batch and no stage at all (the
  ordered fallback): GPU == oracle (which copies every item's entries at the
  start of the call, as the reference's gather does, raft_append_entry.go:50-54)."""
import numpy as np
import pytest

from message_cases import all_follower_items, results_of, stale_cycle_state, stale_second_leader_state
from oracle_lib import Oracle, assert_states_equal

from multiraft_amd import DEVICE, Engine, _abi, synth_seed, synth_tick_state
from multiraft_amd._abi import AE_ARGS, AE_REPLY, AE_RESULT

pytestmark = pytest.mark.gpu


def test_back_to_back_steps_without_host_sync_gpu():
    import torch
    G, P, L, K = 512, 5, 256, 4
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3) + 9)
    slots, peers = all_follower_items(lp, G, P)
    n = len(slots)
    dev = torch.device("cuda", 0)
    lib = _abi.lib()
    z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    args = [z(n, 10) for _ in range(K)]
    gerr, herr, ferr, flags = ([z(n) for _ in range(K)] for _ in range(4))
    rep, res = [z(n, 4) for _ in range(K)], [z(n, 8) for _ in range(K)]
    sl_d, pe_d = torch.from_numpy(slots).to(dev), torch.from_numpy(peers).to(dev)
    seg = np.concatenate([[0], np.cumsum(np.bincount(slots // P, minlength=G)[lp >= 0])]).astype(np.int64)
    seg_d = torch.from_numpy(seg).to(dev)
    with Engine(G, P, L) as e:
        e.load_state(st)
        stream = torch.cuda.ExternalStream(e.stream(), device=dev)
        e.synchronize()
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(2e8))  # ~0.1 s of device spin ahead of the calls
        for k in range(K):
            assert lib.mraft_gather_append_args(e._h, sl_d.data_ptr(), pe_d.data_ptr(), n, args[k].data_ptr(),
                                                gerr[k].data_ptr(), DEVICE) == 0, _abi.last_error()
            assert lib.mraft_handle_append_entries_ex(e._h, args[k].data_ptr(), n, None, 0, rep[k].data_ptr(),
                                                      res[k].data_ptr(), herr[k].data_ptr(), DEVICE) == 0, \
                _abi.last_error()
            assert lib.mraft_process_append_replies(e._h, res[k].data_ptr(), n, seg_d.data_ptr(), len(seg) - 1,
                                                    flags[k].data_ptr(), ferr[k].data_ptr(), DEVICE) == 0, \
                _abi.last_error()
        # every call returned with the device still behind the spin: nothing waited on it
        assert not stream.query(), "a message call waited on the device"
        e.synchronize()
        got = e.store_state()
    o = Oracle(G, P, L, st)
    for k in range(K):
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args[k].cpu().numpy().view(AE_ARGS).reshape(-1), oargs), k
        assert np.array_equal(gerr[k].cpu().numpy(), ogerr), k
        orep, oherr = o.handle_append_entries(oargs, None)
        assert np.array_equal(rep[k].cpu().numpy().view(AE_REPLY).reshape(-1), orep), k
        assert np.array_equal(herr[k].cpu().numpy(), oherr), k
        # the handler's reply records: the host-assembled records of the items it handled,
        # slot = peer = -1 for the others (a gather that failed forwards
        # zeroed args; with no host in between the batch carries them on)
        # (an item whose gather failed carries zeroed args: the device folds
        # its record as handled, the host helper below does not build one)
        gres = res[k].cpu().numpy().view(AE_RESULT).reshape(-1)
        okh = oherr == 0
        sel = okh & (ogerr == 0)
        hand = gres[sel][np.argsort(gres["slot"][sel], kind="stable")]
        want = results_of(slots, peers, oargs, orep, np.where(ogerr == 0, oherr, 1), G, P)[0]
        assert np.array_equal(hand, want), k
        assert (gres["slot"][~okh] == -1).all(), k
        # the fold over exactly what the device folded
        of, oferr = o.process_append_replies(gres, seg)
        assert np.array_equal(flags[k].cpu().numpy(), of) and np.array_equal(ferr[k].cpu().numpy(), oferr), k
    assert_states_equal(got, o.state(), G, P, L, f"{K} steps, no host sync")


def test_growing_batches_without_host_sync_gpu():
    """K message steps whose batches GROW (each larger than
    any before, so every call enlarges the engine's buffers: the handler's
    set/deferral/order slots and the fold's segment and scan slots, plus the
    first call's claims, counters and stage) enqueued behind a device spin on
    a fresh engine: every call returns with the stream still busy (buffers
    grow in stream order, no host wait) and the K steps equal K oracle steps
    on the same growing batches."""
    import torch
    G, P, L, K = 1024, 5, 256, 4
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3) + 11)
    dev = torch.device("cuda", 0)
    lib = _abi.lib()
    z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    batches = []
    for k in range(K):
        gk = G * (k + 1) // K                      # groups [0, gk): a strictly larger batch each step
        lpk = np.where(np.arange(G) < gk, lp, -1).astype(np.int32)
        slots, peers = all_follower_items(lpk, G, P)
        n = len(slots)
        seg = np.concatenate([[0], np.cumsum(np.bincount(slots // P, minlength=G)[lpk >= 0])]).astype(np.int64)
        batches.append(dict(slots=slots, peers=peers, n=n, seg=seg,
                            sl=torch.from_numpy(slots).to(dev), pe=torch.from_numpy(peers).to(dev),
                            sg=torch.from_numpy(seg).to(dev), args=z(n, 10), gerr=z(n), herr=z(n), ferr=z(n),
                            flags=z(n), rep=z(n, 4), res=z(n, 8)))
    assert all(batches[k]["n"] > batches[k - 1]["n"] for k in range(1, K))
    torch.cuda.synchronize()
    with Engine(G, P, L) as e:
        e.load_state(st)
        e.synchronize()
        stream = torch.cuda.ExternalStream(e.stream(), device=dev)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(2e8))  # ~0.1 s of device spin ahead of the calls
        for b in batches:
            n = b["n"]
            assert lib.mraft_gather_append_args(e._h, b["sl"].data_ptr(), b["pe"].data_ptr(), n, b["args"].data_ptr(),
                                                b["gerr"].data_ptr(), DEVICE) == 0, _abi.last_error()
            assert lib.mraft_handle_append_entries_ex(e._h, b["args"].data_ptr(), n, None, 0, b["rep"].data_ptr(),
                                                      b["res"].data_ptr(), b["herr"].data_ptr(), DEVICE) == 0, \
                _abi.last_error()
            assert lib.mraft_process_append_replies(e._h, b["res"].data_ptr(), n, b["sg"].data_ptr(), len(b["seg"]) - 1,
                                                    b["flags"].data_ptr(), b["ferr"].data_ptr(), DEVICE) == 0, \
                _abi.last_error()
        assert not stream.query(), "a growing message call waited on the device"
        e.synchronize()
        got = e.store_state()
    o = Oracle(G, P, L, st)
    for k, b in enumerate(batches):
        oargs, ogerr = o.gather_append_args(b["slots"], b["peers"])
        assert np.array_equal(b["args"].cpu().numpy().view(AE_ARGS).reshape(-1), oargs), k
        assert np.array_equal(b["gerr"].cpu().numpy(), ogerr), k
        orep, oherr = o.handle_append_entries(oargs, None)
        assert np.array_equal(b["rep"].cpu().numpy().view(AE_REPLY).reshape(-1), orep), k
        assert np.array_equal(b["herr"].cpu().numpy(), oherr), k
        # (as in test_back_to_back_steps_without_host_sync_gpu: an item whose
        # gather failed carries zeroed args on to the handler and the fold)
        gres = b["res"].cpu().numpy().view(AE_RESULT).reshape(-1)
        okh = oherr == 0
        sel = okh & (ogerr == 0)
        want = results_of(b["slots"], b["peers"], oargs, orep, np.where(ogerr == 0, oherr, 1), G, P)[0]
        assert np.array_equal(gres[sel][np.argsort(gres["slot"][sel], kind="stable")], want), k
        assert (gres["slot"][~okh] == -1).all(), k
        of, oferr = o.process_append_replies(gres, b["seg"])
        assert np.array_equal(b["flags"].cpu().numpy(), of) and np.array_equal(b["ferr"].cpu().numpy(), oferr), k
    assert_states_equal(got, o.state(), G, P, L, f"{K} growing steps, no host sync")


def test_back_to_back_copies_without_host_sync_gpu():
    """The bench's pattern: K steps, each on its own pristine state copy
    (mraft_bind_state), enqueued back to back with no synchronisation: every
    call's scratch is reused by the next while the device is still behind;
    every copy must end as one oracle step on the original state."""
    import torch
    G, P, L, K = 1024, 5, 512, 5
    st, lp, _ = synth_tick_state(G, P, L, seed=synth_seed(3) + 10)
    slots, peers = all_follower_items(lp, G, P)
    n = len(slots)
    dev = torch.device("cuda", 0)
    lib = _abi.lib()
    copies = [{k: torch.from_numpy(v.copy()).to(dev) for k, v in st.items()} for _ in range(K)]
    z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    args, gerr, herr, ferr, flags, rep, res = z(n, 10), z(n), z(n), z(n), z(n), z(n, 4), z(n, 8)
    fl_all = z(K, n)
    sl_d, pe_d = torch.from_numpy(slots).to(dev), torch.from_numpy(peers).to(dev)
    seg = np.concatenate([[0], np.cumsum(np.bincount(slots // P, minlength=G)[lp >= 0])]).astype(np.int64)
    seg_d = torch.from_numpy(seg).to(dev)
    torch.cuda.synchronize()
    with Engine(G, P, L, alloc=False) as e:
        e.bind(copies[0])
        stream = torch.cuda.ExternalStream(e.stream(), device=dev)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(2e8))
        for k in range(K):
            e.bind(copies[k])
            assert lib.mraft_gather_append_args(e._h, sl_d.data_ptr(), pe_d.data_ptr(), n, args.data_ptr(),
                                                gerr.data_ptr(), DEVICE) == 0
            assert lib.mraft_handle_append_entries_ex(e._h, args.data_ptr(), n, None, 0, rep.data_ptr(),
                                                      res.data_ptr(), herr.data_ptr(), DEVICE) == 0
            assert lib.mraft_process_append_replies(e._h, res.data_ptr(), n, seg_d.data_ptr(), len(seg) - 1,
                                                    fl_all[k].data_ptr(), ferr.data_ptr(), DEVICE) == 0
        assert not stream.query(), "a message call waited on the device"
        e.synchronize()
    o = Oracle(G, P, L, st)
    oargs, ogerr = o.gather_append_args(slots, peers)
    assert (ogerr == 0).all()
    orep, oherr = o.handle_append_entries(oargs, None)
    ores, oseg = results_of(slots, peers, oargs, orep, oherr, G, P)
    of, _ = o.process_append_replies(ores, oseg)
    want = o.state()
    for k in range(K):
        assert np.array_equal(fl_all[k].cpu().numpy(), of), k
        assert_states_equal({kk: v.cpu().numpy() for kk, v in copies[k].items()}, want, G, P, L, f"copy {k}")


def _self_reference(st, lp, G, P, L, rng):
    """A gathered batch in which some leaders' first message is addressed to
    the leader's own slot: the item reads the row it writes."""
    slots, peers = all_follower_items(lp, G, P)
    return slots, peers, rng.choice(G // 4, size=G // 8, replace=False)


CASES = ["stale_leader", "ring2", "ring3", "self"]


@pytest.mark.parametrize("cap", ["default", "small", "zero", "auto"])
@pytest.mark.parametrize("case", CASES)
def test_deferred_items_gpu(case, cap):
    G, P, L = 256, 5, 128
    rng = np.random.default_rng(11 * CASES.index(case) + len(cap))
    st, lp, _ = synth_tick_state(G, P, L, seed=77 + CASES.index(case))
    self_groups = None
    if case == "stale_leader":
        st, slots, peers = stale_second_leader_state(st, lp, G, P, L, rng, range(0, G, 2))
    elif case.startswith("ring"):
        st, slots, peers = stale_cycle_state(st, lp, G, P, L, rng, range(0, G, 3), int(case[-1]))
    else:
        slots, peers, self_groups = _self_reference(st, lp, G, P, L, rng)
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if cap in ("small", "auto"):
            e.set_stage_capacity(64)
        elif cap == "zero":
            e.set_stage_capacity(0)
        if cap == "auto":  # MRAFT_STAGE_AUTO from 64 words: the first call's need grows it for the second
            e.set_stage_capacity(-1)
        assert e.stage_capacity() == {"default": 1 << 22, "small": 64, "zero": 0, "auto": 64}[cap]
        args, gerr = e.gather_append_args(slots, peers)
        oargs, ogerr = o.gather_append_args(slots, peers)
        assert np.array_equal(args, oargs) and np.array_equal(gerr, ogerr)
        batch = args[gerr == 0].copy()
        if self_groups is not None:
            first = {}
            for j, a in enumerate(batch):
                g = int(a["slot"]) // P
                if g in set(self_groups.tolist()) and g not in first:
                    first[g] = j
            for g, j in first.items():
                batch[j]["slot"] = int(batch[j]["entries_offset"]) // L   # the leader's own slot
        rep, herr, gres = e.handle_append_entries(batch, None, results=True)
        orep, oherr = o.handle_append_entries(batch, None)
        assert np.array_equal(herr, oherr), case
        assert np.array_equal(rep, orep), case
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{case}, stage {cap}")
        # a second call on the same engine after the fallback: the counters re-arm
        args2, gerr2 = e.gather_append_args(slots, peers)
        oargs2, ogerr2 = o.gather_append_args(slots, peers)
        assert np.array_equal(args2, oargs2)
        rep2, herr2 = e.handle_append_entries(args2[gerr2 == 0], None)
        orep2, oherr2 = o.handle_append_entries(oargs2[ogerr2 == 0], None)
        assert np.array_equal(herr2, oherr2) and np.array_equal(rep2, orep2)
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{case}, stage {cap}, second call")
        if cap == "auto" and case.startswith("ring"):
            assert e.stage_capacity() >= 1 << 20, e.stage_capacity()  # grown (1 Mi-word steps)


@pytest.mark.parametrize("fold", ["append", "vote", "install"])
def test_segment_owner_rule_gpu(fold):
    """Reply segments that name the same replica slot (the chain above makes
    them: a failed gather forwards zeroed args): the lowest non-empty segment
    naming a slot owns it even when its own records are bad, and a later one
    is MRAFT_ITEM_DUP_SLOT (include/mraft.h) — GPU == oracle for each fold."""
    from multiraft_amd._abi import IS_RESULT, RV_RESULT
    G, P, L = 64, 5, 64
    st, lp, _ = synth_tick_state(G, P, L, seed=5150)
    rng = np.random.default_rng(3)
    dt = {"append": AE_RESULT, "vote": RV_RESULT, "install": IS_RESULT}[fold]
    recs, seg = [], [0]
    for g in range(G):
        slot = g * P + int(max(lp[g], 0))
        for k in range(int(rng.integers(1, 4))):
            r = np.zeros(1, dtype=dt)[0]
            r["slot"], r["peer"] = slot, (slot % P + 1 + k) % P
            r["args_term"] = int(st["current_term"][slot])
            if fold == "append":
                r["args_prev_log_index"] = int(st["next_index"][slot * P + r["peer"]]) - 1
                r["reply_term"], r["reply_success"], r["args_n_entries"] = r["args_term"], 1, 1
            elif fold == "vote":
                r["reply_term"], r["vote_granted"] = r["args_term"], 1
            else:
                r["args_last_included_index"], r["reply_term"] = int(st["dummy_index"][slot]), r["args_term"]
            recs.append(r)
        seg.append(len(recs))
    recs = np.array(recs, dtype=dt)
    seg = np.array(seg, np.int64)
    # corrupt: segment 3's second-to-first record names another slot (BAD_SLOT),
    # segment 9 repeats segment 3's slot (DUP: 3 owns it), segment 12 repeats
    # segment 5's slot (DUP), segment 20 is empty, segment 21 names an
    # out-of-range slot
    b3, b9, b12, b5 = seg[3], seg[9], seg[12], seg[5]
    if seg[4] - b3 > 1:
        recs["slot"][b3 + 1] = recs["slot"][b3] + 1
    recs["slot"][b9:seg[10]] = recs["slot"][b3]
    recs["slot"][b12:seg[13]] = recs["slot"][b5]
    recs["slot"][seg[21]:seg[22]] = G * P + 7
    seg = np.concatenate([seg[:21], [seg[20]], seg[21:]])   # an empty segment before 21
    o = Oracle(G, P, L, st)
    with Engine(G, P, L) as e:
        e.load_state(st)
        if fold == "append":
            got, want = e.process_append_replies(recs, seg), o.process_append_replies(recs, seg)
        elif fold == "vote":
            got, want = e.process_vote_replies(recs, seg), o.process_vote_replies(recs, seg)
        else:
            got, want = e.process_install_snapshot_replies(recs, seg), o.process_install_snapshot_replies(recs, seg)
        assert np.array_equal(got[1], want[1]), fold
        assert np.array_equal(got[0], want[0]), fold
        assert (want[1] == _abi.ITEM_DUP_SLOT).sum() > 0 and (want[1] == _abi.ITEM_BAD_SLOT).sum() > 0
        assert_states_equal(e.store_state(), o.state(), G, P, L, f"{fold} owner rule")
