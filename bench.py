"""Headline benchmark: quorum commit decisions/s at 64k groups x 5 peers
(BASELINE.json) and the HBM-roofline fraction of the
dominant kernel.

One step = one fused replication tick over a fresh, HBM-resident copy of the
seeded config-#3 state: for each of the G groups the leader gathers an
AppendEntries per follower (a3), each follower handles it (a4: term check,
prevLog match, ConflictIndex scan, entry merge/truncate/append, follower
commit), and the leader folds the P-1 replies in peer order with the
majority/current-term commit rule (a2 + a1); then GetState words are exported
(and, with N > 1, all-gathered over RCCL for the shard router, §8e).
decisions/s = groups x steps / time. Every timed step runs on its own pristine
copy of the state (a tick mutates the state; re-running it on mutated state
would be a different, lighter workload).

Usage: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either launch
with torch.distributed.run (one process per GPU) or let bench.py start the N
rank processes itself; N > 1 defaults to BASELINE config #4 (262,144 groups
split over the GPUs, strong scaling) with one RCCL all-gather of the GetState
words per tick through the C ABI. Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "quorum commit decisions/sec @64k groups×5 peers; % HBM roofline"
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip-level parameters


def kernel_src_sha() -> str:
    import hashlib
    h = hashlib.sha1()
    for f in ("mraft_tick.hip", "mraft_tick_body.inc", "mraft_device.h", "mraft_pass.h"):
        h.update(open(os.path.join(ROOT, "multiraft_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:12]


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_share() -> dict:
    """The host cores this process may use: its CPU affinity, capped by a
    cgroup CPU quota when one is set (the GPU box's nproc shows the whole
    machine). `threads` is what the CPU baseline runs on."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return {"threads": max(1, min(aff, quota) if quota else aff), "affinity": aff, "cgroup_quota": quota,
            "nproc": os.cpu_count()}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def sleep_cycles_per_ms(stream) -> float:
    """torch.cuda._sleep's units on this device (a spin on the GPU clock
    counter), measured once with HIP events."""
    import torch
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        a.record()
        torch.cuda._sleep(int(1e6))
        b.record()
    b.synchronize()
    return 1e6 / max(a.elapsed_time(b), 1e-3)


def message_path(master, copies, lp, G, P, L, dev, S, steps, words=False, offset_ms=0.0, split=False):
    """The config #3 message-level path (gather -> HandleAppendEntries by
    reference -> processAppendEntriesReply + a1) as S shard
    pipelines: shard s = groups [G*s/S, G*(s+1)/S) of every state copy (SoA
    slices, no copies), its own engine on a hardware queue of its own
    (MRAFT_CREATE_DEDICATED_QUEUE) driven by its own host thread — the Go
    host's goroutine per shard: ctypes releases the GIL in
    the engine calls, so one shard's host-side work does not hold the other
    back (no call waits on the device: round 5). Step i runs on copy i restored
    from `master`; the warm-up on copy `steps`.
    split (S = 1): one event between consecutive calls (the per-call split;
    each event is a marker packet, a bubble of ~6 us on the queue: profiles/r5_c1);
    otherwise one event per step on each queue, as the headline records one
    per tick (the device span per step);
    shard s > 0 starts `offset_ms` * s / (S - 1) after shard 0 (a device
    spin on its queue), so the shards' short latency-bound calls (gather,
    claims, fold) can run beside another shard's streaming handler
    instead of in lock-step with it.
    words=True: the algorithmic words of one batch (tools/msg_words.py) from
    the warm-up's inputs (S = 1 only)."""
    import threading

    import torch

    from multiraft_amd import DEVICE, Engine, _abi
    lib = _abi.lib()

    def ck(rc, what):
        assert rc == 0, (what, _abi.last_error())

    for c in copies[:steps + 1]:
        for k, v in master.items():
            c[k].copy_(v)
    torch.cuda.synchronize()
    per_group = {k: v.numel() // G for k, v in master.items()}
    shards = []
    for si in range(S):
        g0, g1 = G * si // S, G * (si + 1) // S
        n_g = g1 - g0
        e = Engine(n_g, P, L, device=dev.index or 0, alloc=False, dedicated_queue=True)
        st = torch.cuda.ExternalStream(e.stream(), device=dev)
        lps = lp[g0:g1]
        ldr = (np.arange(n_g) * P + lps).repeat(P - 1)
        q = np.tile(np.arange(P - 1), n_g)
        peers = np.where(q < np.repeat(lps, P - 1), q, q + 1)
        keep = np.repeat(lps >= 0, P - 1)
        ldr, peers = ldr[keep].astype(np.int32), peers[keep].astype(np.int32)
        n = len(ldr)
        z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
        sh = {"eng": e, "st": st, "g": (g0, g1), "n": n,
              "slots": torch.from_numpy(ldr).to(dev), "peers": torch.from_numpy(peers).to(dev),
              "args": z(n, 10), "gerr": z(n), "herr": z(n), "ferr": z(n), "flags": z(n), "rep": z(n, 4),
              "res": z(n, 8),
              "seg": torch.from_numpy(np.concatenate([[0], np.cumsum(np.bincount(ldr // P, minlength=n_g)[lps >= 0])])
                                      .astype(np.int64)).to(dev),
              "views": [{k: v[g0 * per_group[k]:g1 * per_group[k]] for k, v in c.items()} for c in copies[:steps + 1]]}
        shards.append(sh)
    torch.cuda.synchronize()

    def run(sh, i, marks):
        e, st, n, a = sh["eng"], sh["st"], sh["n"], sh["args"]
        e.bind(sh["views"][i])
        if marks is not None and len(marks) > 1:
            marks[0].record(st)
        ck(lib.mraft_gather_append_args(e._h, sh["slots"].data_ptr(), sh["peers"].data_ptr(), n, a.data_ptr(),
                                        sh["gerr"].data_ptr(), DEVICE), "gather")
        if marks is not None and len(marks) > 1:
            marks[1].record(st)
        # the handler also writes each reply's record for the leader's fold
        # (mraft_handle_append_entries_ex: no host-side assembly)
        ck(lib.mraft_handle_append_entries_ex(e._h, a.data_ptr(), n, None, 0, sh["rep"].data_ptr(),
                                              sh["res"].data_ptr(), sh["herr"].data_ptr(), DEVICE), "handle")
        if marks is not None and len(marks) > 1:
            marks[2].record(st)
        ck(lib.mraft_process_append_replies(e._h, sh["res"].data_ptr(), n, sh["seg"].data_ptr(),
                                            len(sh["seg"]) - 1, sh["flags"].data_ptr(), sh["ferr"].data_ptr(),
                                            DEVICE), "fold")
        if marks is not None:
            marks[-1].record(st)

    out = {}
    # warm-up (and the algorithmic words) on copy `steps`
    for sh in shards:
        run(sh, steps, None)
    for sh in shards:
        sh["eng"].synchronize()
    for sh in shards:
        assert int(sh["gerr"].abs().sum()) == 0 and int(sh["herr"].abs().sum()) == 0
        assert int(sh["ferr"].abs().sum()) == 0
    if words:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from msg_words import fold_words, handle_words
        sh = shards[0]
        host = {k: v.cpu().numpy() for k, v in master.items()}
        args_h = sh["args"].cpu().numpy().view(_abi.AE_ARGS).reshape(-1)
        hw = handle_words(host, args_h, sh["rep"].cpu().numpy().view(_abi.AE_REPLY).reshape(-1),
                          sh["herr"].cpu().numpy(), G, P, L)
        # the fold reads only leader replicas, which no message of this batch
        # targets: their pre-handle state is the fold's input
        res_h = sh["res"].cpu().numpy().view(_abi.AE_RESULT).reshape(-1)
        assert not np.isin(res_h["slot"], args_h["slot"]).any()
        fw = fold_words(host, res_h, sh["seg"].cpu().numpy(), P, L)
        ld_sl = np.unique(res_h["slot"])
        assert np.array_equal(fw["commit"][ld_sl], copies[steps]["commit_index"].cpu().numpy()[ld_sl]), \
            "fold word count: replayed commits differ from the device's"
        out["hw"], out["fw"] = hw, fw
    nm = 4 if S == 1 and split else 1
    marks = [[[torch.cuda.Event(enable_timing=True) for _ in range(nm)] for _ in range(steps)] for _ in range(S)]
    # A gate: every queue waits for an event recorded behind a ~5 ms device
    # spin on torch's stream, so all threads have enqueued their first step
    # when the device starts on them (thread start-up is not device time).
    t_begin = torch.cuda.Event(enable_timing=True)
    cpm = sleep_cycles_per_ms(torch.cuda.current_stream()) if offset_ms > 0 and S > 1 else 0.0
    torch.cuda.synchronize()
    torch.cuda._sleep(int(12e6))
    t_begin.record()
    for si, sh in enumerate(shards):
        sh["st"].wait_event(t_begin)
        if cpm and si > 0:
            with torch.cuda.stream(sh["st"]):
                torch.cuda._sleep(int(cpm * offset_ms * si / (S - 1)))

    errors = []

    def worker(si):
        try:
            for i in range(steps):
                run(shards[si], i, marks[si][i])
        except BaseException as x:  # re-raised after the join
            errors.append(x)

    th = [threading.Thread(target=worker, args=(si,)) for si in range(S)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]
    for sh in shards:
        sh["eng"].synchronize()
    torch.cuda.synchronize()
    out["device_ms_per_step"] = max(t_begin.elapsed_time(marks[si][-1][-1]) for si in range(S)) / steps
    out["steps"] = steps
    if S == 1 and split:
        m = marks[0]
        out["ms_per_call"] = {"gather": float(np.mean([x[0].elapsed_time(x[1]) for x in m])),
                              "handle": float(np.mean([x[1].elapsed_time(x[2]) for x in m])),
                              "fold": float(np.mean([x[2].elapsed_time(x[3]) for x in m]))}
    for sh in shards:
        assert int(sh["gerr"].abs().sum()) == 0 and int(sh["herr"].abs().sum()) == 0
        assert int(sh["ferr"].abs().sum()) == 0
        sh["eng"].close()
    return out


def deferred_batch_state(host, lp, G, P, L, kind, seed=0xDEF):
    """Config #3's state with a stale second leader q = (lp + 1) % P in every
    other group, and the batch a node receives then: every
    real leader's AppendEntries to its P - 1 followers plus one from each stale
    leader, to r = (lp + 2) % P ("stale": lp -> q is `written`, q's row being
    read by q -> r: deferred, in place) or to lp itself ("cycles": lp -> q and
    q -> lp each read the row the other rewrites: a 2-cycle, both staged, past
    the stage capacity the fallback's cycles). q is a Leader one term below
    lp with nextIndex[target] inside its log. Returns (state, slots, peers)."""
    rng = np.random.default_rng(seed)
    st = {k: v.copy() for k, v in host.items()}
    g = np.arange(0, G, 2)
    g = g[lp[g] >= 0]
    l = lp[g].astype(np.int64)
    q, r = (l + 1) % P, (l + 2) % P
    ls, qs = g * P + l, g * P + q
    st["state"][qs] = 1  # Leader
    st["current_term"][qs] = np.maximum(1, st["current_term"][ls] - 1)
    tgt = l if kind == "cycles" else r
    d, last = st["dummy_index"][qs].astype(np.int64), st["last_index"][qs].astype(np.int64)
    st["next_index"][qs * P + tgt] = rng.integers(d + 1, last + 2)
    lq = np.where(lp >= 0)[0]
    ldr = (lq * P + lp[lq]).repeat(P - 1)
    k = np.tile(np.arange(P - 1), len(lq))
    fp = np.where(k < np.repeat(lp[lq], P - 1), k, k + 1)
    if kind != "cycles":
        # r receives from q instead of from lp (one message per receiving
        # slot, include/mraft.h): the batch keeps the plain batch's size
        drop = np.zeros(G, bool)
        drop[g] = True
        keep = ~(drop[ldr // P] & (fp == np.repeat(np.where(drop, (lp + 2) % P, -1)[lq], P - 1)))
        ldr, fp = ldr[keep], fp[keep]
    slots = np.concatenate([ldr, qs]).astype(np.int32)
    peers = np.concatenate([fp, tgt]).astype(np.int32)
    return st, slots, peers


def message_path_deferred(master, copies, lp, G, P, L, dev, steps=5):
    """The handle call (mraft_handle_append_entries_ex by reference) on config
    #3 batches heavy in deferred items (deferred_batch_state), against the
    plain batch on the same copies: per call, and per message. Each variant on
    a fresh engine: its first call runs on the minimal deferred grid (no
    earlier count) and, past the stage, in the ordered fallback
    (`first_call_ms`), then `steps` timed calls, each on a state copy restored
    from that variant's master (one event before and one after the handle
    call); under MRAFT_STAGE_AUTO (the default) the second call grows the stage
    to the first call's need (`ms_calls` has every call)."""
    import torch

    from multiraft_amd import DEVICE, Engine, _abi
    lib = _abi.lib()
    host = {k: v.cpu().numpy() for k, v in master.items()}
    dm = {k: v.clone() for k, v in master.items()}
    z = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    out = {}
    lq = np.where(lp >= 0)[0]
    plain_slots = (lq * P + lp[lq]).repeat(P - 1).astype(np.int32)
    kk = np.tile(np.arange(P - 1), len(lq))
    plain_peers = np.where(kk < np.repeat(lp[lq], P - 1), kk, kk + 1).astype(np.int32)
    variants = [("plain", None, None), ("stale", "stale", None), ("stale_stage0", "stale", 0),
                ("cycles", "cycles", None), ("cycles_stage0", "cycles", 0)]
    for name, kind, cap in variants:
        if kind is None:
            st_h, slots, peers = host, plain_slots, plain_peers
        else:
            st_h, slots, peers = deferred_batch_state(host, lp, G, P, L, kind)
        for kx, v in st_h.items():
            dm[kx].copy_(torch.from_numpy(v))
        n = len(slots)
        sl_d, pe_d = torch.from_numpy(slots).to(dev), torch.from_numpy(peers).to(dev)
        args, gerr, herr, rep, res = z(n, 10), z(n), z(n), z(n, 4), z(n, 8)
        e = Engine(G, P, L, device=dev.index or 0, alloc=False, dedicated_queue=True)
        st = torch.cuda.ExternalStream(e.stream(), device=dev)
        times = []
        ndef = 0
        for i in range(steps + 1):
            c = copies[i]
            for kx, v in dm.items():
                c[kx].copy_(v)
            torch.cuda.synchronize()
            e.bind(c)
            if cap is not None and i == 0:  # (a bound engine: the call checks the state)
                assert lib.mraft_set_stage_capacity(e._h, cap) == 0, _abi.last_error()
            assert lib.mraft_gather_append_args(e._h, sl_d.data_ptr(), pe_d.data_ptr(), n, args.data_ptr(),
                                                gerr.data_ptr(), DEVICE) == 0, _abi.last_error()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            assert lib.mraft_handle_append_entries_ex(e._h, args.data_ptr(), n, None, 0, rep.data_ptr(),
                                                      res.data_ptr(), herr.data_ptr(), DEVICE) == 0, \
                _abi.last_error()
            b.record(st)
            e.synchronize()
            times.append(a.elapsed_time(b))
            if i == 0:
                ah = args.cpu().numpy().view(_abi.AE_ARGS).reshape(-1)
                ok = gerr.cpu().numpy() == 0
                src = np.where(ok & (ah["n_entries"] > 0), ah["entries_offset"] // L, -1)
                ndef = int((ok & np.isin(ah["slot"], src[src >= 0])).sum())
                assert ok.all(), f"{name}: gather errors"
        cap_end = int(lib.mraft_get_stage_capacity(e._h))
        e.close()
        out[name] = {"messages": n, "deferred_items": ndef, "stage_capacity_words": cap if cap is not None else
                     "MRAFT_STAGE_AUTO (from 4 Mi)", "stage_capacity_words_end": cap_end,
                     "first_call_ms": times[0], "ms_per_call": float(np.mean(times[1:])),
                     "ms_calls": [round(t, 4) for t in times], "ns_per_message": float(np.mean(times[1:])) * 1e6 / n}
    base = out["plain"]
    for name in out:
        if name != "plain":
            out[name]["vs_plain"] = out[name]["ms_per_call"] / base["ms_per_call"]
            out[name]["per_message_vs_plain"] = out[name]["ns_per_message"] / base["ns_per_message"]
    del dm
    torch.cuda.empty_cache()
    return out


def steady_state(master, copies, lp, G, P, L, dev, steps=40, ss0=24, seed=0x5EAD):
    """Config #3 ticked in place: one state copy, and per
    step a Start of 1-4 entries at every leader (mraft_start, raft.go:90-104)
    then one mraft_replicate_tick — a heartbeat / append round of a running
    deployment, where followers are caught up after the first rounds. All
    calls enqueued back to back on one engine stream (no shards), an event
    before and after each call, once with the full tick (one launch) and once
    with the light tick (MRAFT_TICK_LIGHT: its two launches) on a second copy
    of the same state, whose final state must equal the first's; a third pass
    on a fresh copy interleaves mraft_replicate_tick_count before each tick
    (side-effect free) for the algorithmic bytes, and a fourth runs the light
    sequence with a host wait per step to read each tick's fallback count;
    then the floor of a launch that does no group's work (leader_peer -1
    everywhere: every wave exits after one load)."""
    import torch

    from multiraft_amd import DEVICE, TICK_FULL, TICK_LIGHT, Engine, _abi
    lib = _abi.lib()
    rng = np.random.default_rng(seed)
    lq = np.where(lp >= 0)[0]
    ldr = torch.from_numpy((lq * P + lp[lq]).astype(np.int32)).to(dev)
    nl = len(lq)
    cnts_h = [rng.integers(1, 5, size=nl).astype(np.int32) for _ in range(steps)]
    cnts = [torch.from_numpy(c).to(dev) for c in cnts_h]
    # the same Starts per group, for mraft_start_and_tick (0 where no leader)
    gcnts = []
    for c in cnts_h:
        gc = np.zeros(G, np.int32)
        gc[lq] = c
        gcnts.append(torch.from_numpy(gc).to(dev))
    oi, ot, ol, oe = (torch.zeros(nl, dtype=torch.int32, device=dev) for _ in range(4))
    lp_d = torch.from_numpy(lp.astype(np.int32)).to(dev)
    gf = torch.zeros(G, dtype=torch.int32, device=dev)
    e = Engine(G, P, L, device=dev.index or 0, alloc=False, dedicated_queue=True)
    st = torch.cuda.ExternalStream(e.stream(), device=dev)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def restore(c):
        for k, v in master.items():
            c[k].copy_(v)
        torch.cuda.synchronize()
        e.bind(c)

    def start(k):
        assert lib.mraft_start(e._h, ldr.data_ptr(), cnts[k].data_ptr(), nl, oi.data_ptr(), ot.data_ptr(),
                               ol.data_ptr(), oe.data_ptr(), DEVICE) == 0, _abi.last_error()

    def timed(mode, c):
        restore(c)
        e.set_tick_mode(mode)
        marks = [[ev() for _ in range(3)] for _ in range(steps)]
        for k in range(steps):
            marks[k][0].record(st)
            start(k)
            marks[k][1].record(st)
            e.replicate_tick(lp_d, gf, where=DEVICE)
            marks[k][2].record(st)
        e.synchronize()
        return ([m[0].elapsed_time(m[1]) for m in marks], [m[1].elapsed_time(m[2]) for m in marks],
                marks[ss0][0].elapsed_time(marks[-1][2]) / (steps - ss0), gf.cpu().numpy())

    start_ms, tick_ms, span_ss, flags = timed(TICK_FULL, copies[0])
    log_full = int((oe.cpu().numpy() == 3).sum())
    lstart_ms, ltick_ms, lspan_ss, lflags = timed(TICK_LIGHT, copies[1])
    same = bool(np.array_equal(flags, lflags)) and all(torch.equal(copies[0][k], copies[1][k]) for k in master)
    # the same sequence as one call per step (mraft_start_and_tick, light
    # tick: Start inside its first launch), on a third copy
    restore(copies[2])
    e.set_tick_mode(TICK_LIGHT)
    fmarks = [ev() for _ in range(steps + 1)]
    fmarks[0].record(st)
    for k in range(steps):
        e.start_and_tick(lp_d, gcnts[k], gf, where=DEVICE)
        fmarks[k + 1].record(st)
    e.synchronize()
    fstep_ms = [fmarks[k].elapsed_time(fmarks[k + 1]) for k in range(steps)]
    fflags = gf.cpu().numpy()
    fsame = bool(np.array_equal(flags, fflags)) and all(torch.equal(copies[0][k], copies[2][k]) for k in master)
    # count pass (same sequence, the count before each tick)
    restore(copies[0])
    e.set_tick_mode(TICK_FULL)
    words = np.zeros((steps, 3), np.int64)
    for k in range(steps):
        start(k)
        words[k] = e.replicate_tick_count(lp)
        e.replicate_tick(lp_d, gf, where=DEVICE)
    e.synchronize()
    # the light sequence again, a host wait per step: each tick's fallback count
    restore(copies[1])
    e.set_tick_mode(TICK_LIGHT)
    fallbacks = []
    for k in range(steps):
        start(k)
        e.replicate_tick(lp_d, gf, where=DEVICE)
        e.synchronize()
        fallbacks.append(e.tick_light_fallbacks())
    e.set_tick_mode(TICK_FULL)
    # a launch with no group's work
    none = torch.full((G,), -1, dtype=torch.int32, device=dev)
    empty = []
    for _ in range(5):
        a, b = ev(), ev()
        a.record(st)
        e.replicate_tick(none, gf, where=DEVICE)
        b.record(st)
        e.synchronize()
        empty.append(a.elapsed_time(b))
    e.close()
    # steady state: the last steps - ss0 steps. The synthetic state's backlog
    # (followers with conflicting or missing tails) is repaired over the first
    # ~15 ticks: the light tick's fallback count per step drains to its floor
    # (fallback_groups_steps), and the steps before carry that work
    ss = slice(ss0, steps)
    tick_ss = float(np.mean(tick_ms[ss]))
    ltick_ss = float(np.mean(ltick_ms[ss]))
    bytes_ss = float(np.mean(4 * (words[ss, 0] + words[ss, 1])))
    act_ss = float(np.mean(words[ss, 2]))
    empty_ms = float(np.median(empty))
    return {"workload": "config #3 ticked in place: per step mraft_start of 1-4 entries at each of the %d leaders, "
                        "then one mraft_replicate_tick (no shards), %d steps back to back on one engine stream; "
                        "steady state = steps %d..%d (the backlog drained: fallback_groups_steps); top-level fields: the full tick (MRAFT_TICK_FULL, one "
                        "launch), `light`: the same sequence with MRAFT_TICK_LIGHT" % (nl, steps, ss0 + 1, steps),
            "steps": steps, "tick_ms_steps": [round(x, 4) for x in tick_ms],
            "start_ms_mean": float(np.mean(start_ms)),
            "tick_ms_steady": tick_ss, "device_ms_per_step_steady": span_ss,
            "decisions_per_s_steady": G / (span_ss / 1e3),
            "tick_decisions_per_s_steady": G / (tick_ss / 1e3),
            "algorithmic_bytes_per_tick_steady": bytes_ss,
            "algorithmic_bytes_per_decision_steady": bytes_ss / max(act_ss, 1.0),
            "tick_achieved_GBps_steady": bytes_ss / tick_ss / 1e6,
            "tick_hbm_frac_steady": bytes_ss / (tick_ss / 1e3) / HBM_PEAK,
            "first_tick_ms": tick_ms[0], "first_tick_algorithmic_bytes": int(4 * (words[0, 0] + words[0, 1])),
            "empty_launch_ms": empty_ms,
            "launch_share_of_tick_steady": empty_ms / tick_ss,
            "launch_share_what": "a tick launch over the same 65,536 groups with no leader (each wave loads "
                                 "leader_peer and exits) over the steady-state tick: the part of a steady tick a "
                                 "launch with no work already costs",
            "gaps_share_steady": 1.0 - (float(np.sum(tick_ms[ss])) + float(np.sum(start_ms[ss]))) /
                                 (span_ss * (steps - ss0)),
            "start_log_full_last_step": log_full,
            "groups_committed_last_step": int(((flags & 2) != 0).sum()),
            "light": {"what": "MRAFT_TICK_LIGHT: k_tick_lite (eight groups per wave; the steady-state groups "
                              "settled there) + k_tick_list (the others through the full tick, grid from the "
                              "previous tick's count)",
                      "tick_ms_steps": [round(x, 4) for x in ltick_ms],
                      "tick_ms_steady": ltick_ss, "device_ms_per_step_steady": lspan_ss,
                      "decisions_per_s_steady": G / (lspan_ss / 1e3),
                      "tick_decisions_per_s_steady": G / (ltick_ss / 1e3),
                      "tick_achieved_GBps_steady": bytes_ss / ltick_ss / 1e6,
                      "tick_hbm_frac_steady": bytes_ss / (ltick_ss / 1e3) / HBM_PEAK,
                      "speedup_tick_steady": tick_ss / ltick_ss,
                      "fallback_groups_steps": fallbacks,
                      "state_equals_full": same},
            "fused": {"what": "mraft_start_and_tick with MRAFT_TICK_LIGHT: the Start of every step inside the light "
                              "tick's first launch, one call and one event per step (the same Starts and ticks as "
                              "above, on a third copy)",
                      "step_ms_steps": [round(x, 4) for x in fstep_ms],
                      "device_ms_per_step_steady": float(np.mean(fstep_ms[ss])),
                      "decisions_per_s_steady": G / (float(np.mean(fstep_ms[ss])) / 1e3),
                      "vs_full_start_then_tick": span_ss / float(np.mean(fstep_ms[ss])),
                      "vs_light_start_then_tick": lspan_ss / float(np.mean(fstep_ms[ss])),
                      "state_equals_full": fsame}}


def secondary(master, copies, lp, G, P, L, stream, dev, headline_ms, steps=8):
    """The survey's other configurations, measured in the same run so they are
    on the driver's record (rank 0, one GPU, after the headline's timed
    region; never part of `value`):
      * the message-level path at config #3 (gather -> handle by reference ->
        fold) on a fresh copy per step, one pipeline and two
        shard pipelines (message_path), with the handler's and the fold's
        rooflines from their algorithmic bytes (tools/msg_words.py);
      * config #5, the election storm (65,536 x 7, 64 rounds per launch);
      * config #2 (1,024 x 3 x 256: cache-resident, launch-bound).
    `copies` are the state copies the headline already used, step i of the
    message path on copy i restored from `master` (so its steps see both
    memory populations, like the headline's)."""
    import torch

    from multiraft_amd import DEVICE, TICK_FULL, Engine, synth_election_state, synth_seed, synth_tick_state

    out = {}

    def ev():
        return torch.cuda.Event(enable_timing=True)

    # -- message-level path, config #3
    one = message_path(master, copies, lp, G, P, L, dev, 1, steps, words=True, split=True)
    flat = message_path(master, copies, lp, G, P, L, dev, 1, len(copies) - 1)
    two = message_path(master, copies, lp, G, P, L, dev, 2, len(copies) - 1)
    three = message_path(master, copies, lp, G, P, L, dev, 3, len(copies) - 1)
    hw, fw, ms = one["hw"], one["fw"], one["ms_per_call"]
    n = 4 * int((lp >= 0).sum())
    step_ms = ms["gather"] + ms["handle"] + ms["fold"]
    hb = 4 * hw["words"]
    out["message_path_config3"] = {
        "workload": "config #3 message-level path: gather -> HandleAppendEntries (entries by reference, "
                    "message sets; the reply records for the fold written by the handler, "
                    "mraft_handle_append_entries_ex) -> processAppendEntriesReply + advanceCommitIndex, fresh "
                    "copy per step",
        "messages": n, "steps": steps, "ms_per_call": {k: round(v, 4) for k, v in ms.items()},
        "decisions_per_s": G / (step_ms / 1e3),
        "calls_ms_sum_vs_headline": step_ms / headline_ms,
        "shards_2": {"what": "two shard pipelines: one engine per half of the groups on a hardware queue of its "
                             "own, one host thread each (the Go goroutine per shard); one event per step per queue; "
                             "device time from a gate every queue waits on to the last queue's last event",
                     "steps": two["steps"], "device_ms_per_step": two["device_ms_per_step"],
                     "decisions_per_s": G / (two["device_ms_per_step"] / 1e3),
                     "vs_headline": two["device_ms_per_step"] / headline_ms},
        "shards_3": {"what": "as shards_2 with three pipelines (a third of the groups each; three engine queues "
                             "and torch's, which idles in the timed region: GPU_MAX_HW_QUEUES = 4)",
                     "steps": three["steps"], "device_ms_per_step": three["device_ms_per_step"],
                     "decisions_per_s": G / (three["device_ms_per_step"] / 1e3),
                     "vs_headline": three["device_ms_per_step"] / headline_ms},
        "one_pipeline_device_ms_per_step": flat["device_ms_per_step"],
        "one_pipeline_vs_headline": flat["device_ms_per_step"] / headline_ms,
        "one_pipeline_what": "the three calls one after another on one queue, one event per step (as the "
                             "headline's per-tick event); the per-call split (ms_per_call) is a separate run "
                             "with an event between calls",
        "vs_headline": min(two["device_ms_per_step"], three["device_ms_per_step"]) / headline_ms,
        "vs_headline_what": "the message path's device time per step with the better of two and three shard "
                            "pipelines, over the headline's ms_per_step on the same box (the calls one after "
                            "another on one queue: calls_ms_sum_vs_headline)",
        "roofline": {"kernel": "mraft_handle_append_entries (whole call: claims + set heads, main and deferred launches)", "bound": "hbm",
                     "algorithmic_bytes": hb, "achieved": hb / ms["handle"] / 1e6, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": hb / (ms["handle"] / 1e3) / HBM_PEAK,
                     "sets": hw["sets"], "merges": hw["merges"]},
        "fold_roofline": {"kernel": "mraft_process_append_replies (whole call: claim + k_fold + k_fold_tail)", "bound": "hbm",
                          "algorithmic_bytes": 4 * fw["words"], "a1_log_bytes": 4 * fw["a1_log_words"],
                          "achieved": 4 * fw["words"] / ms["fold"] / 1e6, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                          "frac": 4 * fw["words"] / (ms["fold"] / 1e3) / HBM_PEAK,
                          "segments": fw["segments"], "a1_evaluations": fw["evaluations"],
                          "note": "tools/msg_words.py fold_words: a1 reads each range's top term and, unless it "
                                  "settles the range (currentTerm, or below it on a replica whose terms_sorted "
                                  "proof holds: include/mraft.h), Go's downward scan; k_fold folds the replies and "
                                  "probes each range's top word, k_fold_tail scans the ranges the probes left open"}}

    # -- steady state: config #3 ticked in place with Start between ticks
    out["steady_state_config3"] = steady_state(master, copies, lp, G, P, L, dev)

    # -- deferred-heavy batches
    md = message_path_deferred(master, copies, lp, G, P, L, dev)
    out["message_path_deferred"] = {
        "workload": "config #3 by reference with a stale second leader in every other group: the real leaders' "
                    "262,144 AppendEntries with 32,768 from the stale leaders (stale: to another follower, in place "
                    "of the real leader's message to it — 262,144 messages; each stale leader's row is read and "
                    "written in the batch, so every lp -> q item is deferred; cycles: in addition, "
                    "back to the real leader, 2-cycles of staged items, past the stage capacity the fallback's "
                    "parallel cycles); the handle call alone, vs the plain 262,144-message batch",
        **md}

    # -- config #5 election storm
    Ge, Pe, R = 65536, 7, 64
    st5, mask = synth_election_state(Ge, Pe, 8, seed=synth_seed(5), rounds=R)
    m5 = {k: torch.from_numpy(v).to(dev) for k, v in st5.items()}
    c5 = {k: v.clone() for k, v in m5.items()}
    mask_d = torch.from_numpy(mask).to(dev)
    e5 = Engine(Ge, Pe, 8, device=dev.index or 0, alloc=False)
    e5.set_stream(stream.cuda_stream)
    gf5 = torch.zeros(Ge, dtype=torch.int32, device=dev)
    t5 = []
    for i in range(steps + 1):
        for k, v in m5.items():
            c5[k].copy_(v)
        e5.bind(c5)
        a, b = ev(), ev()
        a.record(stream)
        e5.election_rounds(mask_d, gf5, where=DEVICE)
        b.record(stream)
        torch.cuda.synchronize()
        if i:
            t5.append(a.elapsed_time(b))
    out["election_storm_config5"] = {
        "workload": "config #5: 65,536 groups x 7 peers, 64 election rounds per launch (mraft_election_rounds)",
        "kernel_ms_mean": float(np.mean(t5)), "group_rounds_per_s": Ge * R / (float(np.mean(t5)) / 1e3),
        "groups_with_new_leader": int(((gf5.cpu().numpy() & 128) != 0).sum()), "bound": "valu",
        "roofline": valu_roofline(float(np.mean(t5)))}
    e5.close()

    # -- config #2
    G2, P2, L2 = 1024, 3, 256
    st2, lp2, _ = synth_tick_state(G2, P2, L2, seed=synth_seed(2))
    m2 = {k: torch.from_numpy(v).to(dev) for k, v in st2.items()}
    c2 = {k: v.clone() for k, v in m2.items()}
    lp2_d = torch.from_numpy(lp2).to(dev)
    e2 = Engine(G2, P2, L2, device=dev.index or 0, alloc=False)
    e2.set_tick_mode(TICK_FULL)  # the fused tick (MRAFT_TICK_AUTO would settle here after one light probe)
    e2.set_stream(stream.cuda_stream)
    gf2 = torch.zeros(G2, dtype=torch.int32, device=dev)
    t2 = []
    for i in range(4 * steps + 1):
        for k, v in m2.items():
            c2[k].copy_(v)
        e2.bind(c2)
        a, b = ev(), ev()
        a.record(stream)
        e2.replicate_tick(lp2_d, gf2, where=DEVICE)
        b.record(stream)
        torch.cuda.synchronize()
        if i:
            t2.append(a.elapsed_time(b))
    out["tick_config2"] = {
        "workload": "config #2: 1,024 groups x 3 peers x 256-entry logs (cache-resident, launch-bound)",
        "kernel_ms_mean": float(np.mean(t2)), "decisions_per_s": G2 / (float(np.mean(t2)) / 1e3)}
    e2.close()
    return out


CONFIG4_ANCHOR = os.path.join(ROOT, "profiles", "config4_n1_anchor.json")
VALU_PMC = os.path.join(ROOT, "profiles", "pmc_valu_config5.json")


def elect_src_sha() -> str:
    import hashlib
    h = hashlib.sha1()
    for f in ("mraft_elect.hip", "mraft_device.h"):
        h.update(open(os.path.join(ROOT, "multiraft_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:12]


def valu_roofline(kernel_ms: float) -> dict:
    """Config #5's roofline: VALU issue (tools/pmc_valu.py). The wave-level
    VALU instruction count of one k_election_rounds<7> launch, from the
    committed PMC pass of the same kernel source, over the chip's issue rate
    (1,024 SIMD-32, 2 cycles per wave64 instruction, 2.4 GHz) in this run's
    kernel time. None when no pass matches the source."""
    if not os.path.exists(VALU_PMC):
        return {"bound": "valu", "frac": None, "why": "no VALU PMC pass committed"}
    pm = json.load(open(VALU_PMC))
    insts = pm.get("counters_per_launch", {}).get("SQ_INSTS_VALU")
    if pm.get("kernel_src_sha") != elect_src_sha() or not insts:
        return {"bound": "valu", "frac": None, "why": "the committed VALU PMC pass is of another kernel source"}
    peak = 1024 * 2.4e9 / 2  # wave-instructions per second
    achieved = insts / (kernel_ms / 1e3)
    return {"bound": "valu", "achieved": achieved / 1e9, "peak": peak / 1e9,
            "unit": "G wave-instructions/s (VALU issue)", "frac": achieved / peak,
            "valu_insts_per_launch": insts, "valu_busy_pmc": pm.get("valu_busy"),
            "source": f"profiles/{os.path.basename(VALU_PMC)} ({pm.get('tag')})",
            "model": pm.get("model")}


def pmc_json_path(G: int, S: int) -> str:
    """The committed PMC traffic summary of the tick at G groups per GPU in S
    shards (tools/pmc_summary.py): pmc_traffic[_g<G>][_s<S>].json."""
    name = "pmc_traffic" + ("" if G == 65536 else f"_g{G}") + ("" if S == 1 else f"_s{S}") + ".json"
    return os.path.join(ROOT, "profiles", name)


def config4_one_gpu(dev, stream, steps=10, shards=(1, 2)):
    """BASELINE config #4 on ONE GPU: all 262,144 groups (config #3's
    generator and mix, the workload the N > 1 lines split N ways) ticked once
    per step, each step on its own fresh HBM-resident copy (as many as fit;
    ~21.5 GB each), timed like the headline (one marker per tick on each tick
    queue), once per shard count in `shards` (the copies restored in between):
    the N = 1 points of the strong-scaling series, one per S the N > 1 lines
    may use."""
    import torch

    from multiraft_amd import DEVICE, TICK_FULL, Engine, synth_seed, synth_tick_state
    G4, P, L = 262144, 5, 4096
    t = time.perf_counter()
    st, lp, _ = synth_tick_state(G4, P, L, seed=synth_seed(3), nthreads=cpu_share()["threads"])
    gen_s = time.perf_counter() - t
    master = {}
    for k in list(st):
        master[k] = torch.from_numpy(st.pop(k)).to(dev)
    clone_bytes = sum(v.numel() * 4 for v in master.values())
    free, _ = torch.cuda.mem_get_info(dev)
    pool = max(1, min(steps, int(free * 0.92 // clone_bytes)))
    clones = [{k: v.clone() for k, v in master.items()} for _ in range(pool)]
    lp_d = torch.from_numpy(lp).to(dev)
    gf = torch.zeros(G4, dtype=torch.int32, device=dev)
    eng = Engine(G4, P, L, device=dev.index or 0, alloc=False)
    eng.set_tick_mode(TICK_FULL)
    eng.set_stream(stream.cuda_stream)
    eng.bind(master)
    rd, wr, active = eng.replicate_tick_count(lp_d, where=DEVICE)
    algo = 4 * (rd + wr)
    out = {"workload": "config #4 on one GPU: 262,144 groups x 5 peers x 4,096-entry logs (config #3's "
                       "generator and mix; the N > 1 lines split it N ways), one tick per step on a fresh "
                       "copy, with 1 and with 2 tick shards (mraft_set_tick_shards)",
           "groups": G4, "steps": pool, "state_copy_gib": clone_bytes / 2**30, "generate_s": gen_s,
           "by_shards": {}}
    pj_traffic = {}
    for S in shards:
        pj = pmc_json_path(G4, S)
        if os.path.exists(pj):
            pm = json.load(open(pj))
            if pm.get("kernel_src_sha") == kernel_src_sha() and pm.get("shards", 1) == S:
                pj_traffic[S] = (pm.get("hbm_bytes_per_step", pm.get("hbm_bytes_per_launch")),
                                 f"profiles/{os.path.basename(pj)} ({pm.get('tag')})")
    for n, S in enumerate(shards):
        eng.set_tick_shards(S)
        qs = [stream] if S == 1 else [torch.cuda.ExternalStream(eng.shard_stream(s), device=dev) for s in range(S)]
        eng.bind(clones[-1])  # warm-up on a copy that is re-timed last
        eng.replicate_tick(lp_d, gf, where=DEVICE)
        eng.synchronize()
        if pool > 1 or n > 0:  # refresh the spent copies for the timed steps
            for c in (clones if n > 0 else clones[-1:]):
                for k in master:
                    c[k].copy_(master[k])
        torch.cuda.synchronize()
        marks = [[torch.cuda.Event(enable_timing=True) for _ in range(pool + 1)] for _ in qs]
        t_begin = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        t_begin.record(stream)
        for i in range(pool):
            eng.bind(clones[i])
            if i == 0:
                for q, m in zip(qs, marks):
                    m[0].record(q)
            eng.replicate_tick(lp_d, gf, where=DEVICE)
            for q, m in zip(qs, marks):
                m[i + 1].record(q)
        eng.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        span = max(t_begin.elapsed_time(m[-1]) for m in marks)
        launch = [[m[i].elapsed_time(m[i + 1]) for i in range(pool)] for m in marks]
        km = span / pool if S > 1 else float(np.mean(launch[0]))
        r = {"ms_per_step": dt / pool * 1e3, "decisions_per_s": G4 * pool / dt,
             "roofline": {"kernel": f"k_tick_group<5,false> x {S}", "bound": "hbm", "algorithmic_bytes": algo,
                          "achieved": algo / (km / 1e3) / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                          "frac": algo / (km / 1e3) / HBM_PEAK, "kernel_ms_mean": km,
                          "launch_ms_mean": [round(float(np.mean(x)), 4) for x in launch],
                          "active_groups": active,
                          "timing": ("HIP events around each launch" if S == 1 else
                                     "device span of the timed region / steps (first start marker to the last "
                                     "shard's end marker)")}}
        if S == 1:
            r["roofline"]["kernel_ms_steps"] = [round(x, 4) for x in launch[0]]
            r["roofline"]["kernel_ms_min"] = float(np.min(launch[0]))
        if S in pj_traffic:
            r["roofline"]["traffic"], r["roofline"]["traffic_source"] = pj_traffic[S]
        out["by_shards"][str(S)] = r
    eng.close()
    del clones, master
    torch.cuda.empty_cache()
    return out


def strong_scaling_ref(strong, world, G_total, shards=1) -> dict:
    """For N > 1 strong-scaling lines of config #4: the N = 1 point of the
    same series (all 262,144 groups on one GPU) with the same number of tick
    shards per GPU, as last measured by a one-GPU bench run
    (secondary.config4_one_gpu -> tools/write_anchor.py)."""
    if not (strong and world > 1 and G_total == 262144):
        return {}
    if not os.path.exists(CONFIG4_ANCHOR):
        return {"strong_scaling_reference_ms": None,
                "strong_scaling_reference": {"what": "no one-GPU config #4 anchor committed"}}
    a = json.load(open(CONFIG4_ANCHOR))
    by = a.get("by_shards") or {}
    e = by.get(str(shards))
    if e is None:
        return {"strong_scaling_reference_ms": None,
                "strong_scaling_reference": {"what": f"no one-GPU config #4 anchor with {shards} tick shard(s) "
                                                     f"committed (have: {sorted(by)})",
                                             "source": f"profiles/{os.path.basename(CONFIG4_ANCHOR)} ({a.get('tag')})"}}
    return {"strong_scaling_reference_ms": e.get("ms_per_step"),
            "strong_scaling_reference": {
                "what": "N = 1 point of this series: config #4's 262,144 groups on one GPU with the same "
                        f"tick shards per GPU ({shards}) (secondary.config4_one_gpu of a one-GPU bench.py run, "
                        "same generator and timing)",
                "shards_per_gpu": shards,
                "source": f"profiles/{os.path.basename(CONFIG4_ANCHOR)} ({a.get('tag')})",
                "ms_per_step": e.get("ms_per_step"), "kernel_ms_mean": e.get("kernel_ms_mean"),
                "decisions_per_s": e.get("decisions_per_s")}}


def placement_probe(copies, G, P, L, dev):
    """After the timed region (the copies are spent): the data-free traffic
    probe (tools/probe_place.hip: the tick's XCD-aware order, writes only)
    on every step's state copy, so the record shows that the slow steps are
    the copies whose memory takes the eight XCDs' writes slowly (DESIGN.md §5
    placement lottery). None if the probe library is not built."""
    import ctypes

    import torch
    path = os.path.join(ROOT, "tools", "libprobe_place.so")
    if not os.path.exists(path) or P < 5:
        return None
    lib = ctypes.CDLL(path)
    lib.probe_place.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    sink = torch.zeros(16, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ms = []
    for c in copies:
        t = ctypes.c_float()
        if lib.probe_place(c["log_term"].data_ptr(), G, P, L, sink.data_ptr(), ctypes.byref(t), 32) != 0:
            return None
        ms.append(round(t.value, 4))
    return {"what": "writes-only probe (tools/probe_place.hip mode 32) on each step's state copy after the "
                    "timed region, ms per copy, in step order", "ms": ms}


def cpu_baseline(G_total, P, L, seed, budget_s, rank):
    """The reference's tick timed on this host's cores, two restatements:
    the Go-shaped one (oracle/mraft_goshape.c: int64 Raft structs, 40-byte
    Entry slices, a fresh entries copy per message as appendOneRound makes,
    trunc + append, advanceCommitIndexForLeader's O((last-commit)*P) count) is
    the reported value; the engine-layout one (oracle/mraft_oracle.c, SoA
    int32, same control flow) is reported beside it. Both on bounded samples
    of the same seeded workload, fresh state per pass (restores untimed)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import GoShaped, Oracle  # test infrastructure: CPU baseline only

    from multiraft_amd import synth_tick_state
    share = cpu_share()
    threads = share["threads"]

    def timed(make, tick, budget, nt, groups):
        done, spent, w0, last = 0, 0.0, time.perf_counter(), time.perf_counter()
        while spent < budget and time.perf_counter() - w0 < 3 * budget + 10:
            obj = make()  # untimed restore of the pristine state
            t = time.perf_counter()
            tick(obj, nt)
            spent += time.perf_counter() - t
            done += groups
            if time.perf_counter() - last > 20:
                last = time.perf_counter()
                log(rank, f"cpu baseline ({nt} threads): {done} decisions in {spent:.1f} s so far")
        return done / spent, done, spent

    # Go-shaped restatement (the value)
    Gg = min(2048, G_total)
    stg, lpg, _ = synth_tick_state(G_total, P, L, seed=seed, g_begin=0, g_end=Gg)
    gsh = GoShaped(Gg, P, L, stg)

    def make_go():
        gsh.reset(threads)
        return gsh

    def tick_go(g, nt):
        assert g.replicate_tick(lpg, nthreads=nt) == 0

    g1, _, _ = timed(make_go, tick_go, min(1.0, budget_s / 8), 1, Gg)
    gt, gdone, gspent = timed(make_go, tick_go, budget_s / 2, threads, Gg)
    gsh.close()
    # engine-layout (SoA int32) restatement
    Gs = min(8192, G_total)
    st, lp, _ = synth_tick_state(G_total, P, L, seed=seed, g_begin=0, g_end=Gs)
    o = Oracle(Gs, P, L, st)

    def make_soa():
        for k, v in st.items():
            np.copyto(o.st[k], v)
        return o

    def tick_soa(obj, nt):
        obj.replicate_tick(lp, nthreads=nt)

    s1, _, _ = timed(make_soa, tick_soa, min(2.0, budget_s / 6), 1, Gs)
    stt, sdone, sspent = timed(make_soa, tick_soa, budget_s / 3, threads, Gs)
    log(rank, f"cpu baseline: go-shaped {gt:.4g} decisions/s on {threads} threads ({g1:.4g} on 1); "
              f"SoA {stt:.4g} ({s1:.4g} on 1)")
    return {"value": gt, "unit": "decisions/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "cores_source": (f"len(os.sched_getaffinity(0)) = {share['affinity']}"
                             + (f", capped by the cgroup CPU quota ({share['cgroup_quota']})"
                                if share["cgroup_quota"] else "")),
            "compiler": "gcc -O3 -march=x86-64-v3 (oracle/Makefile)",
            "sample": (f"oracle/mraft_goshape.c: the tick on the reference's data shapes (int64 Raft "
                       f"structs, 40-byte Entry slices, per-message entries copies, a1's "
                       f"O((last-commit)*P) loop) over groups 0..{Gg - 1} of the same seeded config-#3 "
                       f"workload ({P} peers, L={L}), fresh state per pass; {threads} threads: "
                       f"{gdone} decisions in {gspent:.2f} s; 1 thread: {g1:.4g} decisions/s; excludes "
                       f"the gob persist()/labrpc encoding the Go reference also pays per handler"),
            "single_thread_value": g1,
            "soa_int32": {"value": stt, "single_thread_value": s1, "cores": threads,
                          "sample": (f"oracle/mraft_oracle.c (engine layout, same control flow) over "
                                     f"groups 0..{Gs - 1}: {sdone} decisions in {sspent:.2f} s")}}


def permute_groups(st, lp, G, P, L, how):
    """Dispatch-order experiment: the same groups in another order. lpt-xcd
    sorts each XCD's contiguous range (the tick's XCD-aware mapping) by
    descending estimated work (entries past each follower's prev)."""
    ld = np.arange(G) * P + lp
    last = st["last_index"][ld].astype(np.int64)
    nxt = st["next_index"].reshape(G * P, P)[ld]
    work = np.clip(last[:, None] + 1 - nxt, 0, None).sum(axis=1)
    if how == "random":
        perm = np.random.default_rng(0).permutation(G)
    elif how.startswith("taillight"):
        # natural order, except that each XCD range ends with its lightest
        # groups (the last `frac` of its dispatch order): a lighter tail
        frac = float(how[len("taillight"):] or 0.12)
        per = G // 8
        parts = []
        for x in range(8):
            idx = np.arange(x * per, (x + 1) * per)
            k = int(per * frac)
            light = idx[np.argsort(work[idx], kind="stable")[:k]]
            rest = np.setdiff1d(idx, light, assume_unique=True)
            parts.append(np.concatenate([rest, light[::-1]]))
        perm = np.concatenate(parts + [np.arange(8 * per, G)])
    else:
        per = G // 8
        perm = np.concatenate([x * per + np.argsort(-work[x * per:(x + 1) * per], kind="stable")
                               for x in range(8)] + [np.arange(8 * per, G)])
    out = {}
    for k, v in st.items():
        w = v.size // G
        out[k] = np.ascontiguousarray(v.reshape(G, w)[perm].reshape(-1))
    # the leader's matchIndex/nextIndex rows are per replica; leader_peer per group
    return out, np.ascontiguousarray(lp[perm])


def describe_workload(strong, world, G_total, P, L, config, dist_on, rccl, backend):
    if strong and world > 1:
        w = ((f"config #4: " if G_total == 262144 else "")
             + f"{G_total:,} groups x {P} peers x {L:,}-entry logs split over {world} "
             f"GPUs (strong scaling; config #3's generator and mix)")
    elif strong:
        w = f"{G_total:,} groups x {P} x {L:,} on one GPU (config #4's total; config #3 mix)"
    else:
        w = f"config #{config}" + (f" x {world} ranks (weak scaling)" if world > 1 else "")
    w += " fused replication tick (a3+a4+a2+a1) with the GetState export fused in"
    if dist_on:
        w += (" + RCCL all-gather of commit/term words (C ABI, mraft_allgather_status)"
              if rccl else f" + {backend} all-gather of commit/term words (rehearsal)")
    if config == 2:
        w += " [cache-resident working set: not an HBM measurement]"
    return w


def stream_plan(shards: int, rccl: bool, fanin_cus: int, fanin: str) -> dict:
    """The streams and hardware queues one rank uses (include/mraft.h), and
    what orders the fan-in: the engine owns every queue it creates and
    destroys them in mraft_destroy. Asserted by tests/test_bench_launch.py for
    the N > 1 default (2 shards + the RCCL fan-in)."""
    masked = rccl and fanin_cus > 0
    plan = {
        "engine_stream": "pooled HIP stream (torch's and the engine's; carries no tick when shards > 1)",
        "tick_queues": shards if shards > 1 else 0,
        "tick_queue_mask": ("every CU but the fan-in's %d" % fanin_cus if masked else "every CU")
        if shards > 1 else None,
        "tick_on": "engine stream" + (" (masked off the fan-in's CUs)" if masked else "") if shards == 1
        else f"{shards} shard queues",
        "fanin_queue": (1 if masked else 0) if rccl else None,
        "fanin_on": None if not rccl else ("engine stream" if fanin == "inline" else
                                           "fan-in queue (%d CUs)" % fanin_cus if masked else "fan-in stream (pooled)"),
        "fanin_waits_for": None if not rccl else "the end marker of every shard's tick",
    }
    plan["dedicated_queues"] = plan["tick_queues"] + (plan["fanin_queue"] or 0) + (1 if masked and shards == 1 else 0)
    return plan


def spawn_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N rank processes (one per GPU) and
    wait for them. The parent never touches the GPU (it only forwards the
    arguments); rank 0's stdout is the result line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            c = p.poll()
            if c is None:
                continue
            pending.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in pending:  # one rank failed: end the others (exact PIDs)
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without a torch.distributed launcher bench.py starts "
                         "them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--groups", type=int, default=0,
                    help="groups per GPU (weak scaling); default 65,536 (config #3) on one GPU")
    ap.add_argument("--global-groups", type=int, default=0,
                    help="fixed total split over the ranks (strong scaling); default 262,144 "
                         "(config #4) with more than one rank")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3],
                    help="BASELINE config: 3 = 65,536 x 5 x 4,096 (headline); 2 = 1,024 x 3 x 256 "
                         "(cache-resident: not an HBM measurement)")
    ap.add_argument("--peers", type=int, default=5)
    ap.add_argument("--log", type=int, default=4096, help="log capacity L")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary lines (message path, configs #5 and #2) of a one-GPU run")
    ap.add_argument("--pmc-json", default="",
                    help="PMC traffic summary (default: profiles/pmc_traffic.json for 65,536 groups "
                         "per GPU, profiles/pmc_traffic_g<G>.json otherwise)")
    ap.add_argument("--log-pad", type=int, default=0,
                    help="experiment: pad every log row by this many entries (capacity L + pad, "
                         "same logs and algorithmic words; only the row stride changes)")
    ap.add_argument("--group-order", default="natural",
                    help="experiment: permute the groups (same work, different dispatch order): "
                         "natural, lpt-xcd, random, taillight[FRAC]")
    ap.add_argument("--fanin-at-1", action="store_true",
                    help="rehearsal: run the per-tick RCCL fan-in even with one rank (a one-rank "
                         "communicator: exercises the C-ABI gather + overlap path on a single GPU)")
    ap.add_argument("--fanin", default="overlap", choices=["overlap", "inline"],
                    help="RCCL fan-in placement: overlap = on the engine's fan-in stream beside the "
                         "next tick; inline = on the tick's stream")
    ap.add_argument("--fanin-cus", type=int, default=8,
                    help="CUs reserved for the fan-in stream (mraft_fanin_reserve_cus; 0 = none): "
                         "without them the overlapped gather queues for CU slots behind the next "
                         "tick (0.31 ms vs 0.015 ms on one rank, profiles/r2_v1_fanin_cus*.json)")
    ap.add_argument("--fanin-marks", default="chain", choices=["chain", "legacy"],
                    help="timing/ordering markers on the tick stream: chain = one per tick, shared by "
                         "the timing and the fan-in's wait (MRAFT_FANIN_ORDERED); legacy = round 2's "
                         "start + end marks per tick plus the fan-in's own event (A/B only)")
    ap.add_argument("--extra-marks", type=int, default=0,
                    help="experiment: record this many extra (untimed) events on the tick stream "
                         "after every tick")
    ap.add_argument("--shards", type=int, default=2,
                    help="independent group shards per GPU, one engine and one stream each, ticked "
                         "in turn every step: shard s's tick i+1 follows its tick i on its own stream "
                         "and overlaps the other shards' ticks, so one launch's last generation of "
                         "groups shares the device with the next launch's first (DESIGN.md §6; "
                         "1 = one launch per step)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch plumbing only (no GPU call): start the ranks, build every rank's "
                         "shard of the seeded workload, run the control plane and print the line "
                         "with value null")
    ap.add_argument("--dist-backend", default="nccl",
                    help="fan-in data path: nccl = the library's RCCL all-gather over xGMI (C ABI); "
                         "gloo = host gather through torch.distributed (CPU rehearsal)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # The result line is the only thing on stdout: libraries that print there
    # (RCCL's version banner at communicator init) are sent to stderr.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist_on = world > 1 or args.fanin_at_1
    import torch
    import torch.distributed as dist

    if not args.dry_run:
        ndev = torch.cuda.device_count()
        local_dev = local % max(ndev, 1)  # gloo rehearsals may share one GPU
        torch.cuda.set_device(local_dev)
        dev = torch.device("cuda", local_dev)
    if dist_on:
        if world == 1:  # --fanin-at-1 without a launcher
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29561"), ("RANK", "0"),
                         ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        # control plane (barriers, the communicator id, max-over-ranks time) on
        # the host; the data path (the fan-in) is the library's RCCL gather
        dist.init_process_group("gloo")

    from multiraft_amd import DEVICE, TICK_FULL, Engine, synth_seed, synth_tick_state
    from multiraft_amd.router import RcclFanIn, allgather_status_packed

    if args.config == 2:
        args.groups, args.peers, args.log = 1024, 3, 256
    strong = bool(args.global_groups) or (world > 1 and not args.groups)
    if strong:
        G_total = args.global_groups or 262144  # config #4 (shardkv/config.go:338-380 deployment)
        if G_total % world:
            raise SystemExit("--global-groups must be a multiple of the world size")
        G = G_total // world
    else:
        G = args.groups or 65536
        G_total = G * world
    P, L, K, W = args.peers, args.log, args.steps, args.warmup
    seed = synth_seed(args.config)
    t = time.perf_counter()
    st, lp, _ = synth_tick_state(G_total, P, L, seed=seed, g_begin=rank * G, g_end=(rank + 1) * G,
                                 nthreads=min(16, os.cpu_count() or 1))
    log(rank, f"generated {G}x{P}x{L} state in {time.perf_counter() - t:.1f}s")
    if args.group_order != "natural":
        st, lp = permute_groups(st, lp, G, P, L, args.group_order)
    if args.log_pad:
        st["log_term"] = np.ascontiguousarray(
            np.pad(st["log_term"].reshape(G * P, L), ((0, 0), (0, args.log_pad))).reshape(-1))
        L = L + args.log_pad

    rccl = dist_on and args.dist_backend == "nccl"
    if args.dry_run:
        S_dry = args.shards if (args.shards > 1 and G >= args.shards) else 1
        plans = [stream_plan(S_dry, rccl, args.fanin_cus, args.fanin)]
        if dist_on:
            dist.barrier()
            n = torch.tensor([float(G)], dtype=torch.float64)
            dist.all_reduce(n)
            assert int(n.item()) == G_total, "the shards do not cover the workload"
            plans = [None] * world
            dist.all_gather_object(plans, stream_plan(S_dry, rccl, args.fanin_cus, args.fanin))
        if rank == 0:
            print(json.dumps({
                "metric": METRIC, "value": None, "unit": "decisions/s", "n_gpus": world,
                "steps": K, "warmup": W, "higher_is_better": True,
                "scaling": "strong" if strong else "weak", "dry_run": True,
                "config": {"workload": describe_workload(strong, world, G_total, P, L, args.config,
                                                         dist_on, rccl, args.dist_backend),
                           "groups_per_gpu": G, "global_groups": G_total, "peers": P,
                           "log_capacity": L, "shard_of_rank0": [0, G],
                           "leaders_in_shard_rank0": int((lp >= 0).sum()),
                           "shards_per_gpu": S_dry, "stream_plan_by_rank": plans},
                **strong_scaling_ref(strong, world, G_total, S_dry)}),
                file=result_out, flush=True)
        if dist_on:
            dist.barrier()
            dist.destroy_process_group()
        return

    # Ranks allocate in turn (a CPU rehearsal may put several ranks on one GPU).
    for r in range(world):
        if r == rank:
            master = {k: torch.from_numpy(v).to(dev) for k, v in st.items()}
            clone_bytes = sum(v.numel() * 4 for v in master.values())
            free, _ = torch.cuda.mem_get_info(dev)
            pool = max(1, min(K + 1, int(free * 0.9 // clone_bytes)))
            clones = [{k: v.clone() for k, v in master.items()} for _ in range(pool)]
            torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
    del st
    restore = pool < K + 1
    log(rank, f"{pool} state copies of {clone_bytes / 2**30:.2f} GiB each"
              f"{' (restore inside timed steps)' if restore else ''}")

    # Group shards (--shards): the engine splits every tick into S contiguous
    # group ranges, each launched on a hardware queue the engine owns
    # (mraft_set_tick_shards); shard s's tick i+1 follows only its own tick i.
    S = args.shards if (args.shards > 1 and not restore and G >= args.shards) else 1
    eng = Engine(G, P, L, device=local_dev, alloc=False)
    # The measured path is the fused tick (k_tick_group): on a fresh config-#3
    # copy every group needs it, and MRAFT_TICK_AUTO (the engine default)
    # chooses it after one light probe; set here so no warmup setting changes it.
    eng.set_tick_mode(TICK_FULL)
    eng.set_tick_shards(S)
    if rccl and args.fanin_cus:
        # the tick's queues are masked off the fan-in's reserved CUs (include/mraft.h)
        eng.fanin_reserve_cus(args.fanin_cus)
    if S == 1 and rccl and args.fanin_cus:
        stream = torch.cuda.ExternalStream(eng.stream(), device=dev)
    else:
        # A dedicated (non-null) stream shared by torch and the engine, so the
        # events below bracket exactly the engine's kernels (S = 1) or fork
        # the shard queues after torch's work (S > 1).
        stream = torch.cuda.Stream(dev)
        eng.set_stream(stream.cuda_stream)
    torch.cuda.set_stream(stream)
    tick_streams = ([stream] if S == 1 else
                    [torch.cuda.ExternalStream(eng.shard_stream(si), device=dev) for si in range(S)])
    lp_d = torch.from_numpy(lp).to(dev)
    gf_d = torch.zeros(G, dtype=torch.int32, device=dev)
    plan = stream_plan(S, rccl, args.fanin_cus, args.fanin)
    on_host = dist_on and not rccl
    # Per-step GetState export blocks (commitIndex | term<<1|leader, one buffer
    # so the router's fan-in is ONE collective per tick) and their gathers:
    # never reused within a run, so a step's all-gather can overlap the next
    # step's tick on the fan-in stream with no buffer hazard.
    nbuf = W + K
    status = torch.zeros((nbuf, 2 * G), dtype=torch.int32, device=dev)
    fan = RcclFanIn(eng, rank, world) if rccl else None
    overlap = args.fanin == "overlap"
    gathered = (torch.empty((nbuf, world * 2 * G), dtype=torch.int32, device=dev)
                if fan is not None else None)
    comm_stream = None
    if fan is not None:
        comm_stream = (torch.cuda.ExternalStream(eng.fanin_stream(), device=dev) if overlap
                       else stream)

    # Algorithmic words of one tick on the pristine state.
    eng.bind(master)
    rd, wr, active = eng.replicate_tick_count(lp_d, where=DEVICE)
    algo_bytes = 4 * (rd + wr)

    # Per-launch kernel timing on the tick's queue(s). With nothing else on a
    # queue between ticks (no restores) one marker between consecutive ticks
    # serves as the end of one and the start of the next, and the fan-in
    # stream waits on that same marker (MRAFT_FANIN_ORDERED): one marker
    # packet per tick on each tick queue. Every extra marker there costs the
    # step a few microseconds of idle device (the round-2 fan-in runs recorded
    # four per tick: ~20 us per step beyond the kernel).
    chain = not restore and args.fanin_marks == "chain"
    marks_s = [[torch.cuda.Event(enable_timing=True) for _ in range(K + 1 if chain else 2 * K)]
               for _ in range(S)]
    t_begin = torch.cuda.Event(enable_timing=True)
    t_end = [torch.cuda.Event(enable_timing=True) for _ in range(S)]
    extra = [torch.cuda.Event() for _ in range(args.extra_marks)]

    # The all-gather, timed on its own stream (reported beside the step).
    ag_marks = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)] if fan is not None else []
    ag_ms = []

    def mark_start(i, si=0):
        return marks_s[si][i] if chain else marks_s[si][2 * i]

    def mark_end(i, si=0):
        return marks_s[si][i + 1] if chain else marks_s[si][2 * i + 1]

    def step(i, timed):
        if restore:  # not enough HBM for a copy per step: restore inside the step
            c = clones[i % pool]
            for k in c:
                c[k].copy_(master[k], non_blocking=True)
        else:
            c = clones[i] if timed else clones[K]
        j = i if timed else K + i  # timed steps use blocks 0..K-1, warmup K..K+W-1
        eng.bind(c)
        if timed and (i == 0 or not chain):
            for si in range(S):
                mark_start(i, si).record(tick_streams[si])
        # the tick with the GetState export fused in (one call per step; S
        # launches on the engine's shard queues when S > 1)
        eng.replicate_tick_export(lp_d, gf_d, status[j, :G], status[j, G:], where=DEVICE)
        if timed:
            for si in range(S):
                mark_end(i, si).record(tick_streams[si])
        for x in extra:  # experiment: marker packets between ticks
            x.record(tick_streams[0])
        if dist_on:  # the shard router's fan-in
            if on_host:
                t1 = time.perf_counter()
                allgather_status_packed(status[j].cpu())
                if timed:
                    ag_ms.append((time.perf_counter() - t1) * 1e3)
            else:
                # RCCL all-gather of this tick's words (C ABI). Overlapped: on
                # the fan-in stream after the tick, beside the next tick (which
                # writes another block), so the next batch never waits for it.
                # Untimed steps let the engine order it (it waits for every
                # shard's last launch, include/mraft.h).
                ordered = False
                if timed:
                    # the gather (and its start mark) waits on every shard's
                    # end marker: the fan-in stream (overlap) or the engine
                    # stream (inline; the engine would join the shards there)
                    for si in range(S):
                        comm_stream.wait_event(mark_end(i, si))
                    ordered = overlap
                    ag_marks[2 * i].record(comm_stream)
                fan.gather(status[j], gathered[j], overlap=overlap, ordered=ordered)
                if timed:
                    ag_marks[2 * i + 1].record(comm_stream)

    for i in range(W):
        step(i, False)
    eng.synchronize()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t_begin.record(stream)  # the first tick's shard queues fork from this stream after it
    for i in range(K):
        step(i, True)
    for si in range(S):
        t_end[si].record(tick_streams[si])
    eng.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist_on:
        dist.barrier()
    # device time of the timed region: from the first launch's start marker to
    # the last shard's end
    span_ms = max(t_begin.elapsed_time(e) for e in t_end)
    launch_ms = [[mark_start(i, si).elapsed_time(mark_end(i, si)) for i in range(K)] for si in range(S)]
    if S > 1:
        # the shards' last step (a pristine copy) equals one launch over every
        # group on the same input: flags and export words
        ck = clones[K]
        for k in ck:
            ck[k].copy_(master[k])
        one = Engine(G, P, L, device=local_dev, alloc=False)  # one launch, on torch's stream
        one.set_tick_mode(TICK_FULL)
        one.set_stream(stream.cuda_stream)
        one.bind(ck)
        gf1 = torch.zeros_like(gf_d)
        st1 = torch.zeros_like(status[0])
        one.replicate_tick_export(lp_d, gf1, st1[:G], st1[G:], where=DEVICE)
        one.synchronize()
        one.close()
        assert torch.equal(gf1, gf_d) and torch.equal(st1, status[K - 1]), "sharded tick differs from one launch"
    # per step: one launch (S = 1), or the shards' launches overlapping: the
    # step's share of the device span, apportioned by its launches' durations
    if S == 1:
        ker_ms = launch_ms[0]
    else:
        w = np.sum(np.array(launch_ms), axis=0)
        ker_ms = list(w / w.sum() * span_ms)
        log(rank, f"{S} shards: device span {span_ms / K:.4f} ms per step; shard launch ms mean "
                  + " ".join(f"{float(np.mean(x)):.4f}" for x in launch_ms))
    log(rank, "tick kernel ms per step: " + " ".join(f"{x:.3f}" for x in ker_ms))
    flags = gf_d.cpu().numpy()
    if fan is not None:
        ag_ms = [ag_marks[2 * i].elapsed_time(ag_marks[2 * i + 1]) for i in range(K)]
        # the last tick's words, gathered over RCCL, equal every rank's export
        want = [torch.zeros(2 * G, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(want, status[K - 1].cpu())
        assert torch.equal(gathered[K - 1].cpu(), torch.cat(want)), "RCCL fan-in words differ"
    if dist_on:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        km = torch.tensor([float(np.mean(ker_ms))], dtype=torch.float64)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        ker_max_ms = float(km.item())

    ker_s = float(np.mean(ker_ms)) / 1e3
    achieved = algo_bytes / ker_s
    traffic, traffic_src = None, None
    if not args.pmc_json:
        args.pmc_json = pmc_json_path(G, S)
    if os.path.exists(args.pmc_json):
        # PMC traffic of this exact kernel source and config, from the
        # committed rocprofv3 summary (tools/profile_round.sh + pmc_summary.py).
        try:
            pm = json.load(open(args.pmc_json))
            if ((pm.get("groups"), pm.get("peers"), pm.get("log"), pm.get("shards", 1)) == (G, P, L, S)
                    and pm.get("kernel_src_sha") == kernel_src_sha()):
                traffic = pm.get("hbm_bytes_per_step", pm.get("hbm_bytes_per_launch"))
                traffic_src = f"profiles/{os.path.basename(args.pmc_json)} ({pm.get('tag')})"
        except Exception:
            traffic = None
    workload = describe_workload(strong, world, G_total, P, L, args.config, dist_on, rccl,
                                 args.dist_backend)
    out = {
        "metric": METRIC,
        "value": G_total * K / dt,
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": dt / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic: seeded config-#{args.config} generator (include/mraft_synth.h), fresh "
                "HBM-resident copy per step",
        "config": {"workload": workload,
                   "groups_per_gpu": G, "global_groups": G_total, "peers": P, "log_capacity": L,
                   "committed_groups_last_step": int(((flags & 2) != 0).sum()),
                   "active_groups": active, "restore_in_timed_step": restore,
                   "allgather_ms_mean": float(np.mean(ag_ms)) if ag_ms else None,
                   "allgather_bytes_per_rank": 8 * G if dist_on else 0,
                   "allgather_placement": (args.fanin if fan is not None else None),
                   "fanin_reserved_cus": args.fanin_cus if fan is not None else 0,
                   "tick_stream_marks_per_step": (1 if chain else 2) + args.extra_marks
                   + (1 if fan is not None and not chain else 0),
                   "step_minus_kernel_ms": dt / K * 1e3 - float(np.mean(ker_ms)),
                   "shards_per_gpu": S, "tick_mode": "MRAFT_TICK_FULL (the fused tick; MRAFT_TICK_AUTO, the default, chooses it on this workload)",
                   "shard_pipelining": (None if S == 1 else
                                        f"mraft_set_tick_shards({S}): one engine, {S} contiguous group "
                                        f"ranges of ~{G // S} on {S} hardware queues the engine owns; each "
                                        "shard's tick i+1 follows its own tick i, the shards' launches "
                                        "overlap (DESIGN.md §6)"),
                   "stream_plan": plan},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK,
                     "traffic": traffic,
                     "traffic_unit": ("HBM bytes per step: FETCH_SIZE+WRITE_SIZE, calibrated, summed over the "
                                      f"step's {S} launch(es)"),
                     "traffic_source": traffic_src,
                     "kernel": f"k_tick_group<{P},false>",
                     "algorithmic_read_bytes": 4 * rd, "algorithmic_write_bytes": 4 * wr,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "algorithmic_bytes_per_decision": algo_bytes / max(active, 1),
                     "kernel_ms_mean": ker_s * 1e3,
                     "kernel_ms_min": float(np.min(ker_ms)) if S == 1 else None,
                     "kernel_ms_median": float(np.median(ker_ms)) if S == 1 else None,
                     ("kernel_ms_steps" if S == 1 else "kernel_ms_steps_apportioned"):
                         [round(float(x), 4) for x in ker_ms],
                     "launch_ms_steps": None if S == 1 else [[round(float(x), 4) for x in sh] for sh in launch_ms],
                     "device_ms_per_step": span_ms / K,
                     "launches_per_step": S,
                     "launch_ms_mean": [round(float(np.mean(x)), 4) for x in launch_ms],
                     "timing": ("one launch per step: HIP events around each launch" if S == 1 else
                                f"{S} overlapping launches per step (one per shard and stream): "
                                "kernel_ms_mean = device time of the timed region / steps (events "
                                "from the first launch's start to the last shard's end); "
                                "kernel_ms_steps_apportioned splits it by each step's launch durations "
                                "(derived, not measured per step); launch_ms_steps / launch_ms_mean = "
                                "each shard's measured launch durations, overlap included"),
                     "note": ("each step ticks its own fresh state copy; copies whose log image sits in "
                              "physical memory that takes streaming writes ~10 % slower run ~13 % slower "
                              "(DESIGN.md §5 placement lottery): kernel_ms_steps shows both populations"),
                     "scope": "rank 0's GPU" if world > 1 else "the GPU"},
        "cpu_baseline": None,
    }
    if world > 1:
        out["roofline"]["kernel_ms_mean_max_over_ranks"] = ker_max_ms
    out.update(strong_scaling_ref(strong, world, G_total, S))
    if world == 1 and not restore:
        pp = placement_probe(clones[:K], G, P, L, dev)
        if pp is not None:
            # the two populations the probe separates (two-means on its times),
            # each with its mean kernel time and HBM fraction; `frac` above
            # stays the mean over every step
            pm = np.array(pp["ms"])
            lo_c, hi_c = float(pm.min()), float(pm.max())
            for _ in range(20):
                cut = (lo_c + hi_c) / 2
                if not (pm <= cut).any() or not (pm > cut).any():
                    break
                lo_c, hi_c = float(pm[pm <= cut].mean()), float(pm[pm > cut].mean())
            if (pm <= cut).any() and (pm > cut).any() and hi_c > 1.05 * lo_c:
                km = np.array(ker_ms)
                pops = {}
                for name, sel in (("fast_memory", pm <= cut), ("slow_memory", pm > cut)):
                    kms = float(km[sel].mean())
                    pops[name] = {"steps": int(sel.sum()), "kernel_ms_mean": round(kms, 4),
                                  "frac": algo_bytes / (kms / 1e3) / HBM_PEAK}
                if S > 1:  # per-step device time is apportioned (derived) with overlapping shards
                    for v in pops.values():
                        v["apportioned"] = True
                pp["populations"] = pops
                pp["corr_with_kernel_ms" if S == 1 else "corr_with_apportioned_ms"] = float(np.corrcoef(pm, km)[0, 1])
            out["roofline"]["placement_probe"] = pp
    if (world == 1 and args.config == 3 and not args.no_secondary and G == 65536 and P == 5 and L == 4096
            and fan is None):
        out["secondary"] = secondary(master, clones, lp, G, P, L, stream, dev,
                                     dt / K * 1e3)  # reuses the spent copies
        # config #4's N = 1 anchor: free config #3's copies, then all 262,144 groups on this GPU
        eng.close()
        del clones, master
        ck = None
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        c4 = config4_one_gpu(dev, stream, shards=(1, 2))
        out["secondary"]["config4_one_gpu"] = c4
        for sk, c in c4["by_shards"].items():
            log(rank, f"config #4 on one GPU, {sk} shard(s): {c['ms_per_step']:.4f} ms/step, device "
                      f"{c['roofline']['kernel_ms_mean']:.4f} ms ({c['roofline']['frac']:.3f} of 8 TB/s) over "
                      f"{c4['steps']} fresh copies")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # at N = 1 only (the driver's N > 1 lines carry cpu_baseline null)
        out["cpu_baseline"] = cpu_baseline(G_total, P, L, seed, args.cpu_seconds, rank)
    if rank == 0:
        print(json.dumps(out), file=result_out, flush=True)
    if dist_on:
        dist.barrier()
    if fan is not None:
        eng.fanin_synchronize()
        fan.close()
    eng.close()  # waits for and destroys the engine's shard and fan-in queues
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
