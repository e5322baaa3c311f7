"""The reference's Raft test scenarios (src/raft/test_test.go) on many groups
at once: every group of ONE engine runs its own scenario with its own seed —
partitions, crashes and restarts from persisted bytes, unreliable and
reordering networks, snapshots and InstallSnapshot — and every tick makes one
batched engine call per phase for all groups (tests/sim2b.py MultiSim). Each
group must pass its scenario's assertions: agreement and in-order apply on
every committed index (config.go:144-163), at most one leader per term
(:438-468), one() / nCommitted (:502-622), and the scenario's own checks.

The CPU runs drive the oracle; the GPU runs drive libmraft_hip.so with 1,024
groups per engine (message sets from many leaders per HandleAppendEntries
call, reply segments of many groups per fold, the compacted applier), and a
smaller mix is run on both and must produce the same engine state and the
same applied logs."""
import numpy as np
import pytest

from oracle_lib import Oracle, assert_states_equal
from sim2b import SCENARIOS, MultiSim, run_many

P3 = [n for n, s in SCENARIOS.items() if s.P == 3]
P5 = [n for n, s in SCENARIOS.items() if s.P == 5]
P7 = [n for n, s in SCENARIOS.items() if s.P == 7]


def _oracle(G, P, L, st):
    return Oracle(G, P, L, st)


def _gpu(G, P, L, st):
    from multiraft_amd import Engine
    e = Engine(G, P, L)
    e.load_state(st)
    return e


def _batched(sim, min_items):
    """The batched paths really ran batched."""
    c = sim.calls
    assert max(c["handle_append_entries"][1] / c["handle_append_entries"][0], 0) > 1
    assert c["handle_append_entries"][1] >= min_items
    return {k: v for k, v in sorted(c.items())}


def test_scenarios_cover_every_server_count():
    assert len(P3) + len(P5) + len(P7) == len(SCENARIOS)


@pytest.mark.parametrize("names,groups", [(P3, 64), (P5, 24), (P7, 8)], ids=["P3", "P5", "P7"])
def test_many_groups_oracle(names, groups):
    sim = run_many(_oracle, names, groups)
    assert sim.G == groups and not sim.failures
    _batched(sim, groups)
    # every log a Raft run reaches is sorted, and the engine's rules keep the
    # proof through appends, Start, snapshots, installs and restarts
    # (include/mraft.h MRAFT_TERMS_SORTED): a1 never needs Go's downward scan
    assert (sim.eng.store_state()["terms_sorted"] == 1).all()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("names,groups", [(P3, 1024), (P5, 1024), (P7, 256)], ids=["P3", "P5", "P7"])
def test_many_groups_gpu(names, groups):
    sim = run_many(_gpu, names, groups, compact_apply=True)
    assert sim.G == groups and not sim.failures
    assert (sim.eng.store_state()["terms_sorted"] == 1).all()
    calls = _batched(sim, 10 * groups)
    installs = sum(g.installs for g in sim.groups)
    restores = calls.get("restore", [0])[0]
    print(f"\n{groups} groups x {sim.P}: {sim.now} ticks, {installs} snapshot installs, {restores} restarts; "
          + ", ".join(f"{k} {v[0]} calls / {v[1]} items" for k, v in calls.items()))


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("names,groups", [(P3, 128), (P5, 48)], ids=["P3", "P5"])
def test_many_groups_gpu_equals_oracle(names, groups):
    """The same mixed history on the GPU and on the oracle: identical engine
    state (logs, rings, leader views, persistence bits) and applied logs."""
    sims = []
    for mk in (_oracle, _gpu):
        scs = [SCENARIOS[n] for n in names]
        specs = [(scs[g % len(scs)], 1000 + g) for g in range(groups)]
        sims.append(MultiSim(mk, scs[0].P, max(s.L for s in scs), specs).run())
    o, d = sims
    assert o.now == d.now
    G, P, L = o.G, o.P, o.L
    assert_states_equal(d.eng.store_state(), o.eng.store_state(), G, P, L, "many-group history")
    for a, b in zip(o.groups, d.groups):
        assert a.logs == b.logs and a.rpc_count == b.rpc_count
    assert {k: v for k, v in o.calls.items()} == {k: v for k, v in d.calls.items()}
    assert np.array_equal(o.alive, d.alive)
