"""Config #1: the reference's 2A/2B/2C/2D test scenarios
(src/raft/test_test.go), replayed by the deterministic harness in
tests/sim2b.py through the engine's C ABI. The CPU run (oracle backend) checks
the harness + oracle; the GPU run checks libmraft_hip.so; both must satisfy
the reference tests' assertions (indices 1,2,3; no commit without a majority;
index2 in [2,3]; convergence after divergent partitions; at most one leader
per term; agreement and in-order apply on every committed index; the RPC
budgets of TestCount2B; committed client values after churn; snapshots every
10 entries with InstallSnapshot to lagging or restarted followers, persisted
log size under MAXLOGSIZE, no index regression after a full crash)."""
import pytest

from oracle_lib import Oracle
from sim2b import SCENARIOS, run_scenario


def _oracle(G, P, L, st):
    return Oracle(G, P, L, st)


def _gpu(G, P, L, st):
    from multiraft_amd import Engine
    e = Engine(G, P, L)
    e.load_state(st)
    return e


@pytest.mark.parametrize("name", list(SCENARIOS))
@pytest.mark.parametrize("seed", [1, 2])
def test_scenario_oracle(name, seed):
    run_scenario(_oracle, name, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_scenario_gpu(name):
    run_scenario(_gpu, name, 1)


def test_persistence_is_load_bearing(monkeypatch):
    """Without the persist_dirty flushes, a crash of every server loses
    committed entries and Persist12C must fail the reference's agreement
    check (config.go:144-163): the 2C scenarios above really restart from
    the persisted state."""
    import sim2b
    monkeypatch.setattr(sim2b.MultiSim, "_flush", lambda self: None)
    with pytest.raises(AssertionError):
        run_scenario(_oracle, "Persist12C", 1)
