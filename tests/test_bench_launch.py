"""bench.py's multi-GPU launch plumbing on CPU (no GPU call: --dry-run): with
`--gpus N` and no torch.distributed launcher it starts the N rank processes
itself, defaults to BASELINE config #4 (262,144 groups split over the ranks,
strong scaling), every rank builds its shard of the one global seeded workload
and the control plane runs; rank 0 prints the only stdout line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks_config4_default():
    out = _run("--gpus", "2", "--dry-run", "--dist-backend", "gloo", "--log", "64")
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["dry_run"]
    c = out["config"]
    assert c["global_groups"] == 262144 and c["groups_per_gpu"] == 131072
    assert c["workload"].startswith("config #4: 262,144 groups")
    # the N = 1 point of the strong-scaling series is named on every N > 1 line
    assert "strong_scaling_reference_ms" in out and "what" in out["strong_scaling_reference"]


def test_gpus1_defaults_to_config3():
    out = _run("--dry-run", "--log", "64")
    assert out["n_gpus"] == 1 and out["scaling"] == "weak"
    assert out["config"]["groups_per_gpu"] == 65536
    assert out["config"]["workload"].startswith("config #3")
    assert "strong_scaling_reference_ms" not in out


def test_gpus4_weak_when_groups_given():
    out = _run("--gpus", "4", "--dry-run", "--dist-backend", "gloo", "--groups", "512", "--log", "32")
    assert out["n_gpus"] == 4 and out["scaling"] == "weak"
    assert out["config"]["global_groups"] == 2048


def test_gpus2_rank_stream_plan_two_shards_rccl_fanin():
    """The N > 1 default per rank (verdict r3 #5): 2 tick shards on engine-owned
    queues masked off the fan-in's 8 CUs, the RCCL fan-in on its own 8-CU queue
    waiting for every shard's end marker, no masked tick stream on the engine
    stream, and no more dedicated hardware queues than the box's 4 per process.
    The plan is computed by every rank (gloo, world size 2) and gathered."""
    out = _run("--gpus", "2", "--dry-run", "--log", "64")  # default --dist-backend nccl: the RCCL plan
    c = out["config"]
    assert c["shards_per_gpu"] == 2
    plans = c["stream_plan_by_rank"]
    assert len(plans) == 2 and plans[0] == plans[1]
    p = plans[0]
    assert p["tick_queues"] == 2 and p["tick_queue_mask"] == "every CU but the fan-in's 8"
    assert p["fanin_queue"] == 1 and p["fanin_on"] == "fan-in queue (8 CUs)"
    assert p["fanin_waits_for"] == "the end marker of every shard's tick"
    assert p["dedicated_queues"] == 3 <= 4
    ref = out["strong_scaling_reference"]
    assert ref.get("shards_per_gpu", 2) == 2 or "2 tick shard" in ref["what"]
