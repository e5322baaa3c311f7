"""One-screen summary of a bench.py result line (the headline, its roofline
and, when present, the secondary lines)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, c = d["roofline"], d["config"]
print(f"value {d['value']:.4g} {d['unit']}  ms/step {d['ms_per_step']:.4f}  device ms {r['kernel_ms_mean']:.4f}  "
      f"frac {r['frac']:.3f}  shards {c.get('shards_per_gpu')}  step-kernel {c['step_minus_kernel_ms']:.4f}")
print("launch_ms_mean", r.get("launch_ms_mean"), "traffic", r.get("traffic"), r.get("traffic_source"))
pp = r.get("placement_probe") or {}
if pp.get("populations"):
    print("populations", json.dumps(pp["populations"]))
s = d.get("secondary") or {}
if "message_path_config3" in s:
    m = s["message_path_config3"]
    print("message path ms", m["ms_per_call"], "handle frac", round(m["roofline"]["frac"], 3),
          "fold frac", round(m["fold_roofline"]["frac"], 3))
    print("message path pipelines: S=2", round(m["shards_2"]["vs_headline"], 3),
          "S=3", round(m["shards_3"]["vs_headline"], 3) if "shards_3" in m else None, "x the headline")
if "election_storm_config5" in s:
    e = s["election_storm_config5"]
    print("config5 ms", round(e["kernel_ms_mean"], 4), {k: v for k, v in e.items() if k == "roofline"})
if "config4_one_gpu" in s:
    for k, v in s["config4_one_gpu"]["by_shards"].items():
        print(f"config4 S={k}: ms/step {v['ms_per_step']:.4f} device {v['roofline']['kernel_ms_mean']:.4f} "
              f"frac {v['roofline']['frac']:.3f}")
cb = d.get("cpu_baseline")
if cb:
    print("cpu baseline", f"{cb['value']:.4g}", cb["cores"])
if "steady_state_config3" in s:
    e = s["steady_state_config3"]
    li = e.get("light", {})
    print("steady state tick ms: full", round(e["tick_ms_steady"], 4), "light", round(li.get("tick_ms_steady", 0), 4),
          "speedup", round(li.get("speedup_tick_steady", 0), 2), "same", li.get("state_equals_full"),
          "fallbacks", li.get("fallback_groups_steps", [])[:6], "...", li.get("fallback_groups_steps", [])[-2:])
    fu = e.get("fused")
    if fu:
        print("steady state per step: start_and_tick (light)", round(fu["device_ms_per_step_steady"], 4),
              "vs start+tick full", round(fu["vs_full_start_then_tick"], 2), "x, light",
              round(fu["vs_light_start_then_tick"], 2), "x; same", fu["state_equals_full"])
