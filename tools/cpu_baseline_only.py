"""Runs bench.py's cpu_baseline leg alone (no GPU work) and prints its JSON."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = sys.argv[:1]
import bench  # noqa: E402

t = time.time()
r = bench.cpu_baseline(65536, 5, 4096, 0xC0FFEE + 3, float(os.environ.get("BUDGET", 12)), 0)
r["wall_s"] = time.time() - t
print(json.dumps(r))
