#!/usr/bin/env python3
"""Print key fields of the last JSON line of a bench output file (RCCL may print banners)."""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(path, "NO JSON")
        continue
    d = json.loads(lines[-1])
    c = d.get("config", {})
    print(path, d["value"], d["ms_per_step"], c.get("per_gpu_batch"), c.get("hip_graph"), c.get("overlap"),
          d.get("comm_backend"), d.get("collectives_per_step"), d.get("weak_scaling", ""))
