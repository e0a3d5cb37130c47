#!/usr/bin/env python3
"""Print the DESIGN.md §6.1 rows from the round-end bench lines (gpurun_out/r04final/bench_*.json)."""
import glob
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r04final"
for f in sorted(glob.glob(os.path.join(D, "bench_*.json"))):
    lines = open(f).read().splitlines()
    if not lines:
        continue
    d = json.loads(lines[-1])
    r = d["roofline"]
    print(f"{os.path.basename(f):34s} {d['value']:>10.1f} Mpkts/s  {d['ms_per_step']:.4f} ms/step  launch {r['avg_launch_ms']:.4f} ms  "
          f"frac {r['frac']:.3f}  on_traffic {r.get('frac_on_traffic')}  traffic {r.get('traffic')}  "
          f"t/alg {r.get('traffic_over_algorithmic')}  valu {r.get('valu_busy')}  engine {d['config']['engine']}  "
          f"V {d['config']['vcpus_per_gpu']}  prof {r.get('profile')}")
