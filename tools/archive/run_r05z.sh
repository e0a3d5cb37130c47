#!/bin/bash
# round 5: cfg 2 (V = 262 144) one-lane kernel vs owned spread at Q = 4 (256-row table), 6 alternations
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05z
mkdir -p $D
for k in 1 2 3 4 5 6; do
  for o in 0 1; do
    MIMIC_SPREAD_OWN=$o timeout -k 10 300 python -u bench.py --no-host-resident --no-cpu-baseline > $D/c_own${o}_$k.json 2> $D/c.err || { tail -5 $D/c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c_own${o}_$k.json')); print('own=$o', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['engine'], d['counters_sum'])"
  done
done
