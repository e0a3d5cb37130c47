#!/bin/bash
# the batch interpreter at its 4-wave budget (spills) vs the compiler's own (3 waves), cfg 2 and cfg 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/interp; mkdir -p $D
for c in classifier parse5; do
  for w in 4 3; do
    MIMIC_EXEC=interp MIMIC_INTERP_WAVES=$w timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-host-resident --no-cpu-baseline > $D/${c}_$w.json 2> $D/${c}_$w.err || { tail -5 $D/${c}_$w.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/${c}_$w.json')); print('$c waves=$w', d['config']['engine'], d['value'], d['roofline']['avg_launch_ms'])"
  done
done
