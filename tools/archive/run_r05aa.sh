#!/bin/bash
# round 5: cfg 3 (parse5, V = 262 144, P = 64, 2 KiB rows) one-lane vs owned spread (auto Q)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05aa
mkdir -p $D
for k in 1 2; do
  for o in 0 1; do
    MIMIC_SPREAD_OWN=$o timeout -k 10 300 python -u bench.py --config parse5 --steps 10 --warmup 2 --no-host-resident --no-cpu-baseline > $D/p_own${o}_$k.json 2> $D/p.err || { tail -5 $D/p.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/p_own${o}_$k.json')); print('parse5 own=$o', d['value'], d['ms_per_step'], d['config']['engine'])"
  done
done
for k in 1 2; do
  for o in 0 1; do
    MIMIC_SPREAD_OWN=$o timeout -k 10 300 python -u bench.py --config pass8 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/p8_own${o}_$k.json 2> $D/p.err || { tail -5 $D/p.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/p8_own${o}_$k.json')); print('pass8 own=$o', d['value'], d['ms_per_step'], d['config']['engine'])"
  done
done
