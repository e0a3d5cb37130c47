#!/bin/bash
# round 5: slow-path branches marked [[unlikely]] (MIMIC_JIT_HINT=1) vs not (default), every bench config
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05n
mkdir -p $D
for c in classifier parse5 flowtrack flowtrack_insert skb; do
  for h in 0 1 0 1; do
    MIMIC_JIT_HINT=$h timeout -k 10 300 python -u bench.py --config $c --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/${c}_$h.json 2> $D/${c}_$h.err || { tail -5 $D/${c}_$h.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/${c}_$h.json')); print('$c hint=$h', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
  done
done
