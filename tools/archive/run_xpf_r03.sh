#!/bin/bash
# next-packet header window prefetch (MIMIC_JIT_XPF=1) on cfg 3 / cfg 4 at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/xpf; mkdir -p $D
for c in parse5 flowtrack; do
  for k in X=1 MIMIC_JIT_XPF=1; do
    env $k timeout -k 10 300 python -u bench.py --config $c --no-host-resident --no-cpu-baseline > $D/${c}_$k.json 2> $D/${c}_$k.err || { tail -5 $D/${c}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/${c}_$k.json')); print('$c $k', d['value'], d['roofline']['avg_launch_ms'])"
  done
done
