#!/bin/bash
# round 5: cfg 2 with the lane value cache's row written back non-temporally (MIMIC_VC_NT) vs plain
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05r
mkdir -p $D
for k in 1 2 3; do
  for e in "X=0" "MIMIC_JIT_DEFS=MIMIC_VC_NT"; do
    n=$(echo $e | tr ' =' '_-')
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-resident > $D/b_${n}_$k.json 2> $D/b_${n}_$k.err || { tail -3 $D/b_${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/b_${n}_$k.json')); print('$e', d['value'], d['roofline']['avg_launch_ms'])"
  done
done
