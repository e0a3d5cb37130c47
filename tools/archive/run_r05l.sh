#!/bin/bash
# round 5: cfg-2 launch time under measurement variants (results stores off, lane prefetch, no cold paths)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05l
mkdir -p $D
for e in "MIMIC_JIT_X=0" "MIMIC_JIT_DEFS=MIMIC_MEAS_NORES" "MIMIC_JIT_LPF=1" "MIMIC_JIT_LPF=1 MIMIC_JIT_DEFS=MIMIC_MEAS_NORES" "MIMIC_JIT_NOCOLD=1" "MIMIC_JIT_LPF=1 MIMIC_JIT_NOCOLD=1 MIMIC_JIT_DEFS=MIMIC_MEAS_NORES"; do
  n=$(echo $e | tr ' =' '_-')
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-resident > $D/b_$n.json 2> $D/b_$n.err || { tail -3 $D/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/b_$n.json')); print('$e', d['value'], d['roofline']['avg_launch_ms'])"
done
