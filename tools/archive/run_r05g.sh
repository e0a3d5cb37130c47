#!/bin/bash
# round 5: cfg-5 chain variants at a forced 2-wave budget (MIMIC_JIT_WAVES=2: no AGPR overflow)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r05g
mkdir -p $D
B="python3 bench.py --config skb --no-cpu-baseline --no-host-resident --steps 30"
for e in "MIMIC_JIT_WAVES=0" "MIMIC_JIT_WAVES=2" "MIMIC_JIT_WAVES=2 MIMIC_JIT_SKBTOUCH=1" "MIMIC_JIT_WAVES=2 MIMIC_JIT_SKBTOUCH=2" "MIMIC_JIT_WAVES=2 MIMIC_JIT_SKBFAST=1"; do
  n=$(echo $e | tr ' =' '_-')
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_$n -o a -- $B > $D/kt_$n.log 2>&1 || { tail -5 $D/kt_$n.log; exit 1; }
  f=$(find $D/kt_$n -name '*kernel_stats.csv' | head -1); cp $f $D/kernel_stats_$n.csv
  python3 - <<PY
import csv, json
r = {x['Name']: float(x['AverageNs']) / 1000 for x in csv.DictReader(open('$D/kernel_stats_$n.csv'))}
d = [json.loads(l) for l in open('$D/kt_$n.log') if l.startswith('{')][0]
print('$e', d['ms_per_step'], {k[:22]: round(v, 1) for k, v in r.items() if k.startswith('mimic')})
PY
done
