#!/bin/bash
# round 5: owned spread (MIMIC_SPREAD_OWN=1) vs the default policy (unset) and never (0), classifier shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05u
mkdir -p $D
for vn in "196608 786432" "65536 1048576" "16384 1048576" "4096 1048576" "262144 1048576"; do
  set -- $vn
  for o in 0 1 d; do
    if [ $o = d ]; then unset MIMIC_SPREAD_OWN; else export MIMIC_SPREAD_OWN=$o; fi
    timeout -k 10 300 python -u bench.py --config classifier --vcpus $1 --packets $2 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/c_$1_$2_own$o.json 2> $D/c_$1_$2_own$o.err || { tail -5 $D/c_$1_$2_own$o.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c_$1_$2_own$o.json')); print('V=$1 n=$2 own=$o', d['value'], d['ms_per_step'], d['config'].get('engine'))"
  done
done
