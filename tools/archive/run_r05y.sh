#!/bin/bash
# round 5: owned spread, 256-row table (Q = 4 at V = 262 144), and P = 64..256 against the table spread
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05y
mkdir -p $D
for vn in "262144 1048576" "4096 1048576" "8192 1048576" "16384 1048576"; do
  for k in 1 2; do
  for o in 0 1; do
    set -- $vn
    export MIMIC_SPREAD_OWN=$o
    timeout -k 10 300 python -u bench.py --config classifier --vcpus $1 --packets $2 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/c_$1_$2_own${o}_$k.json 2> $D/c.err || { tail -5 $D/c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c_$1_$2_own${o}_$k.json')); print('V=$1 n=$2 own=$o', d['value'], d['ms_per_step'], d['config']['engine'])"
  done
  done
done
