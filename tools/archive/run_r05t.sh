#!/bin/bash
# round 5: owned spread vs the one-lane kernel where the one-lane kernel underfills the chip (V < 262 144)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05t
mkdir -p $D
for vn in "65536 262144" "131072 524288" "32768 131072" "65536 131072" "16384 65536" "131072 262144"; do
  set -- $vn
  for o in 0 1; do
    MIMIC_SPREAD_OWN=$o timeout -k 10 300 python -u bench.py --config classifier --vcpus $1 --packets $2 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/c_$1_$2_own$o.json 2> $D/c_$1_$2_own$o.err || { tail -5 $D/c_$1_$2_own$o.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c_$1_$2_own$o.json')); print('V=$1 n=$2 own=$o', d['value'], d['ms_per_step'])"
  done
done
