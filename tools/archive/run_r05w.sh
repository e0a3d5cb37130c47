#!/bin/bash
# round 5: owned spread with Q packets per thread (MIMIC_SPREAD_OWN_Q) vs the one-lane kernel, classifier
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05w
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_spread_own.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test_q1.log 2>&1 || { tail -30 $D/test_q1.log; exit 1; }
tail -1 $D/test_q1.log
for q in 2; do
  MIMIC_SPREAD_OWN=1 MIMIC_SPREAD_OWN_Q=$q timeout -k 10 600 python -u -m pytest tests/test_gpu_spread_own.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "classifier and (262144 or 1000-256000)" > $D/test_q$q.log 2>&1 || { tail -30 $D/test_q$q.log; exit 1; }
  tail -1 $D/test_q$q.log
done
for vn in "262144 1048576" "65536 1048576" "131072 524288"; do
  set -- $vn
  for k in 1 2; do
    for c in "0 1" "1 1" "1 2"; do
      set -- $vn $c
      MIMIC_SPREAD_OWN=$3 MIMIC_SPREAD_OWN_Q=$4 timeout -k 10 300 python -u bench.py --config classifier --vcpus $1 --packets $2 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/c_$1_own$3_q$4_$k.json 2> $D/c.err || { tail -5 $D/c.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/c_$1_own$3_q$4_$k.json')); print('V=$1 own=$3 q=$4', d['value'], d['ms_per_step'], d['config']['engine'])"
    done
  done
done
