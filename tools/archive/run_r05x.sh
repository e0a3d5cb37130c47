#!/bin/bash
# round 5: owned spread with Q packets per thread chosen per launch (KParams::own_q): tests, then benches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05x
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_spread_own.py tests/test_gpu_spread.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -30 $D/test.log; exit 1; }
tail -1 $D/test.log
for vn in "262144 1048576" "131072 524288" "65536 1048576" "65536 262144" "16384 1048576"; do
  for o in 0 1 d; do
    set -- $vn
    if [ $o = d ]; then unset MIMIC_SPREAD_OWN; else export MIMIC_SPREAD_OWN=$o; fi
    timeout -k 10 300 python -u bench.py --config classifier --vcpus $1 --packets $2 --steps 50 --warmup 3 --no-host-resident --no-cpu-baseline > $D/c_$1_$2_own$o.json 2> $D/c.err || { tail -5 $D/c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c_$1_$2_own$o.json')); print('V=$1 n=$2 own=$o', d['value'], d['ms_per_step'], d['config']['engine'])"
  done
done
