#!/bin/bash
# round 5: the batch interpreter without SKBuffFromBytes inlined (16 spilled VGPRs instead of 70):
# interpreter / Step / resume / pool paths, the interpreter's cfg 2 / cfg 3 / cfg 5 launch, API rates,
# then the cfg-2 measurement variants of run_r05l.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05m
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_pool.py tests/test_gpu_skb.py tests/test_gpu_kat.py tests/test_gpu_parity.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -40 $D/test.log; exit 1; }
tail -2 $D/test.log
for c in classifier parse5 skb; do
  MIMIC_EXEC=interp timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-host-resident --no-cpu-baseline > $D/interp_$c.json 2> $D/interp_$c.err || { tail -5 $D/interp_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/interp_$c.json')); print('interp $c', d['config'].get('engine'), d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python tools/api_rates.py > $D/api_rates.json 2> $D/api_rates.err || { tail -20 $D/api_rates.err; exit 1; }
cat $D/api_rates.json
bash tools/run_r05l.sh
