#!/bin/bash
# round 5: the sk_buff prep zeroing the rooms without reading them (MIMIC_SKB_ROOMS_ZERO=1) vs reading them
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05v
mkdir -p $D
MIMIC_SKB_ROOMS_ZERO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_bench_size.py -k "skb or cfg5" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -30 $D/test.log; exit 1; }
tail -2 $D/test.log
for k in 1 2 3; do
  for z in 0 1; do
    MIMIC_SKB_ROOMS_ZERO=$z timeout -k 10 300 python -u bench.py --config skb --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/skb_z${z}_$k.json 2> $D/skb_z${z}_$k.err || { tail -5 $D/skb_z${z}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/skb_z${z}_$k.json')); print('zero=$z', d['value'], d['ms_per_step'])"
  done
done
