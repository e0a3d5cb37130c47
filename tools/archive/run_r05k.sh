#!/bin/bash
# round 5: process / pool paths after the block cache, then the API rates
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05k
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_pool.py tests/test_gpu_ctx.py tests/test_gpu_skb.py tests/test_gpu_kat.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -40 $D/test.log; exit 1; }
tail -2 $D/test.log
timeout -k 10 600 python tools/api_rates.py > $D/api_rates.json 2> $D/api_rates.err || { tail -20 $D/api_rates.err; exit 1; }
cat $D/api_rates.json
