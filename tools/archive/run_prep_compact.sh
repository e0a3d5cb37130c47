#!/bin/bash
# round 5: the prep kernel's walk compaction (PREP_COMPACT): the kernel alone before / after, the
# sk_buff GPU tests, then cfg-5 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/prepc; mkdir -p $D
export TMPDIR=/tmp
PREP_SOS="base compact" bash tools/run_prep_variants.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_bench_size.py tests/test_gpu_pool.py \
    tests/test_gpu_step.py tests/test_gpu_ctx.py tests/test_gpu_fastpaths.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/test.log 2>&1 || { tail -30 $D/test.log; exit 1; }
tail -2 $D/test.log
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --config skb --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/skb_$k.json 2> $D/skb_$k.err || { tail -5 $D/skb_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/skb_$k.json')); print('skb', d['value'], d['ms_per_step'])"
done
