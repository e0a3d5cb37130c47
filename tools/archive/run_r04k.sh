#!/bin/bash
# Round 4: the sk_buff prep kernel as a chunk loop with the next chunk's descriptors prefetched
# (127 VGPRs, 4 waves) -- sk_buff GPU tests, then the cfg-5 line under a kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_skb.py tests/test_gpu_step.py tests/test_gpu_pool.py tests/test_gpu_bench_size.py -k "not cfg3 and not cfg4" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="python3 -u bench.py --no-cpu-baseline --no-host-resident"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_skb -o a -- $B --config skb --steps 10 --warmup 2 > $O/skb.json 2> $O/skb.err || exit 1
grep -h "mimic_skb_prep_kernel\|mimic_jit_kernel" $(find $O/kt_skb -name '*kernel_stats.csv')
timeout -k 10 300 $B --config skb > $O/skb2.json 2> $O/skb2.err || exit 1
for f in $O/skb.json $O/skb2.json; do python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
