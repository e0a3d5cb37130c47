#!/bin/bash
# sk_buff GPU tests (incl. the cfg-5 bench-size test), then the cfg-5 and cfg-2 bench lines and
# the cfg-5 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-skb}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_bench_size.py::test_cfg5_skb_chain_bench_size_exact ${EXTRA_TESTS:-} \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gputest.log 2>&1
rc=$?
tail -4 $D/gputest.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-skb classifier}; do
  timeout -k 10 300 python -u bench.py --config $c --no-host-resident --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail -20 $D/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$c.json')); r=d['roofline']; print('$c', d['value'], 'Mpkts/s', r['avg_launch_ms'], 'ms', r['frac'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o a -- python3 bench.py --config skb --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt.log 2>&1 || exit 1
grep -E "mimic_|Name" $(find $D/kt -name '*kernel_stats.csv' | head -1) | cut -c1-150
