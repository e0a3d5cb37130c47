#!/bin/bash
# Deferred slow paths: the full -m gpu suite, then the cfg-5 bench line at V = 64K / 128K / 256K
# and a kernel trace of the default cfg-5 line.  Each step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-defer}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
unset MIMIC_JIT_CACHE
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider --durations=10 > $D/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc wall=$(( $(date +%s) - t0 ))s" | tee -a $D/gputest.log
tail -4 $D/gputest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $D/gputest.log | head -30; exit $rc; }
for v in 65536 131072 262144; do
  timeout -k 10 300 python -u bench.py --config skb --vcpus $v --no-host-resident --no-cpu-baseline > $D/bench_skb_$v.json 2> $D/bench_skb_$v.err || { tail -20 $D/bench_skb_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_skb_$v.json')); r=d['roofline']; print('skb V=$v', d['value'], 'Mpkts/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], 'ms', r['frac'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_skb -o a -- python3 bench.py --config skb --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt_skb.log 2>&1 || exit 1
cat $(find $D/kt_skb -name '*kernel_stats.csv' | head -1)
