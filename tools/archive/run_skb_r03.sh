#!/bin/bash
# sk_buff path: its GPU tests (+ the deferral-heavy KATs), the cfg-5 bench at V = 64K / 128K / 256K,
# then the PMC passes of the cfg-5 line (tools/profile.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-skb}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_step.py tests/test_gpu_kat.py tests/test_gpu_bench_size.py::test_cfg5_skb_chain_bench_size_exact \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gputest.log 2>&1
rc=$?
tail -3 $D/gputest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $D/gputest.log | head -30; exit $rc; }
for v in ${VS:-65536 131072 262144}; do
  timeout -k 10 300 python -u bench.py --config skb --vcpus $v --no-host-resident --no-cpu-baseline > $D/bench_skb_$v.json 2> $D/bench_skb_$v.err || { tail -20 $D/bench_skb_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_skb_$v.json')); r=d['roofline']; print('skb V=$v', d['value'], 'Mpkts/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], 'ms', r['frac'])"
done
[ -n "$NOPROF" ] && exit 0
CFG=skb TAG=$TAG EXTRA="--vcpus ${PV:-131072}" timeout -k 10 900 bash tools/profile.sh || exit 1
cat gpurun_out/prof_$TAG/${TAG}_kernel_stats_skb.csv | cut -c1-200
cat gpurun_out/prof_$TAG/summary_skb.log | tail -20
