#!/bin/bash
# sk_buff GPU tests (+ pool / step / host), then the cfg-5 bench line per knob setting and the
# kernel trace of the default one (per-kernel averages).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-skbkt}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_fastpaths.py tests/test_gpu_pool.py tests/test_gpu_step.py \
    tests/test_gpu_host.py tests/test_gpu_bench_size.py::test_cfg5_skb_chain_bench_size_exact \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gputest.log 2>&1
rc=$?
tail -2 $D/gputest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $D/gputest.log | head -30; exit $rc; }
V=${V:-131072}
for knob in ${KNOBS:-NONE=1}; do
  env $knob timeout -k 10 300 python -u bench.py --config skb --vcpus $V --no-host-resident --no-cpu-baseline > $D/bench_skb_$knob.json 2> $D/bench_skb_$knob.err || { tail -20 $D/bench_skb_$knob.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_skb_$knob.json')); print('skb $knob', d['value'], 'Mpkts/s', d['ms_per_step'], 'ms/step')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o a -- python3 bench.py --config skb --vcpus $V --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt.log 2>&1 || exit 1
cut -d, -f1-4 $(find $D/kt -name '*kernel_stats.csv' | head -1) | grep -v rocprim | cut -c1-120
