#!/bin/bash
# round 5: lane prefetch (MIMIC_JIT_LPF) -- xdp GPU tests, then cfg 2 / cfg 3 / cfg 2 chunked bench lines with it on and off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r05i
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastpaths.py tests/test_gpu_vc.py tests/test_gpu_host.py \
  tests/test_gpu_shard.py tests/test_gpu_spread.py tests/test_gpu_pool.py tests/test_gpu_hash.py tests/test_gpu_bench_size.py -k "not cfg5" \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -40 $D/test.log; exit 1; }
tail -2 $D/test.log
for c in "classifier" "classifier --sched chunked" "parse5 --steps 20" "flowtrack_insert --steps 30"; do
  for v in 1 0; do
    n=$(echo "$c lpf$v" | tr ' -' '__')
    MIMIC_JIT_LPF=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-host-resident > $D/bench_$n.json 2> $D/bench_$n.err || { tail -5 $D/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['status_ok_frac'], d['counters_sum'][:4] if d['counters_sum'] else None)"
  done
done
MIMIC_JIT_MEMTIME=1 timeout -k 10 300 python tools/memtime.py > $D/memtime_lpf1.json 2>/dev/null && cat $D/memtime_lpf1.json
