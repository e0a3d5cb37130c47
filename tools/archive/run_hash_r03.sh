#!/bin/bash
# hash-map GPU tests, then the cfg-4 bench lines (lookup-hit and inserting batches) and the
# kernel trace of the inserting line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-hash}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_shard.py tests/test_gpu_bench_size.py::test_cfg4_flowtrack_bench_size_per_key_exact \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/gputest.log 2>&1
rc=$?
tail -4 $D/gputest.log
[ $rc -eq 0 ] || exit $rc
for c in flowtrack flowtrack_insert; do
  timeout -k 10 300 python -u bench.py --config $c --no-host-resident --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail -20 $D/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$c.json')); r=d['roofline']; print('$c', d['value'], 'Mpkts/s', r['avg_launch_ms'], 'ms', r['frac'], d['hash_keys'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_ins -o a -- python3 bench.py --config flowtrack_insert --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt_ins.log 2>&1 || exit 1
cat $(find $D/kt_ins -name '*kernel_stats.csv' | head -1)
