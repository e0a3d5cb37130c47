#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06f}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_bench_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -5 gpurun_out/$TAG/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config skb --steps 30 --no-cpu-baseline --no-host-resident > gpurun_out/$TAG/bench_skb.json 2> gpurun_out/$TAG/bench_skb.err || { tail -20 gpurun_out/$TAG/bench_skb.err; exit 1; }
cat gpurun_out/$TAG/bench_skb.json | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt_skb -o a -- python3 bench.py --config skb --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > gpurun_out/$TAG/kt_skb.log 2>&1 || { tail -20 gpurun_out/$TAG/kt_skb.log; exit 1; }
cat $(find gpurun_out/$TAG/kt_skb -name '*kernel_stats.csv' | head -1)
timeout -k 10 200 python -u tools/proc_probe.py > gpurun_out/$TAG/probe.json 2>&1 || { tail -20 gpurun_out/$TAG/probe.json; exit 1; }
cat gpurun_out/$TAG/probe.json
