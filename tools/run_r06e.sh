#!/bin/bash
# multi-batch launches + single-process path changes: focused GPU tests, probe, bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06e}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_many.py tests/test_gpu_step.py tests/test_gpu_pool.py tests/test_gpu_spread_own.py tests/test_gpu_skb.py tests/test_gpu_ctx.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -5 gpurun_out/$TAG/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/proc_probe.py > gpurun_out/$TAG/probe.json 2>&1 || { tail -20 gpurun_out/$TAG/probe.json; exit 1; }
cat gpurun_out/$TAG/probe.json
for m in 1 5; do
  timeout -k 10 300 python -u bench.py --many $m --no-cpu-baseline --no-host-resident > gpurun_out/$TAG/bench_many$m.json 2> gpurun_out/$TAG/bench_many$m.err || { tail -20 gpurun_out/$TAG/bench_many$m.err; exit 1; }
  cat gpurun_out/$TAG/bench_many$m.json
done
