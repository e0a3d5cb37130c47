#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06d}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/proc_probe.py > gpurun_out/$TAG/probe.json 2>&1 || { tail -20 gpurun_out/$TAG/probe.json; exit 1; }
cat gpurun_out/$TAG/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt -o a -- python3 tools/proc_probe.py > gpurun_out/$TAG/kt.log 2>&1 || { tail -20 gpurun_out/$TAG/kt.log; exit 1; }
cat $(find gpurun_out/$TAG/kt -name '*kernel_stats.csv' | head -1)
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_step.py tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -5 gpurun_out/$TAG/gputest.log
exit $rc
