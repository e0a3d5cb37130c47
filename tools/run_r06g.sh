#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06g}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shared_map.py tests/test_gpu_hash.py tests/test_gpu_step.py tests/test_gpu_shard.py tests/test_gpu_skb.py tests/test_gpu_many.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -25 gpurun_out/$TAG/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/proc_probe.py > gpurun_out/$TAG/probe.json 2>&1 || { tail -20 gpurun_out/$TAG/probe.json; exit 1; }
cat gpurun_out/$TAG/probe.json
