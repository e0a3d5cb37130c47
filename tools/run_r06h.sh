#!/bin/bash
# proc-JIT tests + shared-table diagnostics + Process.Run probe
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06h}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
if [ "${SHARE:-0}" = 1 ]; then
  timeout -k 10 200 python -u tools/share_diag.py > gpurun_out/$TAG/share_diag.log 2>&1 || { tail -20 gpurun_out/$TAG/share_diag.log; exit 1; }
fi
timeout -k 10 700 python -u -m pytest tests/test_gpu_proc_jit.py tests/test_gpu_shared_map.py tests/test_gpu_step.py tests/test_gpu_skb.py tests/test_gpu_many.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gputest.log 2>&1; rc=$?
tail -25 gpurun_out/$TAG/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/proc_probe.py > gpurun_out/$TAG/probe.json 2>&1 || { tail -20 gpurun_out/$TAG/probe.json; exit 1; }
cat gpurun_out/$TAG/probe.json
