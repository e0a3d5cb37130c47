#!/bin/bash
# lane value cache: parity (vc, fast-path, workload, shard modules), then cfg 2 per-launch times
# with the cache on and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-vc}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_vc.py tests/test_gpu_fastpaths.py tests/test_gpu_parity.py tests/test_gpu_shard.py > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-classifier}; do
  for x in 1 0 1 0; do
    MIMIC_JIT_VC=$x timeout -k 10 200 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-resident \
        > gpurun_out/$TAG/b_${cfg}_$x.json 2>> gpurun_out/$TAG/bench.err || exit $?
    echo "$cfg vc=$x $(python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/b_${cfg}_$x.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
  done
done
