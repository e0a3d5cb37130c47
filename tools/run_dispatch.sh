#!/bin/bash
# single tail-call dispatch block: parity of the tail-call modules, then cfg 5 variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-dispatch}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_skb.py tests/test_gpu_fastpaths.py tests/test_gpu_parity.py tests/test_gpu_kat.py > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG CONFIGS="skb" VARIANTS="disp:MIMIC_JIT_DISPATCH=1;jt:MIMIC_JIT_DISPATCH=0" bash tools/run_variants2.sh
