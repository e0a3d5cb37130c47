#!/bin/bash
# LDS stack window: parity of the stack-heavy modules, then cfg 4 / cfg 5 per-launch variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-ldsstk}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_hash.py tests/test_gpu_skb.py tests/test_gpu_fastpaths.py tests/test_gpu_parity.py tests/test_gpu_kat.py > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG CONFIGS="flowtrack skb" VARIANTS="lds:MIMIC_JIT_LDSSTK=16;nolds:MIMIC_JIT_LDSSTK=0;lds3:MIMIC_JIT_LDSSTK=16 MIMIC_JIT_WAVES=3" bash tools/run_variants2.sh
