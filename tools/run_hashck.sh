#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/hashck
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_hash.py tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_pool.py > gpurun_out/hashck/tests.log 2>&1
rc=$?; tail -3 gpurun_out/hashck/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=hashck CONFIGS="flowtrack skb" VARIANTS="a:X=1" bash tools/run_variants2.sh
