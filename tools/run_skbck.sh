#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/skbck
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_skb.py tests/test_gpu_fastpaths.py tests/test_gpu_host.py > gpurun_out/skbck/tests.log 2>&1
rc=$?; tail -3 gpurun_out/skbck/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=skbck CONFIGS="skb" VARIANTS="a:X=1" bash tools/run_variants2.sh
