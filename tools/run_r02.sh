#!/bin/bash
# round-2 GPU cycle: the GPU test suite (fresh JIT cache), then the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache_$$
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
      -p no:cacheprovider --durations=25 > gpurun_out/gputest.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/gputest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
fi
