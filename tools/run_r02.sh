#!/bin/bash
# round-2 GPU cycle: STAGE=test (GPU suite, fresh JIT cache) | bench (default line + configs) |
# prof (rocprofv3 passes per config) | all
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
      -p no:cacheprovider --durations=25 ${PYTEST_ARGS:-} > gpurun_out/gputest.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/gputest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
  for c in ${BENCH_CONFIGS:-pass8 parse5 flowtrack skb}; do
    timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-host-resident --cpu-seconds 5 >> gpurun_out/bench_configs.jsonl 2>> gpurun_out/bench_configs.err || exit $?
  done
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  for c in ${PROF_CONFIGS:-classifier}; do
    CFG=$c TAG=r02 bash tools/profile.sh || exit $?
  done
fi
