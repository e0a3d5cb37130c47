#!/bin/bash
# measurement only: the hot kernels with and without slow paths compiled in (MIMIC_JIT_NOCOLD=1),
# at several V -- the ceiling a slow-path-free hot kernel would reach
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
O=gpurun_out/nocold.log
for c in classifier parse5; do
  for v in 262144 524288 1048576; do
    for nc in 0 1; do
      echo "NOCOLD=$nc $c V=$v" >> $O
      MIMIC_JIT_NOCOLD=$nc timeout -k 10 200 python bench.py --config $c --vcpus $v --steps 20 --warmup 3 --no-cpu-baseline --no-host-resident >> $O 2>/dev/null || exit $?
    done
  done
done
