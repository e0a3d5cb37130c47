#!/bin/bash
# measurement only: the cfg-5 chain kernel with and without slow paths compiled in, at two V
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
for v in 65536 262144; do
  for nc in 0 1; do
    echo "NOCOLD=$nc skb V=$v" >> gpurun_out/nocold.log
    MIMIC_JIT_NOCOLD=$nc timeout -k 10 300 python bench.py --config skb --vcpus $v --steps 5 --warmup 2 --no-cpu-baseline --no-host-resident >> gpurun_out/nocold.log 2>>gpurun_out/nocold.err || exit $?
  done
done
