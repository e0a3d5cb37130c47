#!/bin/bash
# V sweep of the cfg-2 headline (vCPUs per GPU) and rocprofv3 summaries of the other configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
for v in 256 4096 65536 262144 1048576; do
  timeout -k 10 200 python bench.py --config classifier --vcpus $v --steps 20 --warmup 3 --no-cpu-baseline --no-host-resident >> gpurun_out/vsweep.jsonl 2>> gpurun_out/vsweep.err || exit $?
done
for c in ${PROF_CONFIGS:-parse5 flowtrack skb}; do
  CFG=$c TAG=r02 bash tools/profile.sh || exit $?
done
