#!/bin/bash
# cfg 5 (sk_buff tail-call chain) under JIT codegen variants: VARIANTS="A=1,B=0 ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
for v in ${VARIANTS:-MIMIC_EXEC=jit}; do
  echo "VARIANT $v skb" >> gpurun_out/variants.log
  env ${v//,/ } timeout -k 10 300 python bench.py --config skb --steps 5 --warmup 2 --no-cpu-baseline --no-host-resident >> gpurun_out/variants.log 2>>gpurun_out/variants.err || exit $?
done
