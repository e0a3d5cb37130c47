#!/bin/bash
# JIT codegen variants x configs (short bench runs; one JSON line each, prefixed by the variant)
#   VARIANTS="A=1,B=0 A=0,B=0" CONFIGS="classifier pass8" bash tools/run_variants.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
O=gpurun_out/variants.log
VARIANTS=${VARIANTS:-"MIMIC_JIT_KQ=1,MIMIC_JIT_OPAQUE_LANE=1 MIMIC_JIT_KQ=0,MIMIC_JIT_OPAQUE_LANE=1 MIMIC_JIT_KQ=1,MIMIC_JIT_OPAQUE_LANE=0 MIMIC_JIT_KQ=0,MIMIC_JIT_OPAQUE_LANE=0"}
for rep in 1 2; do
for v in $VARIANTS; do
  for c in ${CONFIGS:-classifier pass8 parse5}; do
    echo "VARIANT $v $c" >> $O
    env ${v//,/ } timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-resident >> $O 2>/dev/null || exit $?
  done
done
done
