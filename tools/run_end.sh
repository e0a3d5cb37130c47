#!/bin/bash
# end-of-round: pass8 profile into profiles/, bench config lines, then the driver rehearsal
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PROF_CONFIGS="${PROF_CONFIGS:-pass8}" bash tools/run_r02.sh prof || exit $?
for c in ${PROF_CONFIGS:-pass8}; do cp gpurun_out/prof_r02/r02_pmc_$c.json gpurun_out/prof_r02/r02_kernel_stats_$c.csv profiles/ || exit 1; done
rm -f gpurun_out/bench_configs.jsonl
BENCH_CONFIGS="pass8 parse5 flowtrack skb" bash tools/run_r02.sh bench || exit $?
TAG=end bash tools/run_driver.sh
