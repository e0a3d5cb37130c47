#!/bin/bash
# round-end measurement at HEAD: rocprofv3 passes per config (into profiles/ on the box, so the
# bench lines that follow read HEAD-matched traffic), default bench line + config lines, V sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r02
PROF_CONFIGS="${PROF_CONFIGS:-classifier parse5 flowtrack skb}" bash tools/run_r02.sh prof || exit $?
cp gpurun_out/prof_r02/r02_pmc_*.json gpurun_out/prof_r02/r02_kernel_stats_*.csv profiles/ || exit 1
rm -f gpurun_out/bench_configs.jsonl gpurun_out/vsweep.jsonl
bash tools/run_r02.sh bench || exit $?
for v in 256 4096 65536 131072 262144 1048576; do
  timeout -k 10 200 python bench.py --config classifier --vcpus $v --steps 20 --warmup 3 --no-cpu-baseline --no-host-resident >> gpurun_out/vsweep.jsonl 2>> gpurun_out/vsweep.err || exit $?
done
