#!/bin/bash
# bench lines (default + configs) and the cfg-2 V sweep at HEAD, reading the committed profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/bench_configs.jsonl gpurun_out/vsweep.jsonl
bash tools/run_r02.sh bench || exit $?
for v in 256 4096 65536 131072 262144 1048576; do
  timeout -k 10 200 python bench.py --config classifier --vcpus $v --steps 20 --warmup 3 --no-cpu-baseline --no-host-resident >> gpurun_out/vsweep.jsonl 2>> gpurun_out/vsweep.err || exit $?
done
