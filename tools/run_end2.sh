#!/bin/bash
# end-of-round: bench config lines, then the driver rehearsal (suite, smoke, default bench line)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/bench_configs.jsonl
BENCH_CONFIGS="pass8 parse5 flowtrack skb" bash tools/run_r02.sh bench || exit $?
TAG=end2 bash tools/run_driver.sh
