#!/bin/bash
# Round-4 first pass: the driver's tiers at HEAD (fresh JIT cache), then the cfg-4 bench line
# (one batch sharded) and the cfg-4 --rccl rehearsal at world size 1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r04a bash tools/run_driver.sh || exit 1
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u bench.py --config flowtrack --no-cpu-baseline --no-host-resident > gpurun_out/r04a/bench_flowtrack.json 2> gpurun_out/r04a/bench_flowtrack.err || exit 1
timeout -k 10 300 python -u bench.py --config flowtrack --rccl --no-cpu-baseline --no-host-resident > gpurun_out/r04a/bench_flowtrack_rccl.json 2> gpurun_out/r04a/bench_flowtrack_rccl.err || exit 1
cat gpurun_out/r04a/bench_flowtrack*.json
