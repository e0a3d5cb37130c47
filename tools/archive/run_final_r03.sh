#!/bin/bash
# Round-3 end: the driver's tiers (fresh JIT cache: -m gpu suite, smoke, default bench line), then
# PMC profiles of the classifier / skb / parse5 / flowtrack lines (their kernel-source hashes are
# what the bench lines look up; copied into profiles/ so the lines below carry them), then one
# bench line per config.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r03final bash tools/run_driver.sh || exit 1
TAG=r03 bash tools/run_prof_r03.sh || exit 1
cp gpurun_out/prof_r03/r03_pmc_*.json profiles/
NOTEST=1 TAG=r03final CONFIGS="classifier parse5 flowtrack flowtrack_insert skb pass8" bash tools/run_r03_full.sh || exit 1
timeout -k 10 300 python -u bench.py --config classifier --sched chunked --no-host-resident --no-cpu-baseline > gpurun_out/r03final/bench_classifier_chunked.json 2> gpurun_out/r03final/bench_classifier_chunked.err || exit 1
timeout -k 10 120 python -u bench.py --gpus 2 > gpurun_out/r03final/gpus2.out 2>&1; echo "bench --gpus 2 on one GPU: rc=$?" | tee -a gpurun_out/r03final/gpus2.out
