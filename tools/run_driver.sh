#!/bin/bash
# Rehearse the driver's round-end GPU tiers on a fresh box: the -m gpu suite (no JIT cache),
# smoke(), then the default bench line. Each step has its own limit; the script stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-driver}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
unset MIMIC_JIT_CACHE
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider --durations=30 > gpurun_out/$TAG/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc wall=$(( $(date +%s) - t0 ))s" | tee -a gpurun_out/$TAG/gputest.log
tail -3 gpurun_out/$TAG/gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -30 gpurun_out/$TAG/smoke.log; exit 1; }
tail -3 gpurun_out/$TAG/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
