#!/bin/bash
# Full GPU check at HEAD: the -m gpu suite (fresh JIT cache), smoke, then one bench line per
# config (rotating batches).  Each step has its own limit; the script stops at the first failure.
#   CONFIGS="parse5 skb" EXTRA_skb="--vcpus 131072" TAG=x bash tools/run_r03_full.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-full}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
unset MIMIC_JIT_CACHE
t0=$(date +%s)
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider --durations=15 > $D/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc wall=$(( $(date +%s) - t0 ))s" | tee -a $D/gputest.log
tail -4 $D/gputest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $D/gputest.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
fi
for c in ${CONFIGS:-classifier parse5 flowtrack flowtrack_insert skb pass8}; do
  ev="EXTRA_$c"
  timeout -k 10 400 python -u bench.py --config $c --no-host-resident --no-cpu-baseline ${!ev} > $D/bench_$c.json 2> $D/bench_$c.err || { tail -20 $D/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$c.json')); r=d['roofline']; print('$c', d['value'], 'Mpkts/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], 'ms', r['frac'], d['config']['batches_rotated'])"
done
