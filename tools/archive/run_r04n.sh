#!/bin/bash
# Round 4: the two-map insert test, then the default bench line (100 timed steps) and the cfg-2
# line at 20 steps for comparison.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-host-resident > $O/bench20.json 2> $O/bench20.err || exit 1
for f in $O/bench.json $O/bench20.json; do python3 -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['frac_on_traffic'])"; done
