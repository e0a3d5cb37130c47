#!/bin/bash
# Round 4: spread flush policy (per-block tables + reduce only when V x counters <= packets per
# block): the classifier at V = 64 / 256 / 512 / 1024, spread tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_spread.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config classifier"
for v in 64 256 512 1024; do $B --vcpus $v > $O/cls_v$v.json 2> $O/cls_v$v.err || exit 1; done
for f in $O/cls_v*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['engine'], d['counters_sum'])"; done
