#!/bin/bash
# Round 4 (session 2): the -m gpu suite at HEAD (Run(ctx) added), then cfg 2 with and without the
# per-packet context check compiled in (MIMIC_JIT_DEFS=MIMIC_MEAS_NOCTX), alternating, 3 runs each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r04t
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider --durations=15 > $D/gputest.log 2>&1
rc=$?
tail -3 $D/gputest.log
[ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python -u bench.py --no-host-resident --no-cpu-baseline"
for k in 1 2 3; do
  $B > $D/ctx_$k.json 2>> $D/bench.err || exit 1
  MIMIC_JIT_DEFS=MIMIC_MEAS_NOCTX $B > $D/noctx_$k.json 2>> $D/bench.err || exit 1
done
for f in $D/ctx_*.json $D/noctx_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$(basename $f)', d['value'], d['roofline']['avg_launch_ms'])"; done
