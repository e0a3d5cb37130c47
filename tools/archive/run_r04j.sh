#!/bin/bash
# Round 4: inserts write their key words before the freelist reservation; the combiner's window
# (s_sleep 1 / 2 / 4 / 8) on the inserting cfg-4 launch; hash and cfg-4 tests first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_shard.py tests/test_gpu_bench_size.py tests/test_gpu_fastpaths.py -k "not cfg3 and not cfg5" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B2="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config flowtrack_insert"
for v in 2 1 4 8; do
  MIMIC_JIT_DEFS=MIMIC_HCOMB_SLEEP=$v $B2 > $O/ftins_s$v.json 2> $O/ftins_s$v.err || exit 1
done
$B2 > $O/ftins_default.json 2> $O/ftins_default.err || exit 1
MIMIC_JIT_COMBINE=0 $B2 > $O/ftins_nocomb.json 2> $O/ftins_nocomb.err || exit 1
for f in $O/ftins_*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'), d['status_ok_frac'])"; done
