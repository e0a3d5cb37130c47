#!/bin/bash
# Round 4: hash probes reading HT_WIN state words per round trip (hashmap.h h_find / the insert
# walk): hash and cfg-4 tests, then cfg-4 lines at HT_WIN = 1 (round 3's walk), 2 (default), 4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_shard.py tests/test_gpu_bench_size.py tests/test_gpu_fastpaths.py -k "not cfg3 and not cfg5" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident"
for w in 2 1 4; do
  for c in flowtrack flowtrack_insert; do
    MIMIC_JIT_DEFS=HT_WIN=${w}u $B --config $c > $O/${c}_w$w.json 2> $O/${c}_w$w.err || exit 1
  done
done
$B --config flowtrack > $O/flowtrack_def.json 2> $O/flowtrack_def.err || exit 1
$B --config flowtrack_insert > $O/flowtrack_insert_def.json 2> $O/flowtrack_insert_def.err || exit 1
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'))"; done
