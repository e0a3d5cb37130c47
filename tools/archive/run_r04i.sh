#!/bin/bash
# Round 4: cfg 5 with the prog-array slot read through the scalar cache when the index is
# wave-uniform (measurement build), two lines each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config skb"
for k in 1 2; do
  $B > $O/skb_$k.json 2> $O/skb_$k.err || exit 1
  MIMIC_JIT_DEFS=MIMIC_MEAS_PASCALAR $B > $O/skb_pas_$k.json 2> $O/skb_pas_$k.err || exit 1
done
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['status_ok_frac'])"; done
# block combining of freelist reservations (hashmap.h h_comb_reserve): hash / cfg-4 tests, then
# the inserting launch with and without it
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_shard.py tests/test_gpu_bench_size.py -k "not cfg3 and not cfg5" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B2="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config flowtrack_insert"
for k in 1 2; do
  $B2 > $O/ftins_comb_$k.json 2> $O/ftins_comb_$k.err || exit 1
  MIMIC_JIT_COMBINE=0 $B2 > $O/ftins_nocomb_$k.json 2> $O/ftins_nocomb_$k.err || exit 1
done
for f in $O/ftins_*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'), d['status_ok_frac'])"; done
