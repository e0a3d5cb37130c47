#!/bin/bash
# round 5: block combiner with slot reader counts (HEAD) vs round 5's mailboxes (.ab/mb) vs round 4's slots (.ab/hx):
# hash tests, then cfg-4 lookup-hit and inserting launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
D=$R/gpurun_out/r05p
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash.py tests/test_gpu_bench_size.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -30 $D/test.log; exit 1; }
tail -2 $D/test.log
for c in flowtrack flowtrack_insert; do
for k in 1 2; do
  for w in ${AB_DIRS:-. .ab/hx}; do
    n=$(basename $w)
    (cd $R/$w && timeout -k 10 300 python -u bench.py --config $c --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/${c}_${n}_$k.json 2> $D/${c}_${n}_$k.err) || { tail -5 $D/${c}_${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/${c}_${n}_$k.json')); print('$c $w', d['value'], d['ms_per_step'])"
  done
done
done
