#!/bin/bash
# round 5: block-combiner variants (A/B worktrees under .ab/), cfg-4 lookup-hit and inserting launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
D=$R/gpurun_out/r05q
mkdir -p $D
for c in flowtrack flowtrack_insert; do
for k in 1 2; do
  for w in ${AB_DIRS:-. .ab/hx .ab/v1 .ab/v2}; do
    n=$(basename $w)
    (cd $R/$w && timeout -k 10 300 python -u bench.py --config $c --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/${c}_${n}_$k.json 2> $D/${c}_${n}_$k.err) || { tail -5 $D/${c}_${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/${c}_${n}_$k.json')); print('$c $w', d['value'], d['ms_per_step'])"
  done
done
done
