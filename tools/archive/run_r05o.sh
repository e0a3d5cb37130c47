#!/bin/bash
# round 5: cfg-4 lookup-hit launch at HEAD vs round 4 (61cde63) vs 5397051 (A/B worktrees under .ab/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
D=$R/gpurun_out/r05o
mkdir -p $D
for k in 1 2; do
  for w in ${AB_DIRS:-. .ab/r04 .ab/c539}; do
    n=$(basename $w)
    (cd $R/$w && timeout -k 10 300 python -u bench.py --config flowtrack --steps 30 --warmup 3 --no-host-resident --no-cpu-baseline > $D/ft_${n}_$k.json 2> $D/ft_${n}_$k.err) || { tail -5 $D/ft_${n}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/ft_${n}_$k.json')); print('$w', d['value'], d['ms_per_step'])"
  done
done
