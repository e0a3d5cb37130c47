#!/bin/bash
# JIT codegen variants of one config under the rotating-batch bench (knobs are env variables read
# by the generator).  VARIANTS: ';'-separated "label|ENV=.. ENV=..|extra bench args".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-sweep}
CFG=${CFG:-classifier}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-default||}"
for v in "${VS[@]}"; do
  IFS='|' read -r label envs extra <<< "$v"
  env $envs timeout -k 10 300 python -u bench.py --config $CFG --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline \
      --no-host-resident $extra > $D/$label.json 2> $D/$label.err || { echo "$label failed"; tail -5 $D/$label.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/$label.json')); r=d['roofline']; print('$label', d['value'], 'Mpkts/s', r['avg_launch_ms'], 'ms', r['frac'])"
done
