#!/bin/bash
# per-launch time of bench configs under JIT knob combinations: VARIANTS="NAME:ENV=.. ENV=..;NAME2:..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-var}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$VARIANTS"
for cfg in ${CONFIGS:-classifier}; do
  for rep in 1 2; do
    for v in "${VS[@]}"; do
      name=${v%%:*}; envs=${v#*:}
      env $envs timeout -k 10 200 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-host-resident \
          > gpurun_out/$TAG/b_${cfg}_${name}_$rep.json 2>> gpurun_out/$TAG/bench.err || exit $?
      echo "$cfg $name $(python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/b_${cfg}_${name}_$rep.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
    done
  done
done
