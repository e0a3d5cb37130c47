#!/bin/bash
# cfg 5: register budget (MIMIC_JIT_WAVES) x vCPUs per GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-skbv}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for rep in 1 2; do
for w in 0 2; do
  for v in 65536 131072 262144; do
    MIMIC_JIT_WAVES=$w timeout -k 10 300 python -u bench.py --config skb --vcpus $v --steps 10 --warmup 3 --no-cpu-baseline --no-host-resident \
        > gpurun_out/$TAG/b_${w}_${v}_$rep.json 2>> gpurun_out/$TAG/bench.err || exit $?
    echo "waves=$w V=$v $(python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/b_${w}_${v}_$rep.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
  done
done
done
