#!/bin/bash
# cfg 3 around the Infinity-Cache size of the counter table (V x 2 KiB)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/p5v; mkdir -p $D
for v in 98304 114688 131072 163840 196608 262144; do
  timeout -k 10 300 python -u bench.py --config parse5 --vcpus $v --no-host-resident --no-cpu-baseline > $D/$v.json 2> $D/$v.err || { tail -5 $D/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$v.json')); print('parse5 V=$v', d['value'], d['roofline']['avg_launch_ms'])"
done
