#!/bin/bash
# round 6: cfg-4 inserting launch with chunked reservations of several sizes (MIMIC_JIT_HCHUNK; 0 =
# the block combiner of round 5), bench lines + kernel traces (JIT kernel, compaction, reset)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r06c}
mkdir -p $D
for hc in ${HCS:-32 0 16 64}; do
  MIMIC_JIT_HCHUNK=$hc timeout -k 10 200 python3 bench.py --config ${CFG:-flowtrack_insert} --steps 20 --warmup 5 --no-cpu-baseline --no-host-resident > $D/bench_hc$hc.json 2> $D/bench_hc$hc.err || exit $?
  MIMIC_JIT_HCHUNK=$hc timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_hc$hc -o a -- python3 bench.py --config ${CFG:-flowtrack_insert} --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt_hc$hc.log 2>&1 || exit $?
  cp $(find $D/kt_hc$hc -name '*kernel_stats.csv' | head -1) $D/kstats_hc$hc.csv
  echo "hc=$hc $(python3 -c "import json,sys; d=json.loads(open('$D/bench_hc$hc.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
