#!/bin/bash
# Round 5, cfg 5 A/B: sk_buff GPU tests, then the skb bench line and a kernel trace for each value
# of one JIT knob (KNOB=MIMIC_JIT_SKBTOUCH VARIANTS="1 0").
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${T:-r05d}
KNOB=${KNOB:-MIMIC_JIT_SKBTOUCH}
D=gpurun_out/$T
mkdir -p $D
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_bench_size.py tests/test_gpu_step.py tests/test_gpu_pool.py \
  -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -40 $D/test.log; exit 1; }
tail -2 $D/test.log
fi
B="python3 bench.py --config ${CFG:-skb} --no-cpu-baseline --no-host-resident ${EXTRA:-}"
for v in ${VARIANTS:-1 0}; do
  for rep in 1 2; do
  env $KNOB=$v timeout -k 10 300 $B > $D/bench_$v.$rep.json 2> $D/bench_$v.$rep.err || { tail -20 $D/bench_$v.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$v.$rep.json')); print('$KNOB=$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
  env $KNOB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_$v -o a -- $B --steps 20 > $D/kt_$v.log 2>&1 || exit 1
  f=$(find $D/kt_$v -name '*kernel_stats.csv' | head -1); cp $f $D/kernel_stats_$v.csv
  head -6 $D/kernel_stats_$v.csv | cut -d, -f1-4
done
