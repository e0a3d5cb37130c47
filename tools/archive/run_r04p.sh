#!/bin/bash
# Round 4: spread launches whose LDS table covers every lane flush through per-block tables and
# one reduce kernel (jit.cpp / interp.hip mimic_spread_reduce_kernel): spread GPU tests, then the
# V = 256 classifier and parse5 lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_spread.py > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident"
$B --config classifier --vcpus 256 > $O/cls_v256.json 2> $O/cls_v256.err || exit 1
$B --config classifier --vcpus 1024 > $O/cls_v1024.json 2> $O/cls_v1024.err || exit 1
$B --config parse5 --vcpus 256 --steps 10 --warmup 2 > $O/p5_v256.json 2> $O/p5_v256.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o a -- python3 bench.py --no-cpu-baseline --no-host-resident --config classifier --vcpus 256 --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err || exit 1
grep -h "mimic_jit_kernel\|spread_reduce" $(find $O/kt -name '*kernel_stats.csv')
for f in $O/cls_v256.json $O/cls_v1024.json $O/p5_v256.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['engine'], d['counters_sum'])"; done
