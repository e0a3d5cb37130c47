#!/bin/bash
# Round 4: hash / spread / shard / pool GPU tests, then bench lines (cfg 2 default and V = 256
# spread, cfg 3 at V = 256, cfg-4 inserting with and without stripe locks, cfg 4 --rccl), then PMC
# passes of the V = 256 spread kernel and the cfg-4 inserting launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_spread.py tests/test_gpu_shard.py tests/test_gpu_pool.py tests/test_gpu_vc.py \
  tests/test_gpu_bench_size.py tests/test_gpu_skb.py -s > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log; grep "host updates" $O/gputest.log
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-resident"
$B --config classifier > $O/cls.json 2> $O/cls.err || exit 1
$B --config classifier --vcpus 256 > $O/cls_v256.json 2> $O/cls_v256.err || exit 1
$B --config parse5 --vcpus 256 --steps 5 --warmup 1 > $O/p5_v256.json 2> $O/p5_v256.err || exit 1
$B --config skb > $O/skb.json 2> $O/skb.err || exit 1
$B --config flowtrack_insert > $O/ftins.json 2> $O/ftins.err || exit 1
MIMIC_JIT_DEFS=MIMIC_HASH_NOLOCK=0 $B --config flowtrack_insert > $O/ftins_locked.json 2> $O/ftins_locked.err || exit 1
$B --config flowtrack --rccl > $O/flowtrack_rccl.json 2> $O/flowtrack_rccl.err; echo "flowtrack rccl rc=$?" >> $O/flowtrack_rccl.err
for f in $O/*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['config']['engine'], d['config']['vcpus_per_gpu'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d.get('hash_keys'))"; done
tail -3 $O/flowtrack_rccl.err
CFG=classifier NAME=classifier_v256 EXTRA="--vcpus 256" SUMMARY_ARGS="--vcpus 256 --spread" TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
CFG=flowtrack_insert TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
grep -h "mimic_jit_kernel" gpurun_out/prof_r04/r04_kernel_stats_*.csv
