#!/bin/bash
# Round 4: cfg 2 default and V = 256 spread bench lines, the cfg-4 --rccl line (stderr kept),
# then PMC passes of the V = 256 spread kernel and of the default classifier.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-resident"
$B --config classifier > $O/cls.json 2> $O/cls.err || exit 1
$B --config classifier --vcpus 256 > $O/cls_v256.json 2> $O/cls_v256.err || exit 1
$B --config parse5 --vcpus 256 --steps 5 --warmup 1 > $O/p5_v256.json 2> $O/p5_v256.err || exit 1
$B --config flowtrack --rccl > $O/flowtrack_rccl.json 2> $O/flowtrack_rccl.err; echo "flowtrack rccl rc=$?" >> $O/flowtrack_rccl.err
CFG=classifier NAME=classifier_v256 EXTRA="--vcpus 256" SUMMARY_ARGS="--vcpus 256 --spread" TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
CFG=classifier TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
for f in $O/*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['config']['engine'], d['config']['vcpus_per_gpu'], d['roofline']['frac'], d.get('hash_keys'))"; done
tail -3 $O/flowtrack_rccl.err
grep -h "mimic_jit_kernel" gpurun_out/prof_r04/r04_kernel_stats_*.csv
