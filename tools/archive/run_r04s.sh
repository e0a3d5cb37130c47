#!/bin/bash
# Round 4: cfg 5 with the rooms zeroed unconditionally by the chain (no room reads anywhere:
# MIMIC_SKB_ROOMS_CHAIN=1 + MIMIC_JIT_ROOMS=0) vs the prep's rooms flag (default); kernel split.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
B="python3 -u bench.py --no-cpu-baseline --no-host-resident --config skb"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_def -o a -- $B --steps 10 --warmup 2 > $O/kt_def.json 2> $O/kt_def.err || exit 1
MIMIC_SKB_ROOMS_CHAIN=1 MIMIC_JIT_ROOMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_zero -o a -- $B --steps 10 --warmup 2 > $O/kt_zero.json 2> $O/kt_zero.err || exit 1
for d in kt_def kt_zero; do echo "== $d"; grep -h "mimic_skb_prep_kernel\|mimic_jit_kernel" $(find $O/$d -name '*kernel_stats.csv'); done
timeout -k 10 300 $B > $O/def.json 2> $O/def.err || exit 1
MIMIC_SKB_ROOMS_CHAIN=1 MIMIC_JIT_ROOMS=0 timeout -k 10 300 $B > $O/zero.json 2> $O/zero.err || exit 1
for f in $O/def.json $O/zero.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['status_ok_frac'])"; done
