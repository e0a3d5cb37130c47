#!/bin/bash
# Round 4: cfg-5 rooms check in prep vs in the chain (kernel split under rocprofv3), cfg 3 as a
# spread launch at V = 262 144, and the --rccl line's stdout (one JSON line).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
B="python3 -u bench.py --no-cpu-baseline --no-host-resident"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_skb -o a -- $B --config skb --steps 10 --warmup 2 > $O/skb.json 2> $O/skb.err || exit 1
MIMIC_SKB_ROOMS_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_skb_rc -o a -- $B --config skb --steps 10 --warmup 2 > $O/skb_rc.json 2> $O/skb_rc.err || exit 1
for d in kt_skb kt_skb_rc; do echo "== $d"; grep -h "mimic_skb_prep_kernel\|mimic_jit_kernel" $(find $O/$d -name '*kernel_stats.csv'); done
timeout -k 10 300 $B --config parse5 --steps 10 --warmup 2 > $O/p5.json 2> $O/p5.err || exit 1
MIMIC_SPREAD=1 timeout -k 10 300 $B --config parse5 --steps 10 --warmup 2 > $O/p5_spread.json 2> $O/p5_spread.err || exit 1
timeout -k 10 300 $B --config flowtrack --rccl > $O/ft_rccl.json 2> $O/ft_rccl.err || exit 1
for f in $O/skb.json $O/skb_rc.json $O/p5.json $O/p5_spread.json $O/ft_rccl.json; do echo "== $f"; python3 -c "import json; L=open('$f').read().splitlines(); print(len(L), 'lines'); d=json.loads(L[-1]); print(d['value'], d['ms_per_step'], d['config']['engine'], d['roofline']['avg_launch_ms'], d['status_ok_frac'])"; done
