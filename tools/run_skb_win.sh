#!/bin/bash
# sk_buff prep with the current header window: skb GPU tests, the prep probe, the cfg-5 bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/skbwin; mkdir -p $D
export TMPDIR=/tmp
unset MIMIC_JIT_CACHE
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "skb or bench_size or step" --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/gputest.log 2>&1 || { tail -30 $D/gputest.log; exit 1; }
tail -1 $D/gputest.log
bash tools/prep_probe.sh || exit 1
timeout -k 10 400 python -u bench.py --config skb --no-host-resident --no-cpu-baseline > $D/bench_skb.json 2> $D/bench_skb.err || { tail -20 $D/bench_skb.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_skb.json')); print('skb', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
