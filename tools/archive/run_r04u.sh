#!/bin/bash
# Round 4 (session 2), run on branch exp/skb-stream (not merged: no gain): streamed sk_buff batches --
# MIMIC_SKB_F_STREAM (alternating, 2 runs each), then the default line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r04u
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_skb.py tests/test_gpu_ctx.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/test.log 2>&1
rc=$?
tail -3 $D/test.log
[ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python -u bench.py --no-host-resident --no-cpu-baseline --config skb"
for k in 1 2; do
  $B > $D/stream_$k.json 2>> $D/bench.err || exit 1
  $B --no-skb-stream > $D/nostream_$k.json 2>> $D/bench.err || exit 1
done
for f in $D/stream_*.json $D/nostream_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$(basename $f)', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['status_ok_frac'])"; done
