#!/bin/bash
# Round 4: one-kernel hash map reset (16-byte fills): hash tests, then the inserting cfg-4 line
# (a reset every step) under a kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_bench_size.py -k "not cfg3 and not cfg5" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o a -- python3 bench.py --no-cpu-baseline --no-host-resident --config flowtrack_insert --steps 10 --warmup 2 > $O/kt.json 2> $O/kt.err || exit 1
cat $(find $O/kt -name '*kernel_stats.csv') | cut -c1-150
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config flowtrack_insert > $O/ftins.json 2> $O/ftins.err || exit 1
python3 -c "import json; d=json.load(open('$O/ftins.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'))"
