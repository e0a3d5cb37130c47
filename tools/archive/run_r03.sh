#!/bin/bash
# Round-3 GPU check: the bench-size parity tests, then the bench lines (rotating batches,
# both schedules) and the --gpus launcher on a 1-GPU box.  Each step has its own limit; the
# script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r03}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_bench_size.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    --durations=10 > $D/gputest.log 2>&1
rc=$?
tail -15 $D/gputest.log
[ $rc -eq 0 ] || exit $rc
for s in interleaved chunked; do
  timeout -k 10 300 python -u bench.py --sched $s --no-host-resident --no-cpu-baseline > $D/bench_$s.json 2> $D/bench_$s.err || { tail -20 $D/bench_$s.err; exit 1; }
  cat $D/bench_$s.json
done
timeout -k 10 120 python -u bench.py --gpus 2 > $D/gpus2.out 2>&1; echo "bench --gpus 2 rc=$?"; cat $D/gpus2.out
