#!/bin/bash
# Process.Run per-call split + the bench lines under the new byte model (no profiles).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06b}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/api_rates.py --xdp-jobs 65536 --skb-jobs 16384 > gpurun_out/$TAG/api_rates.json 2> gpurun_out/$TAG/api_rates.err || { tail -30 gpurun_out/$TAG/api_rates.err; exit 1; }
cat gpurun_out/$TAG/api_rates.json
for c in classifier parse5 flowtrack flowtrack_insert skb; do
  timeout -k 10 300 python -u bench.py --config $c --steps 30 --no-cpu-baseline --no-host-resident > gpurun_out/$TAG/bench_$c.json 2> gpurun_out/$TAG/bench_$c.err || { tail -20 gpurun_out/$TAG/bench_$c.err; exit 1; }
  cat gpurun_out/$TAG/bench_$c.json
done
