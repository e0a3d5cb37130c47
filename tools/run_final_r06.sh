#!/bin/bash
# Round-6 end, part 2: the driver's tiers (fresh JIT cache: -m gpu suite, smoke, default bench line), then
# one bench line per config at HEAD (they read the part-1 profiles from profiles/), the multi-batch line,
# the two-rank rehearsal of the N-GPU path on one GPU, and the reference-shaped API rates.
#   T=r06final PART=1 bash tools/run_final_r06.sh ; T=r06final PART=2 bash tools/run_final_r06.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06final}
D=gpurun_out/$T
B="timeout -k 10 300 python -u bench.py --no-host-resident --no-cpu-baseline"
if [ "${PART:-1}" = 1 ]; then
TAG=$T bash tools/run_driver.sh || exit 1
for c in classifier parse5 flowtrack flowtrack_insert skb pass8; do
  $B --config $c > $D/bench_$c.json 2> $D/bench_$c.err || { tail -20 $D/bench_$c.err; exit 1; }
done
$B --config classifier --many 1 > $D/bench_classifier_many1.json 2> $D/bench_classifier_many1.err || exit 1   # one batch per launch
$B --config classifier --many 5 --batches 5 > $D/bench_classifier_many5.json 2> $D/bench_classifier_many5.err || exit 1   # round 6's first default
fi
if [ "${PART:-2}" = 2 ]; then
mkdir -p $D
$B --config classifier --many 1 --vcpus 256 > $D/bench_classifier_v256.json 2> $D/bench_classifier_v256.err || exit 1
$B --config classifier --many 1 --sched chunked > $D/bench_classifier_chunked.json 2> $D/bench_classifier_chunked.err || exit 1
$B --config classifier --steps 20 > $D/bench_classifier_20steps.json 2> $D/bench_classifier_20steps.err || exit 1
$B --config flowtrack --rccl > $D/bench_flowtrack_rccl.json 2> $D/bench_flowtrack_rccl.err || exit 1
for c in classifier flowtrack; do   # the N-rank path at N = 2, both engines on GPU 0, gloo collectives
  $B --gpus 2 --dist-backend gloo --one-device --config $c --steps 20 > $D/bench_${c}_2rank.json 2> $D/bench_${c}_2rank.err || { tail -20 $D/bench_${c}_2rank.err; exit 1; }
done
timeout -k 10 600 python tools/api_rates.py > $D/api_rates.json 2> $D/api_rates.err && cat $D/api_rates.json
fi
for f in $D/bench_*.json; do python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print('$(basename $f)', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r.get('frac_on_traffic'), r.get('traffic_over_algorithmic'), d['config']['engine'], d['n_gpus'])"; done
