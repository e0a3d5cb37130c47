#!/bin/bash
# Round 4: the driver's tiers at HEAD (fresh JIT cache), then bench lines: cfg 2 at the default
# V and at V = 256 (spread), cfg 2 forced one-lane at V = 256, cfg 4 (one batch sharded).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r04b bash tools/run_driver.sh || exit 1
O=gpurun_out/r04b
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-resident"
$B --config classifier --vcpus 256 > $O/cls_v256.json 2> $O/cls_v256.err || exit 1
MIMIC_SPREAD=1 $B --config classifier > $O/cls_spread_default_v.json 2> $O/cls_spread_default_v.err || exit 1
MIMIC_SPREAD=0 $B --config classifier --vcpus 256 --steps 3 --warmup 1 > $O/cls_v256_onelane.json 2> $O/cls_v256_onelane.err || exit 1
$B --config parse5 --vcpus 256 --steps 5 --warmup 1 > $O/p5_v256.json 2> $O/p5_v256.err || exit 1
$B --config flowtrack > $O/flowtrack.json 2> $O/flowtrack.err || exit 1
$B --config flowtrack --rccl > $O/flowtrack_rccl.json 2> $O/flowtrack_rccl.err || exit 1
for f in $O/*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['config']['engine'], d['config']['vcpus_per_gpu'], d['roofline']['frac'], d.get('hash_keys'))"; done
