#!/bin/bash
# Round 4: where the spread classifier's time goes at V = 256: the LDS table's flush (one
# agent-scope add per non-zero counter per block; MIMIC_MEAS_NOFLUSH drops it, counters wrong) and
# packets per block (MIMIC_SPREAD_PPB 1024 / 2048 / 4096: fewer blocks, fewer flushes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --config classifier --vcpus 256"
$B > $O/v256.json 2> $O/v256.err || exit 1
MIMIC_JIT_DEFS=MIMIC_MEAS_NOFLUSH $B > $O/v256_noflush.json 2> $O/v256_noflush.err || exit 1
MIMIC_SPREAD_PPB=2048 $B > $O/v256_ppb2048.json 2> $O/v256_ppb2048.err || exit 1
MIMIC_SPREAD_PPB=4096 $B > $O/v256_ppb4096.json 2> $O/v256_ppb4096.err || exit 1
MIMIC_SPREAD_PPB=512 $B > $O/v256_ppb512.json 2> $O/v256_ppb512.err || exit 1
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['engine'], d['counters_sum'])"; done
