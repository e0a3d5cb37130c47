#!/bin/bash
# Round 4, cfg 5 traffic attribution: the chain kernel's HBM bytes (reads by request size + WRITE)
# with one kind of memory work switched off at a time (MIMIC_JIT_DEFS measurement knobs: results
# are wrong with them on), then timing lines with the deferral sites' register stores dropped
# (nothing defers in cfg 5, so those results stay exact) at 2 and 3 waves.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
for v in default:"" nopktst:MIMIC_MEAS_NOPKTST nores:MIMIC_MEAS_NORES noatom:MIMIC_MEAS_NOATOM none:MIMIC_MEAS_NOPKTST,MIMIC_MEAS_NORES,MIMIC_MEAS_NOATOM; do
  name=${v%%:*}; defs=${v#*:}
  SQ=$([ $name = default ] && echo 1 || echo 0) MIMIC_JIT_DEFS=$defs CFG=skb NAME=skb_$name TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/prof_r04/r04_pmc_skb_$name.json')); print('$name', d['kernel_stats']['avg_ns'], d.get('fetch_size_kib_per_launch'), d.get('write_size_kib_per_launch'), d.get('read_requests_per_launch'), d.get('read_bytes_per_launch'))"
done
B="timeout -k 10 300 python -u bench.py --config skb --no-cpu-baseline --no-host-resident"
$B > $O/skb_default.json 2> $O/skb_default.err || exit 1
MIMIC_JIT_DEFER_NOREGS=1 $B > $O/skb_noregs.json 2> $O/skb_noregs.err || exit 1
MIMIC_JIT_DEFER_NOREGS=1 MIMIC_JIT_WAVES=3 $B > $O/skb_noregs_w3.json 2> $O/skb_noregs_w3.err || exit 1
for f in $O/skb_*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['status_ok_frac'])"; done
