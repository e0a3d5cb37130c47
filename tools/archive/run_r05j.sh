#!/bin/bash
# round 5: cfg-2 time attribution (tools/memtime.py) across JIT knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05j
mkdir -p $D
for e in "MIMIC_JIT_X=0" "MIMIC_JIT_NOCOLD=1" "MIMIC_JIT_LPF=1" "MIMIC_JIT_LPF=1 MIMIC_JIT_NOCOLD=1" "MIMIC_JIT_NTRES=0" "MIMIC_JIT_WAVES=8 MIMIC_JIT_NOCOLD=1"; do
  n=$(echo $e | tr ' =' '_-')
  env $e MIMIC_JIT_MEMTIME=1 timeout -k 10 200 python tools/memtime.py > $D/memtime_$n.json 2> $D/memtime_$n.err || { tail -3 $D/memtime_$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/memtime_$n.json'))
print('$e', d['launch_us_events'], d['span_us_stamps'], 'start50', d['lane_start_us']['50'], 'end', d['lane_end_us']['50'], d['lane_end_us']['100'], 'pkt50', [d['packet_us'][k]['50'] for k in sorted(d['packet_us'])], 'gap50', [d['gap_to_next_packet_us'][k]['50'] for k in sorted(d['gap_to_next_packet_us'])])"
done
timeout -k 10 600 python tools/api_rates.py > $D/api_rates.json 2> $D/api_rates.err || { tail -20 $D/api_rates.err; exit 1; }
cat $D/api_rates.json
