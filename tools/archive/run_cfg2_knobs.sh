#!/bin/bash
# cfg 2 (default bench line) under JIT knobs / vCPU counts, one bench line each (rotating batches)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/cfg2k; mkdir -p $D
run() {   # name, env, extra args
  env $2 timeout -k 10 300 python -u bench.py --config classifier --no-host-resident --no-cpu-baseline $3 > $D/$1.json 2> $D/$1.err || { tail -5 $D/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$1.json')); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
}
run default "X=1" ""
run xpf "MIMIC_JIT_XPF=1" ""
run v128k "X=1" "--vcpus 131072"
run v512k "X=1" "--vcpus 524288"
run waves5 "MIMIC_JIT_WAVES=5" ""
run chunked "X=1" "--sched chunked"
