#!/bin/bash
# cfg-4 inserting launch (CFG=flowtrack: the lookup-hit launch) at several stripe-lock counts
# (MIMIC_HASH_LOCKS_LOG2; the default is 4 locks per bucket).  The round-3 measurements also had
# the waiting lanes' lock-free re-check as a knob (now always on): 0.456 -> 0.441 ms at 2^19.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/insk; mkdir -p $D
export TMPDIR=/tmp
unset MIMIC_JIT_CACHE
: > $D/lines.jsonl
run() {   # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config ${CFG:-flowtrack_insert} --no-host-resident --no-cpu-baseline \
      > $D/$n.json 2> $D/$n.err || { tail -20 $D/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/$n.json')); d['variant']='$n'; print(json.dumps(d))" >> $D/lines.jsonl
  python3 -c "import json; d=json.load(open('$D/$n.json')); print('$n', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for v in ${VARIANTS:-base lk16 lk19 lk20}; do
  case $v in
    base) run base MIMIC_X=0 ;;
    lk19) run lk19 MIMIC_HASH_LOCKS_LOG2=19 ;;
    lk12) run lk12 MIMIC_HASH_LOCKS_LOG2=12 ;;
    lk20) run lk20 MIMIC_HASH_LOCKS_LOG2=20 ;;
    lk21) run lk21 MIMIC_HASH_LOCKS_LOG2=21 ;;
    lk16) run lk16 MIMIC_HASH_LOCKS_LOG2=16 ;;
  esac
done
