#!/bin/bash
# cfg-4 inserting launch under the hash-insert knobs: stripe-lock count (MIMIC_HASH_LOCKS_LOG2)
# and the lock-free re-check of waiting lanes (MIMIC_JIT_DEFS=MIMIC_HASH_RECHECK)
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
for v in ${VARIANTS:-base lk19 recheck both}; do
  case $v in
    base) run base MIMIC_X=0 ;;
    lk19) run lk19 MIMIC_HASH_LOCKS_LOG2=19 ;;
    lk12) run lk12 MIMIC_HASH_LOCKS_LOG2=12 ;;
    lk20) run lk20 MIMIC_HASH_LOCKS_LOG2=20 ;;
    lk21) run lk21 MIMIC_HASH_LOCKS_LOG2=21 ;;
    lk16) run lk16 MIMIC_HASH_LOCKS_LOG2=16 ;;
    recheck) run recheck MIMIC_JIT_DEFS=MIMIC_HASH_RECHECK ;;
    both) run both MIMIC_HASH_LOCKS_LOG2=19 MIMIC_JIT_DEFS=MIMIC_HASH_RECHECK ;;
  esac
done
