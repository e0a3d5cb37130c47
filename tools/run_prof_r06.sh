#!/bin/bash
# Round-6 end, part 1: PMC passes (kernel trace, FETCH_SIZE, WRITE_SIZE, read requests by size, SQ) of the
# bench lines' kernels at HEAD; summaries under gpurun_out/prof_$T, copied into profiles/ before part 2
# (tools/run_final_r06.sh) so the bench lines carry their traffic.
#   T=r06 CONFIGS="classifier skb" bash tools/run_prof_r06.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${T:-r06}
for c in ${CONFIGS:-classifier classifier_many5 skb parse5 flowtrack flowtrack_insert}; do
  if [ $c = classifier_v256 ]; then
    CFG=classifier NAME=classifier_v256 EXTRA="--vcpus 256" SUMMARY_ARGS="--vcpus 256 --spread" TAG=$T timeout -k 10 600 bash tools/profile.sh || exit 1
  elif [ $c = classifier_many5 ]; then   # five batches per owned launch (mimic_run_xdp_many)
    CFG=classifier NAME=classifier_many5 EXTRA="--many 5 --batches 5" SUMMARY_ARGS="--vcpus 262144 --own --per-launch 5" TAG=$T timeout -k 10 600 bash tools/profile.sh || exit 1
  elif [ $c = classifier_many8 ]; then   # eight batches per owned launch: the default line
    CFG=classifier NAME=classifier_many8 EXTRA="--many 8" SUMMARY_ARGS="--vcpus 262144 --own --per-launch 8 --batches 8" TAG=$T timeout -k 10 600 bash tools/profile.sh || exit 1
  elif [ $c = classifier ]; then   # one batch per owned launch (the bench's default is five: classifier_many5)
    CFG=$c EXTRA="--many 1" SUMMARY_ARGS="--vcpus 262144 --own" TAG=$T timeout -k 10 600 bash tools/profile.sh || { echo "profile $c failed"; exit 1; }
  elif [ $c = parse5 ]; then   # the owned spread form (engine spread_own)
    CFG=$c SUMMARY_ARGS="--vcpus 262144 --own" TAG=$T timeout -k 10 600 bash tools/profile.sh || { echo "profile $c failed"; exit 1; }
  else
    CFG=$c TAG=$T timeout -k 10 600 bash tools/profile.sh || { echo "profile $c failed"; exit 1; }
  fi
  tail -1 gpurun_out/prof_$T/summary_$c.log | cut -c1-300
done
