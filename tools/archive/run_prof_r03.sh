#!/bin/bash
# PMC passes (tools/profile.sh) for the listed bench configs; summaries under gpurun_out/prof_<TAG>.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r03}
for c in ${CONFIGS:-classifier skb parse5 flowtrack}; do
  CFG=$c TAG=$TAG timeout -k 10 900 bash tools/profile.sh || { echo "profile $c failed"; exit 1; }
  tail -3 gpurun_out/prof_$TAG/summary_$c.log
done
