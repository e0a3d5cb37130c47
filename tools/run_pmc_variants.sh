#!/bin/bash
# tools/profile.sh per codegen / bench variant: VARIANTS="name:ENV=1,ENV2=0:--bench-args ..."
#   (fields separated by ':', env assignments by ',', bench args by '+')
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export MIMIC_JIT_CACHE=/tmp/mimic_jitcache
for v in $VARIANTS; do
  name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; args=${rest#*:}
  [ "$args" = "$rest" ] && args=""
  env ${envs//,/ } CFG=${CFG:-classifier} TAG=$name EXTRA="${args//+/ }" bash tools/profile.sh || exit $?
done
