#!/bin/bash
# round 6: the compaction kernel after cfg-4 inserting launches at several grid sizes (kernel traces)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/${TAG:-r06k}
mkdir -p $D
for nb in ${NBS:-32 128 256}; do
  MIMIC_COMPACT_BLOCKS=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_nb$nb -o a -- python3 bench.py --config flowtrack_insert --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt_nb$nb.log 2>&1 || exit $?
  cp $(find $D/kt_nb$nb -name '*kernel_stats.csv' | head -1) $D/kstats_nb$nb.csv
  echo "nb=$nb $(grep compact $D/kstats_nb$nb.csv | cut -d, -f1-4)"
done
for ms in ${MEAS:-1 2 3}; do
  MIMIC_COMPACT_MEAS=$ms timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_ms$ms -o a -- python3 bench.py --config flowtrack_insert --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > $D/kt_ms$ms.log 2>&1 || exit $?
  cp $(find $D/kt_ms$ms -name '*kernel_stats.csv' | head -1) $D/kstats_ms$ms.csv
  echo "meas=$ms $(grep compact $D/kstats_ms$ms.csv | cut -d, -f1-4)"
done
