#!/bin/bash
# rocprofv3 passes for one bench config (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, read requests
# by size, SQ mix),
# each in its own run as MI355X_MICROARCH.md prescribes, then the summary the bench line reads.
#   CFG=classifier TAG=r02 bash tools/profile.sh
#   CFG=classifier NAME=classifier_v256 EXTRA="--vcpus 256" SUMMARY_ARGS="--vcpus 256 --spread" TAG=r04 bash tools/profile.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${CFG:-classifier}
NAME=${NAME:-$CFG}
TAG=${TAG:-r02}
EXTRA=${EXTRA:-}
D=gpurun_out/prof_${TAG}
mkdir -p $D
B="python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt_$NAME -o a -- $B > $D/kt_$NAME.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch_$NAME -o a -- $B > $D/fetch_$NAME.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write_$NAME -o a -- $B > $D/write_$NAME.log 2>&1 || exit $?
# read requests by size (gfx950: 32 / 64 / 128-byte requests; FETCH_SIZE tallies 128-B ones at 64 B)
if [ "${REQ:-1}" = 1 ]; then
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $D/req_$NAME -o a -- $B > $D/req_$NAME.log 2>&1 || exit $?
fi
[ "${SQ:-1}" = 1 ] && { timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $D/sq_$NAME -o a -- $B > $D/sq_$NAME.log 2>&1 || exit $?; }
python3 tools/pmc_summary.py --config $CFG --name $NAME --dir $D --tag $TAG --out $D/${TAG}_pmc_$NAME.json --command "$B" ${SUMMARY_ARGS:-} > $D/summary_$NAME.log 2>&1 || exit $?
cp $(find $D/kt_$NAME -name '*kernel_stats.csv' | head -1) $D/${TAG}_kernel_stats_$NAME.csv
