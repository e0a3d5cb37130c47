# profiles for one workload: bench line (+ CPU baseline, host-resident), kernel trace stats,
# FETCH_SIZE and WRITE_SIZE passes (separately, MI355X_MICROARCH.md), SQ instruction mix
set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
CFG=${CFG:-classifier}
timeout -k 10 300 python bench.py --config $CFG > gpurun_out/$TAG/bench_$CFG.json 2> gpurun_out/$TAG/bench_$CFG.err
B="python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt_$CFG -o a -- $B > gpurun_out/$TAG/kt_$CFG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/$TAG/fetch_$CFG -o a -- $B > gpurun_out/$TAG/fetch_$CFG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/$TAG/write_$CFG -o a -- $B > gpurun_out/$TAG/write_$CFG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/$TAG/sq_$CFG -o a -- $B > gpurun_out/$TAG/sq_$CFG.log 2>&1
cut -c1-300 gpurun_out/$TAG/bench_$CFG.json
