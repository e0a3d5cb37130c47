set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -2 gpurun_out/$TAG/tests.log
for v in 262144 1048576; do timeout -k 10 120 python bench.py --steps 10 --warmup 2 --vcpus $v --no-cpu-baseline >> gpurun_out/$TAG/bench.log 2>&1; done
timeout -k 10 120 python bench.py --config pass8 --steps 10 --no-cpu-baseline >> gpurun_out/$TAG/bench.log 2>&1
for cfg in pass8 classifier; do timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/$TAG/pmc_$cfg -o a -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/pmc_$cfg.log 2>&1; done
