set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_hash.py tests/test_gpu_kat.py -x -q -m gpu > gpurun_out/$TAG/tests_hash.log 2>&1 || { tail -40 gpurun_out/$TAG/tests_hash.log; exit 1; }
tail -2 gpurun_out/$TAG/tests_hash.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/$TAG/tests_parity.log 2>&1 || { tail -40 gpurun_out/$TAG/tests_parity.log; exit 1; }
tail -2 gpurun_out/$TAG/tests_parity.log
timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident > gpurun_out/$TAG/bench.log 2>&1
timeout -k 10 300 python bench.py --config flowtrack --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident >> gpurun_out/$TAG/bench.log 2>&1
cat gpurun_out/$TAG/bench.log | cut -c1-400
