set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/tests_jit.log 2>&1 || { tail -40 gpurun_out/$TAG/tests_jit.log; exit 1; }
tail -1 gpurun_out/$TAG/tests_jit.log
MIMIC_EXEC=interp timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/tests_interp.log 2>&1 || { tail -40 gpurun_out/$TAG/tests_interp.log; exit 1; }
tail -1 gpurun_out/$TAG/tests_interp.log
bash tools/run_bench.sh
