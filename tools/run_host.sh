set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python tools/pcie_probe.py > gpurun_out/$TAG/pcie.log 2>&1
cat gpurun_out/$TAG/pcie.log
timeout -k 10 600 python -m pytest tests/test_gpu_host.py tests/test_gpu_parity.py -x -q > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 300 python bench.py --config classifier --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/hostres.log 2>&1
grep -o '"host_resident": {[^}]*}' gpurun_out/$TAG/hostres.log
