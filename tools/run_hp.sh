set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python tools/host_probe.py > gpurun_out/$TAG/hp.log 2>&1
cat gpurun_out/$TAG/hp.log
timeout -k 10 120 python tools/launch_probe.py >> gpurun_out/$TAG/hp.log 2>&1
cat gpurun_out/$TAG/hp.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/$TAG/hptrace -o a -- python3 tools/host_probe.py > gpurun_out/$TAG/hptrace.log 2>&1
ls gpurun_out/$TAG/hptrace
