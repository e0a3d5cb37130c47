# GPU: sk_buff parity (JIT, then interpreter), then the rest of the GPU suite in JIT mode.
set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_skb.py -x -v --timeout 400 --timeout-method thread > gpurun_out/$TAG/skb_jit.log 2>&1 || { tail -60 gpurun_out/$TAG/skb_jit.log; exit 1; }
tail -1 gpurun_out/$TAG/skb_jit.log
MIMIC_EXEC=interp timeout -k 10 300 python -u -m pytest tests/test_gpu_skb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/skb_interp.log 2>&1 || { tail -60 gpurun_out/$TAG/skb_interp.log; exit 1; }
tail -1 gpurun_out/$TAG/skb_interp.log
