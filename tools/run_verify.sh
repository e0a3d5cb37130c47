# GPU: sk_buff parity (JIT, interpreter), full GPU suite (JIT), smoke, default bench line.
set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
PYT="python -u -m pytest -x --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT -v tests/test_gpu_skb.py > gpurun_out/$TAG/skb_jit.log 2>&1 || { tail -60 gpurun_out/$TAG/skb_jit.log; exit 1; }
tail -1 gpurun_out/$TAG/skb_jit.log
MIMIC_EXEC=interp timeout -k 10 300 $PYT -v tests/test_gpu_skb.py > gpurun_out/$TAG/skb_interp.log 2>&1 || { tail -60 gpurun_out/$TAG/skb_interp.log; exit 1; }
tail -1 gpurun_out/$TAG/skb_interp.log
timeout -k 10 500 $PYT -v -m gpu tests > gpurun_out/$TAG/tests_jit.log 2>&1 || { tail -60 gpurun_out/$TAG/tests_jit.log; exit 1; }
tail -1 gpurun_out/$TAG/tests_jit.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -30 gpurun_out/$TAG/smoke.log; exit 1; }
cat gpurun_out/$TAG/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
