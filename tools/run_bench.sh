set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for c in classifier pass8 parse5 flowtrack; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident >> gpurun_out/$TAG/bench_jit.log 2>&1; done
for c in classifier parse5 flowtrack; do MIMIC_EXEC=interp timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident >> gpurun_out/$TAG/bench_interp.log 2>&1; done
grep -h '"value"' gpurun_out/$TAG/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['engine'], d['config']['workload'][:30], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['insns_per_s']/1e9)"
