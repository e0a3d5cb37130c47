set -e
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG/sweep.log
for f in 1 0; do for k in ptr val; do for c in classifier pass8 flowtrack; do
  echo "FAST=$f KP=$k" >> $O
  MIMIC_JIT_FAST=$f MIMIC_JIT_KP=$k timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident >> $O 2>&1
done; done; done
for v in 65536 131072 524288 1048576; do echo "V=$v" >> $O; timeout -k 10 200 python bench.py --config classifier --vcpus $v --steps 10 --warmup 2 --no-cpu-baseline --no-host-resident >> $O 2>&1; done
timeout -k 10 300 python bench.py --config classifier --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/$TAG/hostres.log 2>&1
python3 - <<'PY'
import json
tag = None
for l in open("gpurun_out/" + __import__("os").environ["TAG"] + "/sweep.log"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l)
        print(tag, d["config"]["workload"][:14], d["config"]["vcpus_per_gpu"], d["value"], d["roofline"]["avg_launch_ms"])
    elif l and not l.startswith("/opt"):
        tag = l
PY
grep -o '"host_resident": {[^}]*}' gpurun_out/$TAG/hostres.log
