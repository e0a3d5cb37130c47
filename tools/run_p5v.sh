cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/p5v
export TMPDIR=/tmp
for cfg in "0 262144" "8 524288" "0 524288" "6 393216"; do set -- $cfg
  MIMIC_JIT_WAVES=$1 timeout -k 10 300 python -u bench.py --config parse5 --vcpus $2 --steps 10 --warmup 3 --no-cpu-baseline --no-host-resident > gpurun_out/p5v/b_$1_$2.json 2>> gpurun_out/p5v/err || exit $?
  echo "waves=$1 V=$2 $(python3 -c "import json; d=json.load(open('gpurun_out/p5v/b_$1_$2.json')); print(d['value'], d['roofline']['avg_launch_ms'])")"
done
