cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/p5k; mkdir -p $D
for k in X=1 MIMIC_JIT_INCAGENT=1 MIMIC_JIT_INC=0; do
  env $k timeout -k 10 300 python -u bench.py --config parse5 --no-host-resident --no-cpu-baseline > $D/$k.json 2> $D/$k.err || { tail -5 $D/$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$k.json')); print('$k', d['value'], d['roofline']['avg_launch_ms'])"
done
