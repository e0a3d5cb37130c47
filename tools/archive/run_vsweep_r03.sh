cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/sweep3; mkdir -p $D
for v in 65536 131072 262144 524288; do
  timeout -k 10 300 python -u bench.py --config parse5 --vcpus $v --no-host-resident --no-cpu-baseline > $D/p5_$v.json 2> $D/p5_$v.err || { tail -5 $D/p5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/p5_$v.json')); r=d['roofline']; print('parse5 V=$v', d['value'], d['ms_per_step'], r['avg_launch_ms'])"
done
for v in 131072 196608 262144; do
  timeout -k 10 300 python -u bench.py --config skb --vcpus $v --no-host-resident --no-cpu-baseline > $D/skb_$v.json 2> $D/skb_$v.err || { tail -5 $D/skb_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/skb_$v.json')); r=d['roofline']; print('skb V=$v', d['value'], d['ms_per_step'], r['avg_launch_ms'])"
done
