#!/bin/bash
# Round 4: cfg 5 with the compact derived-record array (sk_buff GPU tests, bench line, PMC passes),
# then where the cfg-4 inserting launch's time goes: the shared freelist head (measurement
# variants without it, with a same-latency atomic on a per-wave address, without the tail load).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_vc.py tests/test_gpu_skb.py tests/test_gpu_step.py tests/test_gpu_pool.py tests/test_gpu_fastpaths.py tests/test_gpu_bench_size.py -k "not cfg3 and not cfg4" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-resident"
$B --config skb > $O/skb.json 2> $O/skb.err || exit 1
for v in "" MIMIC_MEAS_NOHEAD MIMIC_MEAS_SPREADHEAD MIMIC_MEAS_NOTAIL; do
  MIMIC_JIT_DEFS=$v $B --config flowtrack_insert > $O/ftins_${v:-default}.json 2> $O/ftins_${v:-default}.err || exit 1
done
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'), d['status_ok_frac'])"; done
SQ=0 CFG=skb NAME=skb_compact TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof_r04/r04_pmc_skb_compact.json')); print('skb', d['kernel_stats']['avg_ns'], d.get('read_bytes_per_launch'), d.get('write_size_kib_per_launch'))"
grep -h "mimic_skb_prep_kernel\|mimic_jit_kernel\|mimic_xdp_resume" gpurun_out/prof_r04/r04_kernel_stats_skb_compact.csv
