#!/bin/bash
# round 5: pool tests, then PMC profiles of the cfg-5 chain with the next-offset prefetch (SKBTOUCH=2) and without (=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05f
timeout -k 10 500 python -u -m pytest tests/test_gpu_pool.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05f/pool.log 2>&1; tail -3 gpurun_out/r05f/pool.log
for v in 2 0; do
  MIMIC_JIT_SKBTOUCH=$v CFG=skb NAME=skb_touch$v TAG=r05f timeout -k 10 600 bash tools/profile.sh || { echo "profile $v failed"; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/prof_r05f/r05f_pmc_skb_touch$v.json'))
print('$v', d['kernel_stats']['avg_ns'], d['read_bytes_per_launch'], d['write_size_kib_per_launch'], d['sq_per_wave'], d['valu_busy'])"
done
