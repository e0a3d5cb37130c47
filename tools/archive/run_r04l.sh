#!/bin/bash
# Round 4: the batch interpreter with its map-writing helpers out of line (interp.hip
# INTERP_UPDATE / INTERP_DELETE) vs inlined (libmimic_amd_inlmaps.so, -DMIMIC_INTERP_INLINE_MAPS):
# interpreter KATs / hash / step tests, then interpreter bench lines (cfg 2, cfg 4 inserting, cfg 5).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kat.py tests/test_gpu_hash.py tests/test_gpu_step.py tests/test_gpu_vc.py -k "interp or hash or step or lds_row" > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
B="timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-resident --steps 10 --warmup 2"
for lib in libmimic_amd.so libmimic_amd_inlmaps.so; do
  for c in classifier flowtrack_insert skb; do
    MIMIC_LIB=$lib MIMIC_EXEC=interp $B --config $c > $O/${c}_$lib.json 2> $O/${c}_$lib.err || exit 1
  done
done
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['engine'])"; done
