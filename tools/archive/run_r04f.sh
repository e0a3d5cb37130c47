#!/bin/bash
# Round 4: pop-only hash changes (lookups without the re-read, identity ring, no probe before the
# insert walk): hash / shard / cfg-4 bench-size tests, cfg-4 lines (lookup-hit, inserting, the
# inserting launch without the shared head counter as a measurement), the inserting launch's
# PMC passes, then the cfg-5 traffic attribution (tools/run_r04e.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_hash.py tests/test_gpu_shard.py tests/test_gpu_bench_size.py -k "not cfg3 and not cfg5" -s > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-resident"
$B --config flowtrack > $O/ft.json 2> $O/ft.err || exit 1
$B --config flowtrack_insert > $O/ftins.json 2> $O/ftins.err || exit 1
MIMIC_JIT_DEFS=MIMIC_MEAS_NOHEAD $B --config flowtrack_insert > $O/ftins_nohead.json 2> $O/ftins_nohead.err || exit 1
for f in $O/*.json; do echo "== $f"; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('hash_keys'))"; done
CFG=flowtrack_insert TAG=r04 timeout -k 10 900 bash tools/profile.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/prof_r04/r04_pmc_flowtrack_insert.json')); s=d['sq_per_wave']; print('ftins', d['kernel_stats']['avg_ns'], 'wait', s['SQ_WAIT_ANY']/s['SQ_WAVE_CYCLES'], d.get('bytes_per_launch'))"
bash tools/run_r04e.sh
