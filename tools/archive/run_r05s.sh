#!/bin/bash
# round 5: owned spread launches (MIMIC_SPREAD_OWN=1): parity tests, then cfg 2 / cfg 3 / cfg 1-shape against the one-lane kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r05s
mkdir -p $D
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_spread_own.py tests/test_gpu_spread.py} -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/test.log 2>&1 || { tail -40 $D/test.log; exit 1; }
tail -2 $D/test.log
for c in ${CFGS:-classifier parse5 pass8}; do
  for k in 1 2; do
    for o in 0 1; do
      MIMIC_SPREAD_OWN=$o timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-host-resident --no-cpu-baseline > $D/${c}_own${o}_$k.json 2> $D/${c}_own${o}_$k.err || { tail -5 $D/${c}_own${o}_$k.err; exit 1; }
      python3 -c "import json; d=json.load(open('$D/${c}_own${o}_$k.json')); print('$c own=$o', d['value'], d['ms_per_step'], d.get('last_exec', d['config'].get('engine')))"
    done
  done
done
