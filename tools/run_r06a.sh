#!/bin/bash
# Round 6: the driver's tiers with the one-sync Process.Run, then the reference-shaped API rates.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TAG=${TAG:-r06a}
bash tools/run_driver.sh || exit $?
timeout -k 10 400 python -u tools/api_rates.py > gpurun_out/$TAG/api_rates.json 2> gpurun_out/$TAG/api_rates.err || { tail -30 gpurun_out/$TAG/api_rates.err; exit 1; }
cat gpurun_out/$TAG/api_rates.json
