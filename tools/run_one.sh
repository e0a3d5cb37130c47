#!/bin/bash
# one GPU test selection: TESTS="tests/x.py::y ..." bash tools/run_one.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/one
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/one/tests.log 2>&1
rc=$?; tail -15 gpurun_out/one/tests.log; exit $rc
