cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/vcdbg
for v in 0 1; do
MIMIC_JIT_VC=$v timeout -k 10 200 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider "tests/test_gpu_vc.py::test_lane_value_cache" --maxfail=20 > gpurun_out/vcdbg/vc$v.log 2>&1
echo "vc=$v rc=$?"; grep -E "passed|failed" gpurun_out/vcdbg/vc$v.log | tail -2
done
