#!/bin/bash
# Sanitizer runs on the CPU (host code only; GPU sanitizers are not available on this pool).
#   1. the C oracle built with gcc -fsanitize=address,undefined (make -C oracle asan), gcc's libasan
#      preloaded into pytest: the oracle golden / KAT suites, the sk_buff oracle tests and the cfg-4
#      gloo world-size-2 test (every parity verdict rests on this code);
#   2. the engine library built with host-side ASan + UBSan (hipcc -Xarch_host -fsanitize=...,
#      device code unchanged), clang's ASan runtime preloaded: the JIT generator's host-only entry
#      points (mimic_jit_source_*), over every kernel the GPU suite compiles plus the CPU JIT tests.
# Output: profiles/<tag>_asan.log (pass a tag; default r05).
set -euo pipefail
cd "$(dirname "$0")/.."
TAG=${1:-r05}
LOG=profiles/${TAG}_asan.log
make -C oracle asan -s
if [ ! -f mimic_amd/libmimic_amd_asan.so ] || [ -n "$(find mimic_amd/csrc include -newer mimic_amd/libmimic_amd_asan.so -type f)" ]; then
  python -c "import __graft_entry__ as g; g.write_jit_headers()"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -fPIC -shared -std=c++17 -Wno-unused-value -Wno-unused-result \
    -fno-omit-frame-pointer -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -shared-libsan \
    -o mimic_amd/libmimic_amd_asan.so mimic_amd/csrc/engine.cpp mimic_amd/csrc/jit.cpp mimic_amd/csrc/interp.hip \
    mimic_amd/csrc/skb.hip -lhiprtc
fi
GCC_ASAN=$(gcc -print-file-name=libasan.so)
CLANG_ASAN=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
{
  echo "# $(date -u +%FT%TZ) $(git rev-parse --short HEAD) -- tools/run_asan.sh"
  echo "instrumented: oracle/_asan/liboracle.so $(nm -D oracle/_asan/liboracle.so | grep -c ' U __asan_report') ASan report imports, $(nm -D oracle/_asan/liboracle.so | grep -c ' U __ubsan_handle') UBSan handler imports"
  echo "instrumented: mimic_amd/libmimic_amd_asan.so $(nm -D mimic_amd/libmimic_amd_asan.so | grep -c ' U __asan_report') ASan report imports, $(nm -D mimic_amd/libmimic_amd_asan.so | grep -c ' U __ubsan_handle') UBSan handler imports"
  echo "## 1. oracle (gcc $(gcc -dumpversion), -fsanitize=address,undefined), $GCC_ASAN preloaded"
  LD_PRELOAD=$GCC_ASAN MIMIC_ORACLE_LIB=$PWD/oracle/_asan/liboracle.so python -c "import oracle.pyoracle as o; o.load(); print('oracle loaded from', o.LIB_PATH)" 2>&1
  LD_PRELOAD=$GCC_ASAN MIMIC_ORACLE_LIB=$PWD/oracle/_asan/liboracle.so \
    python -m pytest -q -p no:cacheprovider tests/test_oracle_golden.py tests/test_skb_oracle.py \
    "tests/test_dist.py::test_cfg4_bench_size_shards_merge_to_one_oracle_run" tests/test_ctx.py -m "not gpu" 2>&1
  echo "## 2. engine library host code (hipcc -Xarch_host -fsanitize=address,undefined), $CLANG_ASAN preloaded"
  LD_PRELOAD=$CLANG_ASAN MIMIC_LIB=libmimic_amd_asan.so \
    python -m pytest -q -p no:cacheprovider tests/test_jit_cpu.py tests/test_spread_cpu.py tests/test_abi.py -m "not gpu" 2>&1
  LD_PRELOAD=$CLANG_ASAN MIMIC_LIB=libmimic_amd_asan.so python tools/asan_jit_sources.py 2>&1
} | tee "$LOG"
