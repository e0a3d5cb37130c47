"""Generate the source of every JIT kernel the GPU test suite compiles (each test module's
jit_kernels(), as the session prewarm collects them) through the library's host-only entry points
(mimic_jit_source_vc / mimic_jit_source_spread).  Run by tools/run_asan.sh with the sanitizer build
of the library (MIMIC_LIB=libmimic_amd_asan.so): ASan / UBSan abort on the first error."""
import glob
import hashlib
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from mimic_amd import _lib, jit as J  # noqa: E402


def main():
    assert os.path.basename(_lib.LIB_PATH) == os.environ.get("MIMIC_LIB", ""), _lib.LIB_PATH
    kernels = []
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "test_gpu_*.py"))):
        mod = importlib.import_module(os.path.basename(f)[:-3])
        fn = getattr(mod, "jit_kernels", None)
        if fn is not None:
            kernels.extend(fn())
    seen = set()
    nbytes = 0
    for k in kernels:
        src = J.kernel_source(*k)
        seen.add(hashlib.sha256(src.encode()).hexdigest())
        nbytes += len(src)
    print(f"asan_jit_sources: {len(kernels)} kernels ({len(seen)} distinct sources, {nbytes} bytes) generated "
          f"with {_lib.LIB_PATH}: no sanitizer error")


if __name__ == "__main__":
    main()
