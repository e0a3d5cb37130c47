"""Compile the JIT kernels of the bench / smoke workloads into MIMIC_JIT_CACHE (default
.jitcache) on a CPU host -- hipRTC needs no GPU -- with parallel worker processes
(mimic_amd.jit.prewarm), so a fresh GPU box loads them instead of compiling.  The GPU test suite
prewarms its own kernels the same way (tests/conftest.py)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
os.makedirs(os.environ["MIMIC_JIT_CACHE"], exist_ok=True)

from mimic_amd import _lib, jit as J, workloads as W  # noqa: E402

if __name__ == "__main__":
    kernels = []
    for fn in ("prog_pass8", "prog_classifier", "prog_parse5", "prog_flowtrack", "prog_flowcount"):
        p = getattr(W, fn)()
        kernels.append(([p.raw], _lib.CTX_XDP, J.vc_slots([(p.raw, p.relocs)], p.maps)))
    t0 = time.time()
    out = J.prewarm(kernels)
    print(f"{len(kernels)} kernels in {time.time() - t0:.1f} s", out)
