"""Compile the JIT kernels of the bench / smoke workloads into .jitcache on a CPU host (hipRTC
needs no GPU), so a fresh GPU box loads them instead of compiling.  The test suite's kernels:
MIMIC_JIT_PREWARM=1 python -m pytest tests -m gpu -n 8 -q"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
os.makedirs(os.environ["MIMIC_JIT_CACHE"], exist_ok=True)

from mimic_amd import _lib, workloads as W  # noqa: E402


def prebuild(raws):
    lib = _lib.load()
    bufs = [C.create_string_buffer(bytes(r), max(len(r), 1)) for r in raws]
    arr = (C.c_void_p * len(raws))(*[C.cast(b, C.c_void_p) for b in bufs])
    ns = (C.c_uint32 * len(raws))(*[len(r) // 8 for r in raws])
    return lib.mimic_jit_prebuild(arr, ns, len(raws))


if __name__ == "__main__":
    for fn in ("prog_pass8", "prog_classifier", "prog_parse5", "prog_flowtrack", "prog_flowcount"):
        p = getattr(W, fn)()
        print(fn, "rc", prebuild([p.raw]))
