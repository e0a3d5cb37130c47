"""Register budget of the batch interpreter's kernels as built into libmimic_amd.so (no device): the
code objects are read from the library's `.hip_fatbin` section (clang offload bundles) and their
AMDGPU metadata gives VGPRs, spills and scratch per kernel."""
import os
import struct

import pytest

from mimic_amd import _lib
from mimic_amd import jit as J

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    d = open(path, "rb").read()
    assert d[:4] == b"\x7fELF" and d[4] == 2, "ELF64 expected"
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    hdr = [struct.unpack_from("<IIQQQQIIQQ", d, shoff + k * shentsize) for k in range(shnum)]
    stro = hdr[shstrndx][4]
    for h in hdr:
        nm = d[stro + h[0]:d.index(b"\0", stro + h[0])].decode()
        if nm == name:
            return d[h[4]:h[4] + h[5]]
    raise KeyError(name)


def _code_objects(path):
    fb = _section(path, ".hip_fatbin")
    out = []
    i = fb.find(MAGIC)
    while i >= 0:
        n, = struct.unpack_from("<Q", fb, i + 24)
        p = i + 32
        for _ in range(n):
            o, s, tl = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tl]
            p += 24 + tl
            if s and b"gfx950" in triple:
                out.append(fb[i + o:i + o + s])
        i = fb.find(MAGIC, i + 1)
    return out


def _kernel(name):
    path = _lib.LIB_PATH
    if not os.path.exists(path):
        pytest.skip("libmimic_amd.so not built")
    for co in _code_objects(path):
        try:
            return J.kernel_resources(co, name)
        except KeyError:
            continue
    raise KeyError(name)


def test_batch_interpreter_spills_at_most_16_vgprs():
    """The batch kernel keeps its 4-wave budget (128 VGPRs).  SKBuffFromBytes is compiled out of it
    (the engine launches it only after a full prep, skb_load<false>): 70 spilled VGPRs / 144 B of
    scratch with it inlined, 16 / 64 B without."""
    r = _kernel("mimic_xdp_kernel")
    assert r["vgpr_total"] <= 128 and r["waves_per_simd"] >= 4, r
    assert r["vgpr_spill"] <= 16 and r["scratch"] <= 64, r


def test_resume_and_step_kernels_do_not_spill():
    for k in ("mimic_xdp_resume_kernel", "mimic_xdp_step_kernel"):
        r = _kernel(k)
        assert r["vgpr_spill"] == 0 and r["scratch"] == 0 and r["agpr"] == 0, (k, r)
