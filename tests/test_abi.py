"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every entry point the
header declares, and the status numbering matches the oracle's (no compute calls here)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mimic_amd.h")
ORC_HDR = os.path.join(ROOT, "oracle", "mimic_oracle.h")


def _decls():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|long|void|const char \*)\s*(mimic_\w+)\s*\(", txt, re.M)))


def _enum(path, prefix):
    txt = open(path).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(prefix + r"(\w+)\s*=\s*(\d+)", txt)}


def test_library_exports_every_declared_symbol():
    from mimic_amd import _lib

    lib = _lib.load()  # loads without a GPU
    decls = _decls()
    assert len(decls) >= 18
    for name in decls:
        assert hasattr(lib, name), f"{name} declared in include/mimic_amd.h but not exported"
    assert set(decls) == set(_lib.EXPORTS), "ctypes binding and header disagree"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (mimic_\w+)", out))
    assert set(decls) <= exported


def test_abi_version():
    from mimic_amd import _lib

    assert _lib.load().mimic_abi_version() == _lib.ABI_VERSION
    hdr = int(re.search(r"#define MIMIC_ABI_VERSION (\d+)", open(HDR).read()).group(1))
    # 2: mimic_skb_batch grew `custom`, statuses 29/30, mimic_last_exec may return MIMIC_EXEC_SPREAD
    # 3: mimic_last_exec may return MIMIC_EXEC_SPREAD_OWN
    assert hdr == _lib.ABI_VERSION == 4


def test_status_numbering_matches_oracle():
    prod = _enum(HDR, r"MIMIC_(?!ABI)")
    orc = _enum(ORC_HDR, r"ORC_(?!MAP)")
    names = [n for n in orc if n not in ("STATUS_COUNT",)]
    for n in names:
        assert prod.get(n) == orc[n], n
    from mimic_amd import _lib

    for n, v in orc.items():
        if n in _lib.STATUS:
            assert _lib.STATUS[n] == v


def test_vm_create_rejects_bad_settings_without_gpu():
    from mimic_amd import _lib

    lib = _lib.load()
    s = _lib.VMSettings(0, 256, 8, 33, 0, 0, 0, 0)
    h = ctypes.c_void_p()
    assert lib.mimic_vm_create(ctypes.byref(s), ctypes.byref(h)) < 0
