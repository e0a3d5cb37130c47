"""JIT tooling around the engine's per-program-set kernels (csrc/jit.cpp), host only.

* ``kernel_source(raws, ctx)`` -- the HIP source the engine generates for a set of loaded
  programs (raw 8-byte slots, in AddProgram order).  It depends only on the instructions and
  the batch context, never on map relocations, so it is also the code-object cache key.
* ``code_object(src)`` / ``kernel_resources(code)`` -- the hipRTC gfx950 code object and the
  register / scratch / LDS usage its AMDGPU metadata note declares (occupancy checks).
* ``prewarm(kernels)`` -- compile many kernels into ``MIMIC_JIT_CACHE`` in parallel worker
  PROCESSES before any device is used (hipRTC serialises compiles inside one process).  The
  workers only load the library and call hipRTC; they never touch a GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import tempfile
from typing import Dict, Iterable, List, Sequence, Tuple

from . import _lib

CTX_XDP, CTX_SKB = 0, 1


def _progs_args(raws: Sequence[bytes]):
    bufs = [C.create_string_buffer(bytes(r), max(len(r), 1)) for r in raws]
    arr = (C.c_void_p * max(len(raws), 1))(*[C.cast(b, C.c_void_p) for b in bufs])
    ns = (C.c_uint32 * max(len(raws), 1))(*[len(r) // 8 for r in raws])
    return bufs, arr, ns


def kernel_source(raws: Sequence[bytes], ctx: int = CTX_XDP, vc: Sequence[Tuple[int, int, int]] = (), spread=None,
                  proc: bool = False) -> str:
    """vc: (program index, slot, E * S) of the LD_IMM64 slots that name a per-CPU array whose
    per-vCPU row is at most 128 bytes, a multiple of 8 -- what a VM with those maps generates (see
    ``vc_slots``).  spread: a ``spread_spec`` -- the VM's spread kernel instead (xdp_md).  proc: the
    single-process form Process.Run tiers up to (MIMIC_PROC_JIT, xdp_md)."""
    if spread is not None:
        return spread_source(raws, *spread)[0]
    lib = _lib.load()
    keep, arr, ns = _progs_args(raws)
    flat = [v for t in vc for v in t]
    vca = (C.c_uint32 * max(len(flat), 1))(*flat)
    kind = ctx | (0x100 if proc else 0)
    n = lib.mimic_jit_source_vc(arr, ns, len(raws), kind, vca, len(vc), None, 0)
    if n < 0:
        raise ValueError(f"cannot decode programs ({n})")
    buf = C.create_string_buffer(n + 1)
    lib.mimic_jit_source_vc(arr, ns, len(raws), kind, vca, len(vc), buf, n + 1)
    return buf.value.decode()


def vc_slots(progs: Sequence[Tuple[bytes, Sequence]], maps: Sequence[dict]) -> List[Tuple[int, int, int]]:
    """The (program index, slot, E * S) triples of kernel_source's ``vc`` for programs (raw,
    relocations [(slot, map name), ...]) loaded next to ``maps`` (name, type, value_size,
    max_entries): the LD_IMM64 slots whose constant is the object of a per-CPU array (type 6)
    whose row E * S is at most 128 bytes and a multiple of 8.  A PseudoMapValue slot names the
    object only when its offset is 0 (Q16: the constant is the object address + offset)."""
    by_name = {m["name"]: m for m in maps}
    out = []
    for pi, (raw, rel) in enumerate(progs):
        for r in rel:
            slot, name = r[0], r[1]
            m = by_name.get(name)
            if m is None or m["type"] != 6:
                continue
            rb = m["max_entries"] * m["value_size"]
            if not (0 < rb <= 128 and rb % 8 == 0):
                continue
            src, off = raw[8 * slot + 1] >> 4, int.from_bytes(raw[8 * slot + 2:8 * slot + 4], "little", signed=True)
            if src == 1 or (src == 2 and off == 0):
                out.append((pi, slot, rb))
    return out


def spread_spec(progs: Sequence[Tuple[bytes, Sequence]], maps: Sequence[dict], vcpus: int, ppb: int = 1024,
                own: bool = False):
    """What the engine's spread_build() generates the spread kernel from, for programs (raw,
    relocations) loaded next to ``maps`` (created in this order: map id = index) on a VM with
    ``vcpus`` vCPUs: (pc, shapes, lds_rows) -- the (program, slot, map id) of every LD_IMM64 slot
    naming a per-CPU array's object, those maps' (id, E * S, S), and the LDS table's rows
    (min(ppb, V) when that many rows of the largest such row fit 32 KiB, else 0).  own: the owned
    form's (spread_build_own: min(256, 32 KiB / row) rows, bit 31 set)."""
    by_name = {m["name"]: (i, m) for i, m in enumerate(maps)}
    pc, shapes = [], {}
    for pi, (raw, rel) in enumerate(progs):
        for r in rel:
            slot, name = r[0], r[1]
            if name not in by_name or by_name[name][1]["type"] != 6:
                continue
            mid, m = by_name[name]
            src, off = raw[8 * slot + 1] >> 4, int.from_bytes(raw[8 * slot + 2:8 * slot + 4], "little", signed=True)
            if src == 1 or (src == 2 and off == 0):
                pc.append((pi, slot, mid))
                shapes[mid] = (mid, m["max_entries"] * m["value_size"], m["value_size"])
    row = max((s[1] for s in shapes.values()), default=0)
    if own:
        return pc, list(shapes.values()), (min(256, 32768 // row) if row else 0) | (1 << 31)
    rows = min(ppb, vcpus)
    return pc, list(shapes.values()), rows if rows * row <= 32768 else 0


def spread_source(raws: Sequence[bytes], pc, shapes, lds_rows: int) -> Tuple[str, bool]:
    """(source, allowed): the spread kernel's source and whether the programs allow one (else the
    source is the plain kernel's).  jit.cpp analyze_spread decides."""
    lib = _lib.load()
    keep, arr, ns = _progs_args(raws)
    pcf = [v for t in pc for v in t]
    shf = [v for t in shapes for v in t]
    pca = (C.c_uint32 * max(len(pcf), 1))(*pcf)
    sha = (C.c_uint32 * max(len(shf), 1))(*shf)
    ok = C.c_int32()
    n = lib.mimic_jit_source_spread(arr, ns, len(raws), pca, len(pc), sha, len(shapes), lds_rows, C.byref(ok), None, 0)
    if n < 0:
        raise ValueError(f"cannot decode programs ({n})")
    buf = C.create_string_buffer(n + 1)
    lib.mimic_jit_source_spread(arr, ns, len(raws), pca, len(pc), sha, len(shapes), lds_rows, C.byref(ok), buf, n + 1)
    return buf.value.decode(), bool(ok.value)


def code_object(src: str) -> bytes:
    lib = _lib.load()
    size = C.c_size_t()
    if lib.mimic_jit_code(src.encode(), None, 0, C.byref(size)) != 0:
        raise RuntimeError("hipRTC compile failed")
    buf = C.create_string_buffer(size.value)
    lib.mimic_jit_code(src.encode(), buf, size.value, C.byref(size))
    return buf.raw[:size.value]


def _notes(elf: bytes):
    """(name, type, desc) of every note in the ELF's SHT_NOTE sections (64-bit little endian)."""
    import struct

    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for i in range(shnum):
        sh = shoff + i * shentsize
        stype, = struct.unpack_from("<I", elf, sh + 4)
        if stype != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            nsz, dsz, typ = struct.unpack_from("<III", elf, p)
            name = elf[p + 12:p + 12 + nsz].rstrip(b"\0").decode()
            d0 = p + 12 + ((nsz + 3) & ~3)
            yield name, typ, elf[d0:d0 + dsz]
            p = d0 + ((dsz + 3) & ~3)


def kernel_resources(code: bytes, kernel: str = "mimic_jit_kernel") -> Dict[str, int]:
    """VGPR / AGPR / SGPR counts, spills, scratch and LDS bytes of a kernel, and the waves per
    SIMD its registers allow on gfx950 (512 unified VGPRs per SIMD lane, granule 8, max 8)."""
    import msgpack

    for name, typ, desc in _notes(code):
        if name != "AMDGPU" or typ != 32:  # NT_AMDGPU_METADATA
            continue
        md = msgpack.unpackb(desc, raw=False)
        for k in md.get("amdhsa.kernels", []):
            if k.get(".name") != kernel:
                continue
            # gfx950: .vgpr_count is the unified total (arch VGPRs, aligned, + AGPRs)
            total, a = int(k.get(".vgpr_count", 0)), int(k.get(".agpr_count", 0))
            alloc = max(8, (total + 7) & ~7)
            return {"vgpr": total - a, "agpr": a, "vgpr_total": total, "sgpr": int(k.get(".sgpr_count", 0)),
                    "vgpr_spill": int(k.get(".vgpr_spill_count", 0)), "sgpr_spill": int(k.get(".sgpr_spill_count", 0)),
                    "scratch": int(k.get(".private_segment_fixed_size", 0)),
                    "lds": int(k.get(".group_segment_fixed_size", 0)), "waves_per_simd": min(8, 512 // alloc)}
    raise KeyError(f"kernel {kernel} not in the code object's metadata")


def _cache_dir() -> str:
    d = os.environ.get("MIMIC_JIT_CACHE", "")
    if not d:
        raise RuntimeError("MIMIC_JIT_CACHE is not set: prewarming needs an on-disk kernel cache")
    os.makedirs(d, exist_ok=True)
    return d


def _no_early_load_source(k) -> str:
    """The form of kernel k the engine falls back to when its 4-wave build spills (engine.cpp:
    the kernel without early packet loads, MIMIC_JIT_SPEC=0)."""
    old = os.environ.get("MIMIC_JIT_SPEC")
    os.environ["MIMIC_JIT_SPEC"] = "0"
    try:
        return kernel_source(list(k[0]), *k[1:])
    finally:
        if old is None:
            del os.environ["MIMIC_JIT_SPEC"]
        else:
            os.environ["MIMIC_JIT_SPEC"] = old


def prewarm(kernels: Iterable[Tuple], workers: int = 0) -> Dict[str, float]:
    """Compile the kernels of (raws, ctx[, vc]) program sets into MIMIC_JIT_CACHE using `workers`
    parallel processes (0: min(16, cpus) - 1), then, for those whose 4-wave build spills, the
    form without early loads the engine will also try.  Returns {"kernels": n, "seconds": t}."""
    import time

    t0 = time.time()
    _cache_dir()
    kernels = list(kernels)
    srcs: Dict[str, Tuple] = {}
    for k in kernels:
        srcs.setdefault(kernel_source(list(k[0]), *k[1:]), k)
    info = _compile_parallel(list(srcs), workers)
    alt: Dict[str, None] = {}
    for src, k in srcs.items():
        if "issued early" in src and "amdgpu_waves_per_eu(4)" in src:
            try:
                if kernel_resources(code_object(src))["scratch"] > 0:
                    alt[_no_early_load_source(k)] = None
            except RuntimeError:
                pass
    info2 = _compile_parallel(list(alt), workers)
    return {"kernels": len(srcs) + len(alt), "seconds": time.time() - t0,
            "worker_failures": info["worker_failures"] + info2["worker_failures"],
            "failed_after_retry": info["failed_after_retry"] + info2["failed_after_retry"]}


def _compile_parallel(srcs, workers: int) -> Dict[str, int]:
    todo = sorted(srcs, key=len, reverse=True)        # longest first: better packing
    if not todo:
        return {"worker_failures": 0, "failed_after_retry": 0}
    if workers <= 0:
        workers = max(1, min(16, os.cpu_count() or 1) - 1)
    workers = min(workers, len(todo))
    with tempfile.TemporaryDirectory(prefix="mimic_jitwarm_") as tmp:
        lists = [[] for _ in range(workers)]
        for k, s in enumerate(todo):                  # round-robin over the sorted list
            path = os.path.join(tmp, f"k{k}.hip")
            with open(path, "w") as f:
                f.write(s)
            lists[k % workers].append(path)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

        def launch(w):
            env = dict(os.environ)
            env["TMPDIR"] = os.path.join(tmp, f"t{w}")    # compiler temp files: one directory per worker
            os.makedirs(env["TMPDIR"], exist_ok=True)
            return subprocess.Popen([sys.executable, "-m", "mimic_amd.jit", os.path.join(tmp, f"w{w}.txt")],
                                    env=env, cwd=root)

        for w, paths in enumerate(lists):
            with open(os.path.join(tmp, f"w{w}.txt"), "w") as f:
                f.write("\n".join(paths))
        rcs = [p.wait() for p in [launch(w) for w in range(workers)]]
        # a worker that died retries its list once (finished kernels are cache hits); kernels still
        # missing after that are compiled by the engine when first used
        retry = [w for w, rc in enumerate(rcs) if rc]
        rcs2 = [p.wait() for p in [launch(w) for w in retry]]
    return {"worker_failures": len(retry), "failed_after_retry": sum(1 for rc in rcs2 if rc)}


def _worker(list_file: str) -> int:
    lib = _lib.load()
    rc = 0
    with open(list_file) as f:
        for path in f.read().split():
            with open(path) as g:
                if lib.mimic_jit_cache_source(g.read().encode()) != 0:
                    print(f"mimic_amd.jit: compile failed: {path}", file=sys.stderr)
                    rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(_worker(sys.argv[1]))
