#!/usr/bin/env python3
"""Writes tests/golden/xdp_count.o: a small eBPF ELF object in the layout clang emits for
`clang -target bpf -O2 -c` (this image has no BPF backend, so the object is assembled here).

    SEC("xdp")       int xdp_count(struct xdp_md *ctx)   calls add3 (global, .text) and twice
                                                          (static, .text, called through the
                                                          .text section symbol), reads the
                                                          first packet byte, counts into the
                                                          per-CPU array `counters`, adds the
                                                          .data variable `gvar`
    SEC("xdp/pass")  int xdp_pass(...)                   return XDP_PASS
    .text            add3(x) = x + 3 (via the stack), twice(x) = 2x
    maps             counters: percpu_array K4 V8 E4;  flows: hash K4 V8 E64 (bpf_map_def)
    .data            u64 pad, u64 gvar = 0x1122334455667788

Relocations (.relxdp): R_BPF_64_32 on the two calls (function symbol / section symbol), and
R_BPF_64_64 on the two LD_IMM64 (map symbol / .data object).  `expected_linked()` is the same
program written as raw slots the way cilium/ebpf + VM.AddProgram would hand it to the engine.
"""
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mimic_amd import asm as A  # noqa: E402

OUT = os.path.join(HERE, "xdp_count.o")
OUT_BTF = os.path.join(HERE, "xdp_count_btf.o")


def main_items(call_add3, call_twice, ld_counters, ld_gvar):
    return [
        A.mov64_reg(6, 1),
        A.mov64_imm(1, 7),
        call_add3,                                  # r0 = 10
        A.mov64_reg(7, 0),
        A.mov64_reg(1, 7),
        call_twice,                                 # r0 = 20
        A.mov64_reg(7, 0),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 1),
        A.jmp("jgt", 4, 3, "skip", reg=True),
        A.ldx(1, 5, 2, 0),
        A.alu64("add", 7, 5, reg=True),
        "skip",
        A.st(4, 10, -4, 1),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -4),
        ld_counters,
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "nomap"),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 7, reg=True),
        A.stx(8, 0, 0, 1),
        "nomap",
        ld_gvar,
        A.ldx(8, 0, 1, 8),
        A.alu64("add", 0, 7, reg=True),
        A.exit_(),
    ]


TEXT = [A.stx(8, 10, -8, 1), A.ldx(8, 0, 10, -8), A.alu64("add", 0, 3), A.exit_(),      # add3 at slot 0
        A.mov64_reg(0, 1), A.alu64("mul", 0, 2), A.exit_()]                               # twice at slot 4


def expected_linked():
    """(raw slots, [(slot, map)]) of xdp_count after linking: main, add3, twice."""
    items = main_items(A.call_local("add3"), A.call_local("twice"), A.ld_map_fd(1, "counters"),
                       A.ld_map_value(1, ".data")) + ["add3"] + TEXT[:4] + ["twice"] + TEXT[4:]
    raw, rel = A.assemble(items)
    raw = bytearray(raw)
    for slot, name in rel:                 # cilium: the data-section variable's offset (8) in the 2nd slot
        if name == ".data":
            struct.pack_into("<I", raw, 8 * slot + 12, 8)
    return bytes(raw), rel


def btf_section(maps_var_names=("counters", "flows")) -> bytes:
    """The .BTF section clang writes for

        struct { __uint(type, BPF_MAP_TYPE_PERCPU_ARRAY); __uint(max_entries, 4);
                 __type(key, __u32); __type(value, __u64); } counters SEC(".maps");
        struct { __uint(type, BPF_MAP_TYPE_HASH); __uint(max_entries, 64);
                 __uint(key_size, 4); __uint(value_size, 8); } flows SEC(".maps");

    (libbpf's bpf_helpers.h: __uint(name, val) is `int (*name)[val]`, __type(name, val) is
    `typeof(val) *name`); types follow linux/btf.h."""
    strs = bytearray(b"\0")

    def sname(n):
        if not n:
            return 0
        o = len(strs)
        strs.extend(n.encode() + b"\0")
        return o

    types = []

    def add(kind, name, st, extra=b"", vlen=0):
        types.append(struct.pack("<III", sname(name), (kind << 24) | vlen, st) + extra)
        return len(types)

    t_int = add(1, "int", 4, struct.pack("<I", (1 << 24) | 32))            # INT signed 32

    def uint_attr(n):   # int (*)[n]
        arr = add(3, "", 0, struct.pack("<III", t_int, t_int, n))
        return add(2, "", arr)

    t_u32 = add(1, "unsigned int", 4, struct.pack("<I", 32))
    t_u32td = add(8, "__u32", t_u32)                                         # TYPEDEF
    t_u64 = add(1, "unsigned long long", 8, struct.pack("<I", 64))
    t_u64td = add(8, "__u64", t_u64)
    # counters
    a_type, a_max = uint_attr(6), uint_attr(4)
    p_key, p_val = add(2, "", t_u32td), add(2, "", t_u64td)
    mem = b"".join(struct.pack("<III", sname(n), t, 64 * k)
                   for k, (n, t) in enumerate([("type", a_type), ("max_entries", a_max), ("key", p_key),
                                               ("value", p_val)]))
    s_counters = add(4, "", 32, mem, vlen=4)
    v_counters = add(14, maps_var_names[0], s_counters, struct.pack("<I", 1))
    # flows
    b_type, b_max, b_ks, b_vs = uint_attr(1), uint_attr(64), uint_attr(4), uint_attr(8)
    mem = b"".join(struct.pack("<III", sname(n), t, 64 * k)
                   for k, (n, t) in enumerate([("type", b_type), ("max_entries", b_max), ("key_size", b_ks),
                                               ("value_size", b_vs)]))
    s_flows = add(4, "", 32, mem, vlen=4)
    v_flows = add(14, maps_var_names[1], s_flows, struct.pack("<I", 1))
    secinfo = struct.pack("<III", v_counters, 0, 32) + struct.pack("<III", v_flows, 32, 32)
    add(15, ".maps", 64, secinfo, vlen=2)
    tb = b"".join(types)
    hdr = struct.pack("<HBBIIIII", 0xEB9F, 1, 0, 24, 0, len(tb), len(tb), len(strs))
    return hdr + tb + bytes(strs)


def build(btf: bool = False) -> bytes:
    # the ELF sections' raw bytes: calls with imm -1 / section offsets, LD_IMM64 with src 0
    main, _ = A.assemble(main_items(A.raw(0x85, 0, 1, 0, -1), A.raw(0x85, 0, 1, 0, 3), A.ld_imm64(1, 0),
                                    A.ld_imm64(1, 0)))
    text, _ = A.assemble(TEXT)
    slots = [main[i:i + 8] for i in range(0, len(main), 8)]
    call_slots = [i for i, s in enumerate(slots) if s[0] == 0x85 and (s[1] >> 4) == 1]
    ld_slots = [i for i, s in enumerate(slots) if s[0] == 0x18]
    xdp_pass, _ = A.assemble([A.mov64_imm(0, A.XDP_PASS), A.exit_()])
    if btf:   # BTF-defined maps: the .maps section holds the (zeroed) pointer structs
        maps = bytes(64)
        map_sec = ".maps"
    else:
        maps = struct.pack("<5I", 6, 4, 8, 4, 0) + struct.pack("<5I", 1, 4, 8, 64, 0)
        map_sec = "maps"
    data = struct.pack("<QQ", 0, 0x1122334455667788)

    shnames = ["", ".text", "xdp", "xdp/pass", map_sec, ".data", ".relxdp", ".symtab", ".strtab", ".shstrtab"]
    if btf:
        shnames.append(".BTF")
    shstr = b"\0".join(n.encode() for n in shnames) + b"\0"
    shoff = {n: shstr.index(n.encode() + b"\0") if n else 0 for n in shnames}
    shoff[".text"] = shstr.index(b".text\0")
    shoff["xdp"] = shstr.index(b"\0xdp\0") + 1
    shoff[map_sec] = shstr.index(b"\0" + map_sec.encode() + b"\0") + 1
    # symbols: locals first (null, .text section, twice), then globals
    strtab = b"\0"
    syms = []

    def sym(name, value, size, typ, bind, shndx):
        nonlocal strtab
        o = 0
        if name:
            o = len(strtab)
            strtab += name.encode() + b"\0"
        syms.append(struct.pack("<IBBHQQ", o, (bind << 4) | typ, 0, shndx, value, size))

    sym("", 0, 0, 0, 0, 0)
    sym("", 0, 0, 3, 0, 1)                 # STT_SECTION .text
    sym("twice", 32, 24, 2, 0, 1)          # local function
    nlocal = len(syms)
    sym("add3", 0, 32, 2, 1, 1)
    sym("xdp_count", 0, len(main), 2, 1, 2)
    sym("xdp_pass", 0, len(xdp_pass), 2, 1, 3)
    msz = 32 if btf else 20
    sym("counters", 0, msz, 1, 1, 4)
    sym("flows", msz, msz, 1, 1, 4)
    sym("gvar", 8, 8, 1, 1, 5)
    symtab = b"".join(syms)
    rel = b""
    for slot, (si, typ) in zip(call_slots, [(3, 10), (1, 10)]):       # add3 / .text section symbol
        rel += struct.pack("<QQ", 8 * slot, (si << 32) | typ)
    for slot, si in zip(ld_slots, [6, 8]):                            # counters / gvar
        rel += struct.pack("<QQ", 8 * slot, (si << 32) | 1)

    bodies = [b"", text, main, xdp_pass, maps, data, rel, symtab, strtab, shstr]
    if btf:
        bodies.append(btf_section())
    out = bytearray(64)
    offs = []
    for b in bodies:
        while len(out) % 8:
            out += b"\0"
        offs.append(len(out))
        out += b
    while len(out) % 8:
        out += b"\0"
    e_shoff = len(out)
    # (name, type, flags, link, info, align, entsize)
    meta = [(0, 0, 0, 0, 0, 0, 0), (shoff[".text"], 1, 6, 0, 0, 8, 0), (shoff["xdp"], 1, 6, 0, 0, 8, 0),
            (shoff["xdp/pass"], 1, 6, 0, 0, 8, 0), (shoff[map_sec], 1, 3, 0, 0, 4, 0),
            (shoff[".data"], 1, 3, 0, 0, 8, 0), (shoff[".relxdp"], 9, 0, 7, 2, 8, 16),
            (shoff[".symtab"], 2, 0, 8, nlocal, 8, 24), (shoff[".strtab"], 3, 0, 0, 0, 1, 0),
            (shoff[".shstrtab"], 3, 0, 0, 0, 1, 0)]
    if btf:
        meta.append((shoff[".BTF"], 1, 0, 0, 0, 4, 0))
    for (nm, typ, flags, link, info, align, ent), off, b in zip(meta, offs, bodies):
        out += struct.pack("<IIQQQQIIQQ", nm, typ, flags, 0, off if typ else 0, len(b), link, info, align, ent)
    hdr = b"\x7fELF" + bytes([2, 1, 1, 0]) + bytes(8)
    hdr += struct.pack("<HHIQQQIHHHHHH", 1, 247, 1, 0, 0, e_shoff, 0, 64, 0, 0, 64, len(meta), 9)   # .shstrtab
    out[:64] = hdr
    return bytes(out)


if __name__ == "__main__":
    for path, btf in ((OUT, False), (OUT_BTF, True)):
        data = build(btf)
        with open(path, "wb") as f:
            f.write(data)
        print(f"wrote {path} ({len(data)} bytes)")
