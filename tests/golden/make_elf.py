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


def build() -> bytes:
    # the ELF sections' raw bytes: calls with imm -1 / section offsets, LD_IMM64 with src 0
    main, _ = A.assemble(main_items(A.raw(0x85, 0, 1, 0, -1), A.raw(0x85, 0, 1, 0, 3), A.ld_imm64(1, 0),
                                    A.ld_imm64(1, 0)))
    text, _ = A.assemble(TEXT)
    slots = [main[i:i + 8] for i in range(0, len(main), 8)]
    call_slots = [i for i, s in enumerate(slots) if s[0] == 0x85 and (s[1] >> 4) == 1]
    ld_slots = [i for i, s in enumerate(slots) if s[0] == 0x18]
    xdp_pass, _ = A.assemble([A.mov64_imm(0, A.XDP_PASS), A.exit_()])
    maps = struct.pack("<5I", 6, 4, 8, 4, 0) + struct.pack("<5I", 1, 4, 8, 64, 0)
    data = struct.pack("<QQ", 0, 0x1122334455667788)

    shnames = ["", ".text", "xdp", "xdp/pass", "maps", ".data", ".relxdp", ".symtab", ".strtab", ".shstrtab"]
    shstr = b"\0".join(n.encode() for n in shnames) + b"\0"
    shoff = {n: shstr.index(n.encode() + b"\0") if n else 0 for n in shnames}
    shoff[".text"] = shstr.index(b".text\0")
    shoff["xdp"] = shstr.index(b"\0xdp\0") + 1
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
    sym("counters", 0, 20, 1, 1, 4)
    sym("flows", 20, 20, 1, 1, 4)
    sym("gvar", 8, 8, 1, 1, 5)
    symtab = b"".join(syms)
    rel = b""
    for slot, (si, typ) in zip(call_slots, [(3, 10), (1, 10)]):       # add3 / .text section symbol
        rel += struct.pack("<QQ", 8 * slot, (si << 32) | typ)
    for slot, si in zip(ld_slots, [6, 8]):                            # counters / gvar
        rel += struct.pack("<QQ", 8 * slot, (si << 32) | 1)

    bodies = [b"", text, main, xdp_pass, maps, data, rel, symtab, strtab, shstr]
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
            (shoff["xdp/pass"], 1, 6, 0, 0, 8, 0), (shoff["maps"], 1, 3, 0, 0, 4, 0),
            (shoff[".data"], 1, 3, 0, 0, 8, 0), (shoff[".relxdp"], 9, 0, 7, 2, 8, 16),
            (shoff[".symtab"], 2, 0, 8, nlocal, 8, 24), (shoff[".strtab"], 3, 0, 0, 0, 1, 0),
            (shoff[".shstrtab"], 3, 0, 0, 0, 1, 0)]
    for (nm, typ, flags, link, info, align, ent), off, b in zip(meta, offs, bodies):
        out += struct.pack("<IIQQQQIIQQ", nm, typ, flags, 0, off if typ else 0, len(b), link, info, align, ent)
    hdr = b"\x7fELF" + bytes([2, 1, 1, 0]) + bytes(8)
    hdr += struct.pack("<HHIQQQIHHHHHH", 1, 247, 1, 0, 0, e_shoff, 0, 64, 0, 0, 64, len(meta), len(meta) - 1)
    out[:64] = hdr
    return bytes(out)


if __name__ == "__main__":
    data = build()
    with open(OUT, "wb") as f:
        f.write(data)
    print(f"wrote {OUT} ({len(data)} bytes)")
