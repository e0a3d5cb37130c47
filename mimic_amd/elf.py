"""ELF ingest: clang-built eBPF objects -> MapSpecs and ready-to-load ProgramSpecs.

The reference takes *ebpf.ProgramSpec from cilium/ebpf v0.9.0 (go.mod:5), whose
LoadCollectionSpec parses the object; VM.AddProgram then pads a Nop after every LD_IMM64
(vm.go:102-112), LinuxEmulator.RewriteProgram turns map references into map object addresses
(emulator_linux_.go:292-339) and fixupJumpsAndCalls resolves BPF-to-BPF calls by symbol
(vm.go:142-194).  cilium/ebpf is not in this image; this module restates the part of its ELF
reader the hot path needs, with the engine's raw-slot boundary as the output:

* raw slots keep LD_IMM64 as its two ELF slots -- the second slot (opcode 0) is exactly the
  Nop the reference inserts, so slot indexes equal the reference's instruction indexes;
* a program = a global function symbol of an executable section other than .text, followed by
  every function it calls (transitively) appended in order of first reference, as the linker of
  cilium/ebpf appends the .text functions a program references; each call's immediate is then
  fixed up to `target - i - 1` (vm.go:163-169, Q12);
* R_BPF_64_64 relocations of LD_IMM64 against a symbol of the legacy "maps" section become map
  references with src = BPF_PSEUDO_MAP_FD (1); against .data / .rodata / .bss they become
  references to that data-section map with src = BPF_PSEUDO_MAP_VALUE (2) and the variable's
  offset in the second slot's immediate (the reference ignores it, using inst.Offset: Q16);
* the "maps" section holds struct bpf_map_def {type, key_size, value_size, max_entries, flags}
  per map symbol; data sections become datasec array maps (key 4, value = section size, one
  entry) with the section bytes as their contents;
* BTF-defined maps (the ".maps" section every current clang / libbpf object uses): the .BTF
  section's DATASEC ".maps" lists one VAR per map, whose STRUCT type encodes the attributes the
  way libbpf's __uint / __type macros do -- `type`, `max_entries`, `map_flags`, `key_size`,
  `value_size`, `pinning` as a pointer to an array whose element count is the value, `key` /
  `value` as a pointer to the key / value type (its BTF size is the key / value size).  This is
  cilium/ebpf v0.9.0's loadBTFMaps + mapSpecFromBTF (elf_reader.go) with its errors for unknown
  members and for both `key` and `key_size` (or `value` and `value_size`); `values` (map-in-map
  and program-array initial contents) is rejected.  LD_IMM64 relocations against a ".maps"
  symbol are map references like the legacy section's.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .vm import MapSpec, MimicError, ProgramSpec

EM_BPF = 247
SHT_PROGBITS, SHT_SYMTAB, SHT_STRTAB, SHT_NOBITS, SHT_REL = 1, 2, 3, 8, 9
SHF_EXECINSTR = 0x4
STT_OBJECT, STT_FUNC, STT_SECTION = 1, 2, 3
STB_GLOBAL = 1
R_BPF_64_64, R_BPF_64_ABS64, R_BPF_64_ABS32, R_BPF_64_32 = 1, 2, 3, 10
PSEUDO_MAP_FD, PSEUDO_MAP_VALUE, PSEUDO_CALL = 1, 2, 1
DATA_SECTIONS = (".data", ".rodata", ".bss")


@dataclass
class CollectionMap(MapSpec):
    Contents: List[Tuple[bytes, bytes]] = field(default_factory=list)   # (key, value) to Update after AddMap


@dataclass
class CollectionSpec:
    Maps: Dict[str, CollectionMap]
    Programs: Dict[str, ProgramSpec]
    ProgramSections: Dict[str, str]   # program name -> ELF section name (its program type)


@dataclass
class _Sec:
    idx: int
    name: str
    type: int
    flags: int
    off: int
    size: int
    link: int
    info: int
    data: bytes


@dataclass
class _Sym:
    name: str
    value: int
    size: int
    type: int
    bind: int
    shndx: int


def _parse(elf: bytes):
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise MimicError("not a 64-bit little-endian ELF file")
    (e_type, e_machine, _, _, _, e_shoff, _, _, _, _, e_shentsize, e_shnum, e_shstrndx) = struct.unpack_from(
        "<HHIQQQIHHHHHH", elf, 16)
    if e_machine != EM_BPF:
        raise MimicError(f"ELF machine {e_machine} is not EM_BPF")
    raw = []
    for i in range(e_shnum):
        name, typ, flags, _, off, size, link, info, _, _ = struct.unpack_from("<IIQQQQIIQQ", elf, e_shoff + i * e_shentsize)
        raw.append((name, typ, flags, off, size, link, info))
    shstr = raw[e_shstrndx]
    names = elf[shstr[3]:shstr[3] + shstr[4]]

    def cstr(tab, o):
        return tab[o:tab.index(b"\0", o)].decode()

    secs = []
    for i, (nm, typ, flags, off, size, link, info) in enumerate(raw):
        data = b"" if typ == SHT_NOBITS else elf[off:off + size]
        secs.append(_Sec(i, cstr(names, nm), typ, flags, off, size, link, info, data))
    syms: List[_Sym] = []
    symtab = next((s for s in secs if s.type == SHT_SYMTAB), None)
    if symtab is not None:
        strtab = secs[symtab.link].data
        for o in range(0, len(symtab.data), 24):
            nm, info, _, shndx, value, size = struct.unpack_from("<IBBHQQ", symtab.data, o)
            syms.append(_Sym(cstr(strtab, nm), value, size, info & 0xF, info >> 4, shndx))
    rels: Dict[int, Dict[int, Tuple[int, int]]] = {}   # target section -> {byte offset: (sym index, type)}
    for s in secs:
        if s.type == SHT_REL:
            m = rels.setdefault(s.info, {})
            for o in range(0, len(s.data), 16):
                off, info = struct.unpack_from("<QQ", s.data, o)
                m[off] = (info >> 32, info & 0xFFFFFFFF)
    return secs, syms, rels


# BTF kinds (linux/btf.h, as cilium/ebpf v0.9.0 btf/types.go reads them)
BTF_INT, BTF_PTR, BTF_ARRAY, BTF_STRUCT, BTF_UNION, BTF_ENUM, BTF_FWD, BTF_TYPEDEF, BTF_VOLATILE, BTF_CONST, \
    BTF_RESTRICT, BTF_FUNC, BTF_FUNC_PROTO, BTF_VAR, BTF_DATASEC, BTF_FLOAT, BTF_DECL_TAG, BTF_TYPE_TAG, \
    BTF_ENUM64 = range(1, 20)
BTF_MAGIC = 0xEB9F


@dataclass
class _BtfType:
    kind: int
    name: str
    size_or_type: int
    vlen: int
    kind_flag: int
    extra: object = None    # ARRAY: (elem, index, nelems); STRUCT/UNION: [(name, type, bit offset)];
                            # DATASEC: [(type, offset, size)]; VAR: linkage


def parse_btf(data: bytes) -> List[Optional[_BtfType]]:
    """The .BTF section's type table (index = type id; id 0 = void -> None).  btf/btf.go +
    btf/types.go of cilium/ebpf v0.9.0 read the same header, type records and string table."""
    if len(data) < 24:
        raise MimicError("BTF section too short")
    magic, version, flags, hdr_len, type_off, type_len, str_off, str_len = struct.unpack_from("<HBBIIIII", data, 0)
    if magic != BTF_MAGIC:
        raise MimicError(f"BTF magic {magic:#x} (big-endian or not BTF)")
    base = hdr_len
    types_b = data[base + type_off:base + type_off + type_len]
    strs = data[base + str_off:base + str_off + str_len]

    def name(o: int) -> str:
        if o >= len(strs):
            raise MimicError(f"BTF string offset {o} out of range")
        e = strs.index(b"\0", o)
        return strs[o:e].decode()

    out: List[Optional[_BtfType]] = [None]
    o = 0
    while o < len(types_b):
        name_off, info, st = struct.unpack_from("<III", types_b, o)
        o += 12
        kind, vlen, kflag = (info >> 24) & 0x1F, info & 0xFFFF, info >> 31
        t = _BtfType(kind, name(name_off), st, vlen, kflag)
        if kind == BTF_INT or kind == BTF_VAR or kind == BTF_DECL_TAG:
            t.extra = struct.unpack_from("<I", types_b, o)[0]
            o += 4
        elif kind == BTF_ARRAY:
            t.extra = struct.unpack_from("<III", types_b, o)
            o += 12
        elif kind in (BTF_STRUCT, BTF_UNION):
            mem = []
            for _ in range(vlen):
                mn, mt, moff = struct.unpack_from("<III", types_b, o)
                o += 12
                mem.append((name(mn), mt, (moff & 0xFFFFFF) if kflag else moff))
            t.extra = mem
        elif kind == BTF_ENUM:
            o += 8 * vlen
        elif kind == BTF_ENUM64:
            o += 12 * vlen
        elif kind == BTF_FUNC_PROTO:
            o += 8 * vlen
        elif kind == BTF_DATASEC:
            t.extra = [struct.unpack_from("<III", types_b, o + 12 * k) for k in range(vlen)]
            o += 12 * vlen
        elif kind in (BTF_PTR, BTF_FWD, BTF_TYPEDEF, BTF_VOLATILE, BTF_CONST, BTF_RESTRICT, BTF_FUNC, BTF_FLOAT,
                      BTF_TYPE_TAG):
            pass
        else:
            raise MimicError(f"BTF type {len(out)}: unknown kind {kind}")
        out.append(t)
    return out


def _btf_resolve(types, tid: int) -> int:
    """skip typedefs and qualifiers (btf.UnderlyingType / skipQualifiers)"""
    for _ in range(64):
        t = types[tid] if 0 < tid < len(types) else None
        if t is None or t.kind not in (BTF_TYPEDEF, BTF_VOLATILE, BTF_CONST, BTF_RESTRICT, BTF_TYPE_TAG):
            return tid
        tid = t.size_or_type
    raise MimicError("BTF: qualifier chain too long")


def btf_sizeof(types, tid: int) -> int:
    """btf.Sizeof: the byte size of a type"""
    tid = _btf_resolve(types, tid)
    t = types[tid] if 0 < tid < len(types) else None
    if t is None:
        raise MimicError("BTF: size of void")
    if t.kind in (BTF_INT, BTF_ENUM, BTF_ENUM64, BTF_STRUCT, BTF_UNION, BTF_DATASEC, BTF_FLOAT):
        return t.size_or_type
    if t.kind == BTF_PTR:
        return 8
    if t.kind == BTF_ARRAY:
        elem, _, n = t.extra
        return n * btf_sizeof(types, elem)
    if t.kind == BTF_VAR:
        return btf_sizeof(types, t.size_or_type)
    raise MimicError(f"BTF: type {tid} (kind {t.kind}) has no size")


def _btf_uint(types, tid: int, what: str) -> int:
    """uintFromBTF: __uint(name, N) is `int (*name)[N]` -- a pointer to an array of N elements"""
    p = types[_btf_resolve(types, tid)]
    if p is None or p.kind != BTF_PTR:
        raise MimicError(f"BTF map {what}: not a pointer")
    a = types[_btf_resolve(types, p.size_or_type)]
    if a is None or a.kind != BTF_ARRAY:
        raise MimicError(f"BTF map {what}: not a pointer to an array")
    return a.extra[2]


def _btf_maps(secs, syms) -> Dict[str, CollectionMap]:
    """cilium/ebpf v0.9.0 loadBTFMaps / mapSpecFromBTF over the ".maps" DATASEC."""
    btf_sec = next((s for s in secs if s.name == ".BTF"), None)
    if btf_sec is None:
        raise MimicError("BTF-defined maps (.maps) without a .BTF section")
    types = parse_btf(btf_sec.data)
    ds = next((t for t in types if t is not None and t.kind == BTF_DATASEC and t.name == ".maps"), None)
    if ds is None:
        raise MimicError(".BTF has no DATASEC \".maps\"")
    maps: Dict[str, CollectionMap] = {}
    for vt, _off, _size in ds.extra:
        var = types[vt]
        if var is None or var.kind != BTF_VAR:
            raise MimicError(f"DATASEC .maps entry {vt} is not a VAR")
        st = types[_btf_resolve(types, var.size_or_type)]
        if st is None or st.kind != BTF_STRUCT:
            raise MimicError(f"map {var.name}: expected a struct, got kind {st.kind if st else 0}")
        mtype = key_size = value_size = max_entries = None
        key_typed = value_typed = False
        for mname, mt, _bits in st.extra:
            if mname == "type":
                mtype = _btf_uint(types, mt, f"{var.name}.type")
            elif mname == "map_flags" or mname == "pinning" or mname == "map_extra" or mname == "numa_node":
                _btf_uint(types, mt, f"{var.name}.{mname}")
            elif mname == "max_entries":
                max_entries = _btf_uint(types, mt, f"{var.name}.max_entries")
            elif mname == "key":
                if key_size is not None:
                    raise MimicError(f"map {var.name}: both key and key_size")
                p = types[_btf_resolve(types, mt)]
                if p is None or p.kind != BTF_PTR:
                    raise MimicError(f"map {var.name}: key is not a pointer")
                key_size = btf_sizeof(types, p.size_or_type)
                key_typed = True
            elif mname == "key_size":
                if key_typed:
                    raise MimicError(f"map {var.name}: both key and key_size")
                key_size = _btf_uint(types, mt, f"{var.name}.key_size")
            elif mname == "value":
                if value_size is not None:
                    raise MimicError(f"map {var.name}: both value and value_size")
                p = types[_btf_resolve(types, mt)]
                if p is None or p.kind != BTF_PTR:
                    raise MimicError(f"map {var.name}: value is not a pointer")
                value_size = btf_sizeof(types, p.size_or_type)
                value_typed = True
            elif mname == "value_size":
                if value_typed:
                    raise MimicError(f"map {var.name}: both value and value_size")
                value_size = _btf_uint(types, mt, f"{var.name}.value_size")
            elif mname == "values":
                raise MimicError(f"map {var.name}: initial values (map-in-map / program array) are not supported")
            else:
                raise MimicError(f"map {var.name}: unrecognized field {mname!r}")
        if mtype is None:
            raise MimicError(f"map {var.name}: no type")
        maps[var.name] = CollectionMap(var.name, mtype, key_size or 0, value_size or 0, max_entries or 0)
    return maps


def _map_defs(secs, syms) -> Dict[str, CollectionMap]:
    maps: Dict[str, CollectionMap] = {}
    for s in secs:
        if s.name == ".maps":
            maps.update(_btf_maps(secs, syms))
        elif s.name == "maps" or s.name.startswith("maps/"):
            for y in syms:
                if y.shndx != s.idx or y.type == STT_SECTION or not y.name:
                    continue
                if y.size and y.size < 16:
                    raise MimicError(f"map definition {y.name} is {y.size} bytes")
                typ, ks, vs, me = struct.unpack_from("<IIII", s.data, y.value)
                maps[y.name] = CollectionMap(y.name, typ, ks, vs, me)
        elif s.name in DATA_SECTIONS:
            val = bytes(s.size) if s.type == SHT_NOBITS else s.data
            maps[s.name] = CollectionMap(s.name, 2, 4, s.size, 1, True, [(b"\0\0\0\0", val)])
    return maps


def load_collection_spec(elf: bytes) -> CollectionSpec:
    """ebpf.LoadCollectionSpec restated for the engine (see the module docstring)."""
    secs, syms, rels = _parse(elf)
    maps = _map_defs(secs, syms)
    funcs = {}           # (section idx, byte offset) -> symbol
    for y in syms:
        if y.type == STT_FUNC and 0 < y.shndx < len(secs):
            funcs[(y.shndx, y.value)] = y

    def func_slots(y: _Sym):
        s = secs[y.shndx]
        size = y.size or (s.size - y.value)
        return s, bytearray(s.data[y.value:y.value + size])

    def call_target(s: _Sec, y: _Sym, k: int, ins: bytes) -> _Sym:
        """the function a BPF-to-BPF call at slot k of function y (section s) calls"""
        off = y.value + 8 * k
        imm = struct.unpack_from("<i", ins, 4)[0]
        rel = rels.get(s.idx, {}).get(off)
        if rel is not None:
            t = syms[rel[0]]
            if t.type == STT_FUNC:
                return t
            if t.type == STT_SECTION:   # section symbol + the immediate's slot offset
                key = (t.shndx, t.value + 8 * (imm + 1))
                if key in funcs:
                    return funcs[key]
            raise MimicError(f"call at {s.name}+{off}: unresolved target {t.name!r}")
        key = (s.idx, off + 8 * (imm + 1))   # same-section call, no relocation
        if key not in funcs:
            raise MimicError(f"call at {s.name}+{off}: no function at slot {imm + 1} from here")
        return funcs[key]

    programs: Dict[str, ProgramSpec] = {}
    sections: Dict[str, str] = {}
    for y in syms:
        s = secs[y.shndx] if 0 < y.shndx < len(secs) else None
        if (s is None or y.type != STT_FUNC or y.bind != STB_GLOBAL or not (s.flags & SHF_EXECINSTR)
                or s.name == ".text"):
            continue
        order = [y]                      # main function, then callees in order of first reference
        start: Dict[Tuple[int, int], int] = {}
        bodies = []
        refs: List[Tuple[int, str]] = []
        calls: List[Tuple[int, _Sym]] = []
        base = 0
        q = 0
        while q < len(order):
            fy = order[q]
            q += 1
            fs, body = func_slots(fy)
            start[(fy.shndx, fy.value)] = base
            rel = rels.get(fs.idx, {})
            for k in range(len(body) // 8):
                ins = body[8 * k:8 * k + 8]
                op, regs = ins[0], ins[1]
                off = fy.value + 8 * k
                if op == 0x85 and (regs >> 4) == PSEUDO_CALL:
                    t = call_target(fs, fy, k, ins)
                    if (t.shndx, t.value) not in [(o.shndx, o.value) for o in order]:
                        order.append(t)
                    calls.append((base + k, t))
                elif op == 0x18 and off in rel:
                    t = syms[rel[off][0]]
                    tsec = secs[t.shndx] if 0 < t.shndx < len(secs) else None
                    if tsec is None:
                        raise MimicError(f"{fs.name}+{off}: load of undefined symbol {t.name!r}")
                    if tsec.name in DATA_SECTIONS:
                        voff = (t.value if t.type != STT_SECTION else 0) + struct.unpack_from("<i", ins, 4)[0]
                        body[8 * k + 1] = (regs & 0x0F) | (PSEUDO_MAP_VALUE << 4)
                        body[8 * k + 4:8 * k + 8] = b"\0\0\0\0"
                        body[8 * k + 12:8 * k + 16] = struct.pack("<I", voff & 0xFFFFFFFF)
                        refs.append((base + k, tsec.name))
                    elif tsec.name in ("maps", ".maps") or tsec.name.startswith("maps/"):
                        body[8 * k + 1] = (regs & 0x0F) | (PSEUDO_MAP_FD << 4)
                        refs.append((base + k, t.name))
                    else:
                        raise MimicError(f"{fs.name}+{off}: LD_IMM64 of {t.name!r} in section {tsec.name}")
            bodies.append(bytes(body))
            base += len(body) // 8
        insns = bytearray(b"".join(bodies))
        for i, t in calls:               # fixupJumpsAndCalls: imm = symbol offset - i - 1
            struct.pack_into("<i", insns, 8 * i + 4, start[(t.shndx, t.value)] - i - 1)
        programs[y.name] = ProgramSpec(y.name, bytes(insns), refs)
        sections[y.name] = s.name
    return CollectionSpec(maps, programs, sections)


def LoadCollectionSpec(path_or_bytes) -> CollectionSpec:
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    return load_collection_spec(bytes(data))
