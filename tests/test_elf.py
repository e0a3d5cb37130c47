"""ELF ingest (mimic_amd.elf, restating cilium/ebpf's LoadCollectionSpec for the hot path) on a
committed hand-built object (tests/golden/xdp_count.o, written by tests/golden/make_elf.py):
maps from the legacy "maps" section and .data, programs linked with their .text callees,
BPF-to-BPF calls fixed up by symbol (vm.go:142-194), map references with the PseudoMapFD /
PseudoMapValue sources RewriteProgram keys on (emulator_linux_.go:292-339)."""
import os
import struct
import sys

import numpy as np
import pytest

from harness import Scenario, packets_to_buffer, run_oracle
from mimic_amd import elf
from mimic_amd.vm import MimicError

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import make_elf  # noqa: E402

OBJ = os.path.join(GOLDEN, "xdp_count.o")


def scenario_of(spec, prog_names, vcpus=4):
    maps = [dict(name=m.Name, type=m.Type, key_size=m.KeySize, value_size=m.ValueSize, max_entries=m.MaxEntries,
                 datasec=m.Datasec) for m in spec.Maps.values()]
    init = [(m.Name, k, v, 0) for m in spec.Maps.values() for k, v in m.Contents]
    progs = [(n, spec.Programs[n].Instructions, list(spec.Programs[n].References)) for n in prog_names]
    return Scenario(vcpus=vcpus, maps=maps, progs=progs, map_init=init)


def test_fixture_is_reproducible():
    assert open(OBJ, "rb").read() == make_elf.build()


def test_collection_spec():
    spec = elf.LoadCollectionSpec(OBJ)
    assert set(spec.Maps) == {"counters", "flows", ".data"}
    c = spec.Maps["counters"]
    assert (c.Type, c.KeySize, c.ValueSize, c.MaxEntries) == (6, 4, 8, 4)
    d = spec.Maps[".data"]
    assert d.Datasec and d.ValueSize == 16 and d.Contents[0][1][8:] == struct.pack("<Q", 0x1122334455667788)
    assert spec.ProgramSections == {"xdp_count": "xdp", "xdp_pass": "xdp/pass"}


def test_linking_matches_the_reference_pipeline():
    """main function, then add3 and twice appended; call immediates = target - i - 1; LD_IMM64
    sources set to PseudoMapFD / PseudoMapValue with the variable offset in the second slot."""
    spec = elf.LoadCollectionSpec(OBJ)
    raw, rel = make_elf.expected_linked()
    p = spec.Programs["xdp_count"]
    assert p.Instructions == raw
    assert p.References == rel


def test_elf_program_runs_like_raw_slots_on_the_oracle():
    spec = elf.LoadCollectionSpec(OBJ)
    sc = scenario_of(spec, ["xdp_count", "xdp_pass"])
    raw, rel = make_elf.expected_linked()
    sc_raw = Scenario(vcpus=4, maps=sc.maps, progs=[("xdp_count", raw, rel), sc.progs[1]], map_init=sc.map_init)
    pk = [bytes([i % 256]) * (1 + i % 70) for i in range(40)] + [b""]
    buf, off, lens = packets_to_buffer(pk)
    cpu = (np.arange(len(pk)) % 4).astype(np.int32)
    o1 = run_oracle(sc, buf, off, lens, cpu)
    o2 = run_oracle(sc_raw, buf, off, lens, cpu)
    for k in ("r0", "status", "steps"):
        assert np.array_equal(o1[k], o2[k])
    assert o1["maps"] == o2["maps"]
    # Q12 (vm.go:163-169 + inst.go:253): a BPF-to-BPF call lands one slot BEFORE its target, so
    # call add3 runs main's final EXIT and call twice runs add3's EXIT -- both return at once with
    # r0 = 0.  r0 = gvar + first packet byte (packet 40 is empty: nothing added).
    assert int(o1["r0"][1]) == 0x1122334455667788 + 1 and int(o1["r0"][40]) == 0x1122334455667788
    assert set(np.asarray(o1["status"]).tolist()) == {0}


def _elf_bytes(patch):
    b = bytearray(make_elf.build())
    patch(b)
    return bytes(b)


def test_rejects_non_bpf_and_btf_maps_without_btf():
    with pytest.raises(MimicError, match="EM_BPF"):
        elf.load_collection_spec(_elf_bytes(lambda b: b.__setitem__(slice(18, 20), (62).to_bytes(2, "little"))))
    data = make_elf.build()
    i = data.index(b"\0.data\0") + 1          # rename the .data section to .maps
    with pytest.raises(MimicError, match="BTF-defined maps"):
        elf.load_collection_spec(data[:i] + b".maps" + data[i + 5:])


# ---------------------------------------------------------------------------------------------
# BTF-defined maps (".maps" + .BTF): cilium/ebpf v0.9.0 loadBTFMaps / mapSpecFromBTF
# ---------------------------------------------------------------------------------------------
OBJ_BTF = os.path.join(GOLDEN, "xdp_count_btf.o")


def test_btf_fixture_is_reproducible():
    assert open(OBJ_BTF, "rb").read() == make_elf.build(btf=True)


def test_btf_maps_equal_the_legacy_definitions():
    """The same maps declared with __uint / __type in SEC(".maps") parse to the same MapSpecs as
    the bpf_map_def of the legacy object, and the program links to the same slots and refs."""
    a, b = elf.LoadCollectionSpec(OBJ), elf.LoadCollectionSpec(OBJ_BTF)
    assert set(a.Maps) == set(b.Maps)
    for k in a.Maps:
        x, y = a.Maps[k], b.Maps[k]
        assert (x.Type, x.KeySize, x.ValueSize, x.MaxEntries, x.Datasec) == (y.Type, y.KeySize, y.ValueSize,
                                                                             y.MaxEntries, y.Datasec), k
    for n in a.Programs:
        assert a.Programs[n].Instructions == b.Programs[n].Instructions
        assert a.Programs[n].References == b.Programs[n].References


def test_btf_object_runs_like_the_legacy_object_on_the_oracle():
    sa = scenario_of(elf.LoadCollectionSpec(OBJ), ["xdp_count", "xdp_pass"])
    sb = scenario_of(elf.LoadCollectionSpec(OBJ_BTF), ["xdp_count", "xdp_pass"])
    pk = [bytes([i % 256]) * (1 + i % 70) for i in range(40)] + [b""]
    buf, off, lens = packets_to_buffer(pk)
    cpu = (np.arange(len(pk)) % 4).astype(np.int32)
    oa, ob = run_oracle(sa, buf, off, lens, cpu), run_oracle(sb, buf, off, lens, cpu)
    for k in ("r0", "status", "steps"):
        assert np.array_equal(oa[k], ob[k])
    assert oa["maps"] == ob["maps"]


def _btf_with(members):
    """a .BTF section with one map whose struct has the given (name, kind, value) members:
    kind 'u' = __uint(name, value), 't' = __type(name, an INT of `value` bytes)"""
    strs = bytearray(b"\0")

    def sname(n):
        o = len(strs)
        strs.extend(n.encode() + b"\0")
        return o

    types = []

    def add(kind, name_off, st, extra=b"", vlen=0):
        types.append(struct.pack("<III", name_off, (kind << 24) | vlen, st) + extra)
        return len(types)

    t_int = add(1, sname("int"), 4, struct.pack("<I", (1 << 24) | 32))
    mem = b""
    for k, (n, kind, v) in enumerate(members):
        if kind == "u":
            arr = add(3, 0, 0, struct.pack("<III", t_int, t_int, v))
            t = add(2, 0, arr)
        else:
            it = add(1, sname(f"i{v}"), v, struct.pack("<I", 8 * v))
            t = add(2, 0, it)
        mem += struct.pack("<III", sname(n), t, 64 * k)
    s = add(4, 0, 8 * len(members), mem, vlen=len(members))
    v = add(14, sname("m"), s, struct.pack("<I", 1))
    add(15, sname(".maps"), 8 * len(members), struct.pack("<III", v, 0, 8 * len(members)), vlen=1)
    tb = b"".join(types)
    return struct.pack("<HBBIIIII", 0xEB9F, 1, 0, 24, 0, len(tb), len(tb), len(strs)) + tb + bytes(strs)


def _btf_maps_of(members):
    sec = elf._Sec(1, ".BTF", 1, 0, 0, 0, 0, 0, _btf_with(members))
    return elf._btf_maps([sec], [])


def test_btf_map_attribute_forms():
    m = _btf_maps_of([("type", "u", 1), ("max_entries", "u", 10), ("key", "t", 16), ("value", "t", 8),
                      ("map_flags", "u", 1)])["m"]
    assert (m.Type, m.KeySize, m.ValueSize, m.MaxEntries) == (1, 16, 8, 10)
    m = _btf_maps_of([("type", "u", 5), ("key_size", "u", 13), ("value_size", "u", 4), ("max_entries", "u", 3),
                      ("pinning", "u", 1)])["m"]
    assert (m.Type, m.KeySize, m.ValueSize, m.MaxEntries) == (5, 13, 4, 3)


@pytest.mark.parametrize("members,msg", [
    ([("type", "u", 1), ("key", "t", 4), ("key_size", "u", 4)], "both key and key_size"),
    ([("type", "u", 1), ("value_size", "u", 4), ("value", "t", 8)], "both value and value_size"),
    ([("type", "u", 1), ("bogus", "u", 4)], "unrecognized field"),
    ([("type", "u", 3), ("values", "u", 4)], "not supported"),
    ([("max_entries", "u", 4)], "no type"),
])
def test_btf_map_errors(members, msg):
    with pytest.raises(MimicError, match=msg):
        _btf_maps_of(members)


def test_btf_maps_without_btf_section_is_an_error():
    secs = [elf._Sec(1, ".maps", 1, 0, 0, 0, 0, 0, bytes(32))]
    with pytest.raises(MimicError, match=".BTF"):
        elf._map_defs(secs, [])
