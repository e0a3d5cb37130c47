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


def test_rejects_non_bpf_and_btf_maps():
    with pytest.raises(MimicError, match="EM_BPF"):
        elf.load_collection_spec(_elf_bytes(lambda b: b.__setitem__(slice(18, 20), (62).to_bytes(2, "little"))))
    data = make_elf.build()
    i = data.index(b"\0.data\0") + 1          # rename the .data section to .maps
    with pytest.raises(MimicError, match="BTF-defined maps"):
        elf.load_collection_spec(data[:i] + b".maps" + data[i + 5:])
