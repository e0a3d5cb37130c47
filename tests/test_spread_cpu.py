"""Spread kernels on the CPU host (no device): which program sets jit.cpp analyze_spread accepts,
and that the accepted kernels compile for gfx950 within the 4-wave register budget.

A spread kernel runs one vCPU's packets on many lanes.  It is exact only when the per-CPU state
the programs touch is counters they increment (fused increments through one per-CPU array
lookup) and nothing else observes the looked-up value region: no load or store through the
value pointer outside the increment, the pointer never stored or passed to a helper, the
counter never kept in a register after the increment.  The address itself may flow anywhere
(it is a function of the packet's vCPU and key)."""
import pytest

from harness import Scenario, spread_kernel_of
from mimic_amd import asm as A
from mimic_amd import jit as J
from mimic_amd import workloads as W

PCPU = dict(name="c", type=6, key_size=4, value_size=8, max_entries=4)


def _allowed(items, maps=(PCPU,), vcpus=256):
    raw, rel = A.assemble(items)
    sc = Scenario(vcpus=vcpus, maps=list(maps), progs=[("p", raw, rel)])
    raws, _, _, spec = spread_kernel_of(sc)
    return J.spread_source(raws, *spec)[1]


def _lookup(key=1, m="c"):
    return [A.st(4, 10, -4, key), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, m),
            A.call(A.FN_MAP_LOOKUP_ELEM)]


def _inc(base=0, reg=1, off=0, size=8):
    return [A.ldx(size, reg, base, off), A.alu64("add", reg, 1), A.stx(size, base, off, reg)]


@pytest.mark.parametrize("fn,want", [("prog_classifier", True), ("prog_parse5", True), ("prog_flowtrack", False),
                                     ("prog_flowcount", False), ("prog_pass8", False)])
def test_workload_programs(fn, want):
    p = getattr(W, fn)()
    sc = Scenario(vcpus=256, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    raws, _, _, spec = spread_kernel_of(sc)
    src, ok = J.spread_source(raws, *spec)
    assert ok == want
    assert ("#define MIMIC_SPREAD 1" in src) == want


def test_accepted_forms():
    tail = [A.mov64_imm(0, 2), A.exit_()]
    # plain counter; a copied pointer; the address returned in R0; get_smp_processor_id; 4-byte ALU32 counter
    assert _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc() + tail)
    assert _allowed(_lookup() + [A.mov64_reg(6, 0), A.jmp("jeq", 6, 0, 3)] + _inc(base=6) + tail)
    assert _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc() + [A.exit_()])
    assert _allowed([A.call(A.FN_GET_SMP_PROCESSOR_ID), A.stx(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4),
                     A.ld_map_fd(1, "c"), A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, 3)] + _inc() + tail)
    m4 = dict(PCPU, value_size=4)
    assert _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3), A.ldx(4, 1, 0, 0), A.alu32("add", 1, 1), A.stx(4, 0, 0, 1)] + tail,
                    maps=(m4,))


def test_rejected_forms():
    tail = [A.mov64_imm(0, 2), A.exit_()]
    # the counter loaded into R0 (leaks the order of the vCPU's packets)
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 1), A.ldx(8, 0, 0, 0), A.exit_()])
    # the counter register still live after the increment
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 4)] + _inc() + [A.mov64_reg(0, 1), A.exit_()] + tail)
    # a plain store through the value pointer
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 1), A.st(8, 0, 0, 5)] + tail)
    # the pointer stored to the stack, or passed to a helper as a key
    assert not _allowed(_lookup() + [A.stx(8, 10, -16, 0)] + tail)
    assert not _allowed(_lookup() + [A.mov64_reg(2, 0), A.ld_map_fd(1, "c"), A.call(A.FN_MAP_LOOKUP_ELEM)] + tail)
    # a pointer derived by arithmetic is still the region: a load through it
    assert not _allowed(_lookup() + [A.alu64("add", 0, 8), A.jmp("jeq", 0, 8, 1), A.ldx(8, 1, 0, 0)] + tail)
    # two per-CPU arrays, a shared array, a hash map, map updates, tail calls
    m2 = dict(PCPU, name="d")
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc() + _lookup(m="d") + [A.jmp("jeq", 0, 0, 3)] + _inc() + tail,
                        maps=(PCPU, m2))
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc() + tail, maps=(dict(PCPU, type=2),))
    assert not _allowed(_lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc() + tail, maps=(dict(PCPU, type=1),))
    assert not _allowed(_lookup() + [A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.mov64_reg(3, 10), A.alu64("add", 3, -16),
                                     A.ld_map_fd(1, "c"), A.mov64_imm(4, 0), A.call(A.FN_MAP_UPDATE_ELEM)] + tail)
    # a loop (budget checks) and no counter at all
    assert not _allowed([A.mov64_imm(0, 0), "top", A.alu64("add", 0, 1), A.jmp("jlt", 0, 10, "top"), A.exit_()])
    assert not _allowed(tail)


def test_base_provenance():
    """Loads and stores outside the fused increment must go through a base derived from R1 (the
    context), R10 (the stack) or a packet pointer; anything else may address per-CPU memory
    (memory_controller.go:117-145 resolves any address), so the program set runs one lane per vCPU."""
    cnt = _lookup() + [A.jmp("jeq", 0, 0, 3)] + _inc()
    tail = [A.mov64_imm(0, 2), A.exit_()]
    # packet pointers from the context (data / data_end), arithmetic on them, the stack: accepted
    pkt = [A.mov64_reg(6, 1), A.ldx(4, 2, 6, 0), A.ldx(4, 3, 6, 4), A.mov64_reg(4, 2), A.alu64("add", 4, 14),
           A.jmp("jgt", 4, 3, 2), A.ldx(1, 5, 2, 12), A.stx(1, 2, 0, 5)]
    assert _allowed(pkt + cnt + tail)
    assert _allowed([A.ldx(4, 2, 1, 16), A.stx(4, 10, -8, 2), A.ldx(4, 3, 10, -8)] + cnt + tail)
    # an LD_IMM64 constant as a base (the round-4 guard case), a pointer loaded from memory, a
    # context scalar (ingress_ifindex), a helper's clobbered argument register: rejected
    assert not _allowed(cnt + [A.ld_imm64(3, 0x10000), A.ldx(8, 0, 3, 0), A.exit_()])
    assert not _allowed(cnt + [A.ld_imm64(3, 0x10000), A.st(8, 3, 0, 1)] + tail)
    assert not _allowed([A.stx(8, 10, -8, 1), A.ldx(8, 6, 10, -8), A.ldx(4, 2, 6, 0)] + cnt + tail)
    assert not _allowed([A.ldx(4, 6, 1, 12), A.ldx(4, 2, 6, 0)] + cnt + tail)
    assert not _allowed([A.mov64_reg(6, 1)] + cnt + [A.ldx(4, 2, 1, 0)] + tail)
    # scalars alone (an immediate moved into a register, then arithmetic)
    assert not _allowed(cnt + [A.mov64_imm(3, 0x10000), A.alu64("add", 3, 8), A.ldx(8, 0, 3, 0), A.exit_()])
    # a base that is the context on one path and a constant on the other
    assert not _allowed([A.mov64_reg(6, 1), A.ldx(4, 2, 1, 12), A.jmp("jeq", 2, 0, 1), A.ld_imm64(6, 0x10000),
                         A.ldx(4, 3, 6, 0)] + cnt + tail)


def test_lds_table_or_atomics():
    """The block's counter table lives in LDS when min(1024, V) rows fit 32 KiB, else every
    increment is an agent-scope atomic into the map (spread_spec mirrors engine.cpp spread_build)."""
    p = W.prog_classifier()
    for V, rows in ((256, 256), (4096, 1024), (1 << 18, 1024)):
        assert J.spread_spec([(p.raw, p.relocs)], p.maps, V)[2] == rows
    q = W.prog_parse5()
    assert J.spread_spec([(q.raw, q.relocs)], q.maps, 256)[2] == 0   # 2 KiB rows: atomics
    assert J.spread_spec([(q.raw, q.relocs)], q.maps, 16)[2] == 16


@pytest.mark.parametrize("fn,V", [("prog_classifier", 256), ("prog_classifier", 1 << 18), ("prog_parse5", 256)])
def test_spread_kernels_compile_within_budget(fn, V):
    p = getattr(W, fn)()
    sc = Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    raws, _, _, spec = spread_kernel_of(sc)
    src, ok = J.spread_source(raws, *spec)
    assert ok
    res = J.kernel_resources(J.code_object(src))
    assert res["scratch"] == 0 and res["vgpr_spill"] == 0, res
    assert res["waves_per_simd"] >= 4, res
    assert res["lds"] == (spec[2] * (p.maps[0]["max_entries"] * p.maps[0]["value_size"]) if spec[2] else 0), res


@pytest.mark.parametrize("fn,rows,spill", [("prog_classifier", 256, 0), ("prog_parse5", 16, 4)])
def test_owned_form_compiles_within_budget(fn, rows, spill):
    """The owned form (every packet of a block's vCPUs in the block, jit.cpp spread_own): the same
    analysis, an LDS table of min(256, 32 KiB / row) rows, 4 waves per SIMD; the classifier's without
    scratch, parse5's with at most 4 spilled VGPRs (its 2 KiB rows allow only Q = 1 from P = 16 on)."""
    p = getattr(W, fn)()
    sc = Scenario(vcpus=262144, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    raws, _, _, spec = spread_kernel_of(sc, own=True)
    assert spec[2] == rows | (1 << 31)
    src, ok = J.spread_source(raws, *spec)
    assert ok and "#define MIMIC_SPREAD_OWN 1" in src and f"#define SPREAD_ROWS {rows}u" in src
    r = J.kernel_resources(J.code_object(src))
    assert r["vgpr_spill"] <= spill and (spill or r["scratch"] == 0) and r["waves_per_simd"] >= 4, r


def test_owned_form_refuses_what_spread_refuses():
    items = _lookup() + [A.jmp("jeq", 0, 0, 3), A.ldx(8, 1, 0, 0), A.mov64_reg(0, 1), A.exit_(), A.mov64_imm(0, 2), A.exit_()]
    raw, rel = A.assemble(items)
    sc = Scenario(vcpus=4096, maps=[PCPU], progs=[("p", raw, rel)])
    raws, _, _, spec = spread_kernel_of(sc, own=True)
    src, ok = J.spread_source(raws, *spec)
    assert not ok and "MIMIC_SPREAD_OWN" not in src
