"""The JIT's lane value cache (jit.cpp analyze_vc): a lane's own row of a small per-CPU array is
held across its packets -- in four registers up to 32 bytes, in an LDS slot per lane up to 128 --
and written back when the lane ends.  Programs here read and write the row at every offset and
size (aligned and not, across value boundaries, past the row end), increment counters in it (the
fused form: an LDS add in the LDS form), call map_update on the same map (a cold path: the row is
written back and the cache is switched off), and run on CPU IDs -1 and V (no row).  Every run
compares per-packet R0 / status / steps / err_pc, the packet memory and every map with the oracle,
bit for bit."""
import numpy as np
import pytest

from harness import Scenario, assert_same, kernel_of, run_engine, run_oracle
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu

# (E, S, update): rows of 32, 8, 8, 24, 32 bytes (registers), 20 and 136 bytes (not cached), 40, 64,
# 64, 128 bytes (LDS)
VC_CASES = [(4, 8, False), (2, 4, False), (1, 8, False), (3, 8, True), (2, 16, True), (5, 4, False), (4, 8, True),
            (10, 4, False), (8, 8, True), (4, 16, False), (16, 8, True), (17, 8, False)]


def _vc_prog(E, S, update):
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 8),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(4, 7, 2, 0),                 # r7: offset bits
        A.ldx(4, 8, 2, 4),                 # r8: size / key / update bits
        A.mov64_reg(1, 8),
        A.alu64("rsh", 1, 4),
        A.alu64("mod", 1, E),
        A.stx(4, 10, -4, 1),               # update key = (r8 >> 4) % E
    ]
    if update:   # every 8th packet: map_update(key, value = r8 repeated) -- the generic helper
        items += [
            A.mov64_reg(1, 8),
            A.alu64("and", 1, 7),
            A.jmp("jne", 1, 7, "lookup"),
            A.stx(8, 10, -24, 8),
            A.stx(8, 10, -16, 7),
            A.mov64_reg(2, 10),
            A.alu64("add", 2, -4),
            A.mov64_reg(3, 10),
            A.alu64("add", 3, -24),
            A.ld_map_fd(1, "pc"),
            A.mov64_imm(4, 0),
            A.call(A.FN_MAP_UPDATE_ELEM),
            "lookup",
        ]
    # the access: key 0's value (the row start) + r7 % (E * S + 2), so an 8-byte access may run
    # up to 8 bytes past the row (the gap and the next CPU's sub-array object: an error) but
    # never into the next vCPU's row, which another lane owns (concurrent writes there would race
    # as in the reference's processPool)
    items += [
        A.st(4, 10, -8, 0),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -8),
        A.ld_map_fd(1, "pc"),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "miss"),
        A.mov64_reg(9, 7),
        A.alu64("mod", 9, E * S + 2),
        A.alu64("add", 0, 9, reg=True),
        A.mov64_reg(1, 8),
        A.alu64("and", 1, 7),
    ]
    for k, n in enumerate((1, 2, 4)):
        items += [A.jmp("jne", 1, k, f"s{k + 1}"), A.ldx(n, 5, 0, 0), A.alu64("add", 5, 8, reg=True),
                  A.stx(n, 0, 0, 5), A.ja("done"), f"s{k + 1}"]
    # counter increments (4 / 8 bytes, the register dead after: jit.cpp fusable_inc), aligned or not
    for k, n in ((3, 4), (4, 8)):
        items += [A.jmp("jne", 1, k, f"s{k + 1}"), A.ldx(n, 4, 0, 0), A.alu64("add", 4, 0x10001 * k),
                  A.stx(n, 0, 0, 4), A.mov64_imm(5, 0x5eed + k), A.ja("done"), f"s{k + 1}"]
    items += [
        A.ldx(8, 5, 0, 0), A.alu64("add", 5, 8, reg=True), A.stx(8, 0, 0, 5),
        "done",
        A.mov64_reg(0, 5),
        A.exit_(),
        "miss",
        A.mov64_imm(0, 0xEEEE),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return ("vc", raw, rel)


def _vc_scenario(E, S, update, vcpus=8):
    init = [("pc", k.to_bytes(4, "little"), bytes((c * 16 + k + b) & 0xFF for b in range(S)), c)
            for c in range(vcpus) for k in range(E)]
    return Scenario(vcpus=vcpus, maps=[dict(name="pc", type=6, key_size=4, value_size=S, max_entries=E)],
                    progs=[_vc_prog(E, S, update)], map_init=init)


@pytest.mark.parametrize("case", range(len(VC_CASES)))
@pytest.mark.parametrize("sched", ["interleaved", "explicit"])
def test_lane_value_cache(gpu, case, sched):
    import mimic_amd as M
    from mimic_amd import jit as J

    E, S, update = VC_CASES[case]
    sc = _vc_scenario(E, S, update)
    cached = E * S <= 128 and E * S % 8 == 0
    import os

    if os.environ.get("MIMIC_JIT_VC", "1") != "0":
        src = J.kernel_source(*kernel_of(sc))
        assert ("vc_open(" in src) == cached and ("lvc_open(" in src) == (cached and E * S > 32)
    n = 4096
    buf, off, lens = W.make_packets(n, seed=100 + case)
    rng = np.random.default_rng(case)
    if sched == "explicit":   # CPU IDs -1 and V run too (no row: per-CPU lookups fail)
        cpu = rng.integers(-1, 9, n).astype(np.int32)
        mode = M.SCHED_EXPLICIT
    else:
        cpu = W.schedule_cpu(n, 8, "interleaved")
        mode = M.SCHED_INTERLEAVED
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu if sched == "explicit" else None, schedule=mode, spread=0)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
    ok = o["status"] == 0
    assert ok.any() and (~ok).any()   # some accesses run past the row


def test_lane_value_cache_classifier_many_packets_per_vcpu(gpu):
    """cfg 2's classifier with 64 packets per vCPU: the row stays in registers for 64 counter
    updates and is written back once."""
    import mimic_amd as M

    p = W.prog_classifier()
    n, V = 1 << 16, 1024
    sc = Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    buf, off, lens = W.make_packets(n, seed=5)
    cpu = W.schedule_cpu(n, V, "chunked")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_CHUNKED, spread=0)
    assert_same(o, e)
    assert sum(int(np.frombuffer(v, np.uint64).sum()) for v in e["maps"]["verdicts"]) == n


def jit_kernels():
    p = W.prog_classifier()
    ks = [kernel_of(_vc_scenario(*c)) for c in VC_CASES] + \
        [kernel_of(Scenario(vcpus=1, maps=p.maps, progs=[(p.name, p.raw, p.relocs)]))]
    for E, S in ((8, 8), (16, 8)):
        b = _vc_scenario(E, S, True)
        ks.append(kernel_of(Scenario(vcpus=b.vcpus, maps=b.maps, progs=[_padded(b.progs[0])], map_init=b.map_init)))
    return ks


def _padded(prog, pad=60):
    """The program with `pad` stack loads in front (r9 = the stack word at R10 - 8, overwritten
    by the program later): past the JIT's 48 memory / helper sites, so its kernel defers every
    slow path to the interpreter's resume kernel (jit.cpp defer_mode)."""
    name, raw, rel = prog
    pre, _ = A.assemble([A.ldx(8, 9, 10, -8)] * pad)
    return (name, pre + raw, [(s + pad, m) for s, m in rel])


@pytest.mark.parametrize("E,S", [(8, 8), (16, 8)])
def test_lds_row_cache_with_deferred_slow_paths(gpu, E, S):
    """The LDS row cache in a kernel that defers its slow paths: map_update on the cached map and
    accesses past the row defer the lane; the row is written back once at the deferral exit, so
    the resume kernel (interpreter) continues on the counters the JIT lane left."""
    from mimic_amd import jit as J

    base = _vc_scenario(E, S, True)
    sc = Scenario(vcpus=base.vcpus, maps=base.maps, progs=[_padded(base.progs[0])], map_init=base.map_init)
    src = J.kernel_source(*kernel_of(sc))
    assert "lvc_open(" in src and "DFR(" in src and "L_defer:\n    VC_FLUSH();" in src
    n = 4096
    buf, off, lens = W.make_packets(n, seed=300 + E)
    cpu = W.schedule_cpu(n, 8, "interleaved")
    import mimic_amd as M

    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED, spread=0)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
