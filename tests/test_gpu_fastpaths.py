"""The JIT's inline fast paths against the oracle, each driven into its edge cases and fallbacks
(jit.cpp: early loads and their void flag, inline hash lookups, inline tail calls, flow-keys /
sock pointer accesses, early LD_ABS / LD_IND).  Every run compares per-packet R0 / status / steps
/ err_pc, the packet memory and every map with the oracle, bit for bit."""
import numpy as np
import pytest

from harness import (Scenario, assert_same, kernel_of, packets_to_buffer, run_engine, run_engine_skb, run_oracle, run_oracle_skb,
                     run_sequence_engine, run_sequence_oracle, assert_same_sequence)
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu

S, FK, SK = A.SKB, A.FLOW_KEYS, A.SOCK


def _prog(name, items, maps=()):
    raw, rel = A.assemble(items)
    return (name, raw, rel)


# ---------------------------------------------------------------------------------------------
# early packet loads (analyze_spec): a store through R10 that leaves the stack lands in the packet
# between the early load's issue point and its use -- the void flag must force the reload
# ---------------------------------------------------------------------------------------------
def _escape_prog(off, size=1, through_stack=False):
    # R10 = St + 256; packet data = St + 2048 + 1 (headroom 0): R10 + 1805 = data + 12 (the
    # store leaves the stack and lands on the loaded bytes); R10 - 8 stays in the stack
    r10_off = -8 if through_stack else 1805
    return _prog("esc", [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 34),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.st(size, 10, r10_off, 0xAB),
        A.jmp("jeq", 2, 0, "out"),
        A.ldx(size, 0, 2, off),
        A.ldx(1, 5, 2, off + 1),
        A.alu64("lsh", 0, 8),
        A.alu64("or", 0, 5, reg=True),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ])


def _escape_scenarios():
    return [Scenario(vcpus=4, progs=[_escape_prog(12, s, st)]) for s in (1, 2, 4) for st in (False, True)]


@pytest.mark.parametrize("k", range(6))
def test_early_load_voided_by_stack_escape(gpu, k):
    sc = _escape_scenarios()[k]
    n = 2048
    buf, off, lens = W.make_packets(n, sizes=(64, 128), weights=(1, 1))
    cpu = W.schedule_cpu(n, 4, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert e["last_exec"] == "jit"


# ---------------------------------------------------------------------------------------------
# inline hash-map lookups: key sizes around the 8-byte words and the 32-byte limit, keys at odd
# stack offsets, partly unwritten keys (unwritten stack bytes read as zero), per-CPU hash maps
# ---------------------------------------------------------------------------------------------
HASH_CASES = [(1, 1, 4), (1, 3, 5), (1, 4, 8), (1, 8, 9), (1, 12, 16), (1, 16, 21), (1, 20, 24), (1, 32, 40),
              (1, 33, 40), (1, 40, 48), (5, 4, 8), (5, 16, 19)]


def _hash_prog(K, ko):
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 8),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(4, 7, 2, 0),
        A.alu64("and", 7, 0x3F),               # 64 distinct keys
        A.stx(1, 10, -ko, 7),                  # key byte 0 ...
    ]
    if K >= 4:
        items.append(A.stx(2, 10, -ko + 2, 7))  # ... bytes 2-3; byte 1 stays unwritten (zero)
    if K >= 12:
        items += [A.mov64_reg(8, 7), A.alu64("xor", 8, 0x55), A.stx(4, 10, -ko + 8, 8)]
    items += [
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -ko),
        A.ld_map_fd(1, "h"),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "miss"),
        A.ldx(8, 0, 0, 0),
        A.exit_(),
        "miss",
        A.mov64_imm(0, 0xFFFF),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    return _prog("hl", items)


def _key_of(v, K):
    b = bytearray(K)
    b[0] = v & 0xFF
    if K >= 4:
        b[2] = v & 0xFF
        b[3] = 0
    if K >= 12:
        w = (v ^ 0x55).to_bytes(4, "little")
        b[8:12] = w
    return bytes(b)


def _hash_scenario(mtype, K, ko):
    m = dict(name="h", type=mtype, key_size=K, value_size=8, max_entries=64)
    init = []
    for v in range(0, 64, 2):          # every other key present: hits and misses
        cpus = range(4) if mtype == 5 else [0]
        for c in cpus:
            init.append(("h", _key_of(v, K), (v * 1000 + c + 7).to_bytes(8, "little"), c))
    return Scenario(vcpus=4, maps=[m], progs=[_hash_prog(K, ko)], map_init=init)


@pytest.mark.parametrize("mtype,K,ko", HASH_CASES)
def test_inline_hash_lookup(gpu, mtype, K, ko):
    sc = _hash_scenario(mtype, K, ko)
    n = 4096
    buf, off, lens = W.make_packets(n)
    cpu = W.schedule_cpu(n, 4, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    hits = (o["r0"] != 0xFFFF) & (o["r0"] != 2)
    assert hits.any() and (~hits).any()


def test_inline_hash_lookup_unset_cpu(gpu):
    """Per-CPU hash lookups from a process whose CPU ID is unset (-1) fail in the helper: the
    inline form must leave them to the generic path."""
    sc = _hash_scenario(5, 8, 9)
    n = 512
    buf, off, lens = W.make_packets(n)
    cpu = np.where(np.arange(n) % 3 == 0, -1, np.arange(n) % 4).astype(np.int32)
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert (o["status"] != 0).any()


# ---------------------------------------------------------------------------------------------
# inline tail calls: a program slot, an empty slot, an index past max_entries, a self-call loop
# that runs out of the tail-call budget, and a prog-array pointer that is not the exact object
# ---------------------------------------------------------------------------------------------
def _tail_progs(r2_bump):
    entry = [
        A.mov64_reg(6, 1),
        A.ldx(4, 7, 6, 0),
        A.ldx(4, 8, 6, 4),
        A.mov64_reg(4, 7),
        A.alu64("add", 4, 1),
        A.jmp("jgt", 4, 8, "out", reg=True),
        A.ldx(1, 9, 7, 0),
        A.alu64("and", 9, 7),
        A.mov64_reg(1, 6),
        A.ld_map_fd(2, "progs"),
    ]
    if r2_bump:
        entry.append(A.alu64("add", 2, r2_bump))
    entry += [
        A.mov64_reg(3, 9),
        A.call(A.FN_TAIL_CALL),
        A.mov64_reg(0, 9),
        A.alu64("add", 0, 100),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    other = [A.mov64_imm(0, 7), A.alu64("add", 0, 9, reg=True), A.exit_()]
    return [_prog("entry", entry), _prog("other", other)]


def _tail_scenario(bump):
    # slots: 0 -> other, 1 empty, 2 -> entry (loops until the budget is spent), 3 -> other;
    # indexes 4..7 lie past max_entries
    return Scenario(vcpus=4, maps=[dict(name="progs", type=3, key_size=4, value_size=4, max_entries=4)],
                    progs=_tail_progs(bump), prog_array=[("progs", 0, 1), ("progs", 2, 0), ("progs", 3, 1)],
                    max_tail_calls=9)


@pytest.mark.parametrize("bump", [0, 3])
def test_inline_tail_calls(gpu, bump):
    sc = _tail_scenario(bump)
    n = 2048
    buf, off, lens = W.make_packets(n)
    cpu = W.schedule_cpu(n, 4, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert len(set(o["r0"].tolist())) >= 5


# ---------------------------------------------------------------------------------------------
# sk_buff: flow-keys and sock pointer accesses at every offset and size (including read-only
# fields, slices that panic and offsets past the object, which take the generic path)
# ---------------------------------------------------------------------------------------------
def _ptr_cases():
    cases = []
    for o in list(range(0, 44, 1)):
        for n in (1, 2, 4, 8):
            cases.append(("fk", o, n, True))
            cases.append(("fk", o, n, False))
    for o in list(range(0, 84, 2)):
        for n in (1, 4):
            cases.append(("sk", o, n, True))
    for o in (0, 16, 20, 3):
        cases.append(("sk", o, 4, False))
    return cases


def _ptr_prog(kind, o, n, load):
    field = S["flow_keys"] if kind == "fk" else S["sk"]
    items = [A.mov64_reg(6, 1), A.ldx(4, 1, 6, field)]
    if load:
        items += [A.ldx(n, 0, 1, o)]
    else:
        items += [A.mov64_imm(3, 0x1234567), A.stx(n, 1, o, 3), A.ldx(n, 0, 1, o & ~(n - 1))]
    items += [A.exit_()]
    return _prog(f"{kind}_{o}_{n}_{int(load)}", items)


def _ptr_groups(per=40):
    cs = _ptr_cases()
    return [cs[a:a + per] for a in range(0, len(cs), per)]


def _ptr_scenario(group):
    return Scenario(vcpus=2, progs=[_ptr_prog(*c) for c in group])


@pytest.mark.parametrize("g", range(len(_ptr_groups())))
def test_flow_keys_and_sock_accesses(gpu, g):
    sc = _ptr_scenario(_ptr_groups()[g])
    buf, off, lens = W.make_skb_packets(8, sizes=(64, 90), weights=(1, 1))
    cpu = np.zeros(8, np.int32)
    runs = [dict(skb=True, buf=buf, off=off, lens=lens, cpu=cpu, entry=k, ifindex=1) for k in range(len(sc.progs))]
    o = run_sequence_oracle(sc, runs)
    e = run_sequence_engine(sc, runs)
    assert_same_sequence(o, e, tag=f"group {g}")


# ---------------------------------------------------------------------------------------------
# sk_buff: early LD_ABS / LD_IND -- the index register changes, and a packet store sits between
# ---------------------------------------------------------------------------------------------
def _ldabs_prog(store):
    items = [
        A.mov64_reg(6, 1),
        A.ld_abs(1, 14),
        A.mov64_reg(7, 0),
        A.alu64("and", 7, 0x0F),
        A.alu64("lsh", 7, 2),
        A.jmp("jlt", 7, 20, "bad"),
        A.ld_abs(1, 23),
        A.mov64_reg(9, 0),
        A.stx(4, 10, -4, 0),
    ]
    if store:   # rewrite packet byte 23 (the protocol) through skb->data, BigEndian memory
        items += [A.ldx(4, 2, 6, S["data"]), A.ldx(4, 3, 6, S["data_end"]), A.mov64_reg(4, 2), A.alu64("add", 4, 24),
                  A.jmp("jgt", 4, 3, "bad", reg=True), A.st(1, 2, 23, 0x5A)]
    items += [
        A.ld_ind(2, 7, 14),
        A.mov64_reg(8, 0),
        A.alu64("add", 7, 2),
        A.jmp("jeq", 8, 0, "skip"),
        A.ld_ind(2, 7, 14),
        A.alu64("xor", 8, 0, reg=True),
        "skip",
        A.ld_abs(1, 23),
        A.alu64("lsh", 8, 8),
        A.alu64("or", 8, 0, reg=True),
        A.alu64("lsh", 8, 8),
        A.alu64("or", 8, 9, reg=True),
        A.mov64_reg(0, 8),
        A.exit_(),
        "bad",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    return _prog("ldabs", items)


@pytest.mark.parametrize("store", [False, True])
def test_early_ld_abs(gpu, store):
    sc = Scenario(vcpus=4, progs=[_ldabs_prog(store)])
    n = 4096
    buf, off, lens = W.make_skb_packets(n, **W.IMIX, variety=0.3)
    cpu = W.schedule_cpu(n, 4, "interleaved")
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=1)
    e = run_engine_skb(sc, buf, off, lens, cpu, ifindex=1)
    assert_same(o, e)
    assert e["last_exec"] == "jit"


# ---------------------------------------------------------------------------------------------
# cross-packet window prefetch (analyze_xpf, MIMIC_JIT_XPF=1, off by default: measured slower):
# packet j + 1's first header window is loaded while packet j runs.  Short packets, per-packet headroom, a base of data + c, packet stores followed
# by a tail call back into the entry program (which must reread the stored bytes), and every
# schedule must give the oracle's results.
# ---------------------------------------------------------------------------------------------
def _xpf_prog(c=0, tail=False):
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
    ]
    if c:
        items.append(A.alu64("add", 4, c))
    base = 4 if c else 2
    items += [
        A.mov64_reg(0, 2),
        A.alu64("add", 0, 40),
        A.jmp("jgt", 0, 3, "out", reg=True),
        A.ldx(2, 5, base, 12),
        A.ldx(4, 7, base, 14),
        A.jmp("jeq", 5, 0xFFFF, "out"),
        A.ldx(4, 8, base, 20),
        A.alu64("xor", 7, 8, reg=True),
        A.alu64("xor", 7, 5, reg=True),
    ]
    if tail:   # bump byte 12 of the window, then re-enter this program through the prog array
        items += [
            A.mov64_reg(9, 5),
            A.alu64("add", 9, 1),
            A.stx(1, base, 12, 9),
            A.mov64_reg(1, 6),
            A.ld_map_fd(2, "progs"),
            A.mov64_reg(3, 7),
            A.alu64("and", 3, 1),
            A.call(A.FN_TAIL_CALL),
        ]
    items += [
        A.mov64_reg(0, 7),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    return _prog("xw", items)


XPF_CASES = [(0, False), (14, False), (0, True), (6, True)]


def _xpf_scenario(c, tail):
    if not tail:
        return Scenario(vcpus=8, progs=[_xpf_prog(c)])
    return Scenario(vcpus=8, maps=[dict(name="progs", type=3, key_size=4, value_size=4, max_entries=2)],
                    progs=[_xpf_prog(c, True)], prog_array=[("progs", 0, 0), ("progs", 1, 0)], max_tail_calls=3)


@pytest.mark.parametrize("case", range(len(XPF_CASES)))
@pytest.mark.parametrize("room", ["none", "uniform", "per_packet"])
@pytest.mark.parametrize("sched", ["interleaved", "chunked", "explicit"])
def test_cross_packet_window_prefetch(gpu, case, room, sched, monkeypatch):
    monkeypatch.setenv("MIMIC_JIT_XPF", "1")
    sc = _xpf_scenario(*XPF_CASES[case])
    import mimic_amd as M
    from mimic_amd import jit as J

    assert "xpf_on_" in J.kernel_source(*kernel_of(sc))
    n = 3000
    rng = np.random.default_rng(case)
    headroom = {"none": 0, "uniform": 16, "per_packet": rng.integers(0, 4, n) * 8}[room]
    tailroom = 8 if room == "uniform" else 0
    pkts = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.choice([20, 36, 40, 41, 60, 64, 128], n)]
    buf, off, lens = packets_to_buffer(pkts, headroom, tailroom)
    mode = {"interleaved": M.SCHED_INTERLEAVED, "chunked": M.SCHED_CHUNKED, "explicit": M.SCHED_EXPLICIT}[sched]
    cpu = rng.integers(0, 8, n).astype(np.int32) if sched == "explicit" else W.schedule_cpu(n, 8, sched)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=headroom, tailroom=tailroom)
    e = run_engine(sc, buf, off, lens, cpu if sched == "explicit" else None, headroom=headroom, tailroom=tailroom,
                   schedule=mode, spread=0)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
    assert len(set(o["r0"].tolist())) > 100


@pytest.mark.parametrize("case", [0, 1])
@pytest.mark.parametrize("room", ["none", "uniform", "per_packet"])
@pytest.mark.parametrize("sched", ["interleaved", "chunked", "explicit"])
@pytest.mark.parametrize("V", [400, 700])
def test_lane_prefetch(gpu, case, room, sched, V, monkeypatch):
    """Lane prefetch (jit.cpp lpf_on, MIMIC_JIT_LPF=1: off by default, measured slower on cfg 2; for
    xdp_md program sets that never store into packet memory): a lane's first 4 packets' descriptors and early windows are loaded when the lane
    starts and parked in LDS.  Every schedule, rooms (prefetch off at run time), short packets
    (window past the packet), lanes with fewer and with more than 4 packets (V = 700 / 400; fewer
    than 8 packets per vCPU, so no spread launch): oracle-exact.  The
    windowed program of XPF_CASES without the packet store (case 0: window at data + 12, case 1:
    data + 26)."""
    monkeypatch.setenv("MIMIC_JIT_LPF", "1")
    items_c = XPF_CASES[case][0]
    sc = Scenario(vcpus=V, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=4)],
                  progs=[_lpf_prog(items_c)])
    import mimic_amd as M
    from mimic_amd import jit as J

    assert "lpf_n_" in J.kernel_source(*kernel_of(sc))
    n = 3000
    rng = np.random.default_rng(case + 7)
    headroom = {"none": 0, "uniform": 16, "per_packet": rng.integers(0, 4, n) * 8}[room]
    tailroom = 8 if room == "uniform" else 0
    pkts = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.choice([20, 36, 40, 41, 60, 64, 128], n)]
    buf, off, lens = packets_to_buffer(pkts, headroom, tailroom)
    mode = {"interleaved": M.SCHED_INTERLEAVED, "chunked": M.SCHED_CHUNKED, "explicit": M.SCHED_EXPLICIT}[sched]
    cpu = rng.integers(0, V, n).astype(np.int32) if sched == "explicit" else W.schedule_cpu(n, V, sched)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=headroom, tailroom=tailroom)
    e = run_engine(sc, buf, off, lens, cpu if sched == "explicit" else None, headroom=headroom, tailroom=tailroom,
                   schedule=mode, spread=0)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
    assert len(set(o["r0"].tolist())) > 100


def test_lane_prefetch_needs_packet_memory_untouched(monkeypatch):
    """A program set that may store into packet memory (a store through a packet pointer, or
    through a base the analysis cannot place) gets no lane prefetch."""
    from mimic_amd import jit as J

    monkeypatch.setenv("MIMIC_JIT_LPF", "1")
    sc = _xpf_scenario(0, True)
    assert "lpf_n_" not in J.kernel_source(*kernel_of(sc))   # _xpf_prog(tail) stores into the packet
    assert "lpf_n_" in J.kernel_source(*kernel_of(Scenario(vcpus=8, maps=[dict(name="c", type=6, key_size=4,
                                                                                value_size=8, max_entries=4)],
                                                            progs=[_lpf_prog(0)])))


def _lpf_prog(c):
    """Reads a window of packet bytes at data + 12 + c (early loads), folds them into R0 and a
    per-CPU counter[r0 & 3] += 1; no store into the packet."""
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 24 + c),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(2, 7, 2, 12 + c),
        A.ldx(4, 8, 2, 14 + c),
        A.ldx(1, 9, 2, 21 + c),
        A.alu64("lsh", 8, 8),
        A.alu64("xor", 7, 8, reg=True),
        A.alu64("add", 7, 9, reg=True),
        A.mov64_reg(5, 7),
        A.alu64("and", 5, 3),
        A.stx(4, 10, -4, 5),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -4),
        A.ld_map_fd(1, "c"),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, 3),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
        A.mov64_reg(0, 7),
        A.exit_(),
        "out",
        A.mov64_imm(0, 2),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return ("lpf", raw, rel)


# ---------------------------------------------------------------------------------------------
# LDS stack window (runtime.h, MIMIC_LDS_STACK_Q): frame 0's top 128 bytes live in LDS, the rest
# of the stack in HBM.  Stores and loads of every size at offsets around the window's lower edge
# (R10 - 128), unaligned and straddling it, never-written bytes (read as zero), a stack address
# read back through another register (the generic path), and a BPF-to-BPF call (frame 1 above).
# ---------------------------------------------------------------------------------------------
def _stack_window_prog(variant):
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 16),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(8, 7, 2, 0),
        A.ldx(8, 8, 2, 8),
        A.mov64_imm(0, 0),
    ]
    offs = [-140, -136, -133, -131, -130, -129, -128, -127, -125, -121, -120, -117, -8, -3, -256]
    for k, o in enumerate(offs):
        n = (1, 2, 4, 8)[(k + variant) % 4]
        items += [A.stx(n, 10, o, 7 if k % 2 else 8), A.alu64("rsh", 7, 3), A.alu64("add", 8, 0x1357)]
    for k, o in enumerate(offs + [-144, -200, -64]):   # read back with other sizes / alignments
        n = (8, 4, 2, 1)[(k + variant) % 4]
        o2 = o - (k % 3)
        if o2 < -256:
            o2 = -256
        items += [A.ldx(n, 5, 10, o2), A.alu64("xor", 0, 5, reg=True), A.alu64("lsh", 0, 1)]
    items += [A.mov64_reg(9, 10), A.alu64("add", 9, -130), A.ldx(4, 5, 9, 0), A.alu64("add", 0, 5, reg=True),
              A.stx(2, 9, 1, 0), A.ldx(8, 5, 10, -136), A.alu64("xor", 0, 5, reg=True)]
    if variant == 1:   # a BPF-to-BPF call: the callee's frame lies above the window
        items += [A.mov64_reg(1, 0), A.call("sub"), A.alu64("xor", 0, 1, reg=True)]
    items += [A.exit_(), "out", A.mov64_imm(0, 2), A.exit_()]
    if variant == 1:
        items += ["sub", A.stx(8, 10, -128, 1), A.stx(1, 10, -129, 1), A.ldx(8, 0, 10, -129), A.ldx(8, 2, 10, -8),
                  A.alu64("add", 0, 2, reg=True), A.exit_()]
    return _prog("stkw", items)


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_lds_stack_window(gpu, variant):
    from mimic_amd import jit as J

    sc = Scenario(vcpus=4, progs=[_stack_window_prog(variant)])
    assert "MIMIC_LDS_STACK_Q" in J.kernel_source(*kernel_of(sc))
    n = 2048
    buf, off, lens = W.make_packets(n, sizes=(14, 64, 128), weights=(1, 2, 2))
    cpu = W.schedule_cpu(n, 4, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
    assert len(set(o["r0"].tolist())) > 1000


# ---------------------------------------------------------------------------------------------
# fused counter increments (jit.cpp fusable_inc): ldx / add / stx on a map value as one atomic add,
# read back at once (the lane must see its own add), 8- and 4-byte (ALU32) forms, an unaligned
# word (falls back to the three slots), and a register still live after the store (not fused)
# ---------------------------------------------------------------------------------------------
def _inc_prog(variant):
    o8 = 4 if variant == 2 else 0      # variant 2: the 8-byte counter is unaligned -> fallback
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),
        A.ldx(4, 3, 6, 4),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 1),
        A.mov64_imm(0, 1),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(1, 7, 2, 0),
        A.alu64("and", 7, 3),
        A.stx(4, 10, -4, 7),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -4),
        A.ld_map_fd(1, "cnt"),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "out"),
        A.ldx(8, 1, 0, o8),
        A.alu64("add", 1, 1),
        A.stx(8, 0, o8, 1),
        A.ldx(8, 8, 0, o8),                # read back after the add
        A.ldx(4, 5, 0, 8),
        A.alu32("add", 5, 7),
        A.stx(4, 0, 8, 5),
    ]
    if variant == 3:
        items += [A.alu64("add", 8, 5, reg=True)]   # r5 read after its store: not fused
    items += [
        A.ldx(4, 9, 0, 8),
        A.alu64("lsh", 8, 32),
        A.alu64("or", 8, 9, reg=True),
        A.mov64_reg(0, 8),
        "out",
        A.exit_(),
    ]
    return _prog("inc", items)


def _inc_scenario(variant):
    mtype = 2 if variant == 1 else 6   # variant 1: a plain (shared) array, one vCPU
    return Scenario(vcpus=1 if variant == 1 else 4, progs=[_inc_prog(variant)],
                    maps=[dict(name="cnt", type=mtype, key_size=4, value_size=16, max_entries=4)])


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_fused_counter_increments(gpu, variant):
    from mimic_amd import jit as J

    sc = _inc_scenario(variant)
    src = J.kernel_source(*kernel_of(sc))
    # the fused form: an atomic add in the lookup's value region; for the per-CPU array (a 64-byte
    # row: the lane value cache's LDS form) an LDS add first when the row is cached
    assert src.count("CNT_ADD(L.t_ptr") == {0: 2, 1: 2, 2: 2, 3: 1}[variant], src
    assert src.count("lvc_add(lvt_") == {0: 2, 1: 0, 2: 2, 3: 1}[variant], src
    n = 4096
    buf, off, lens = W.make_packets(n, sizes=(14, 64), weights=(1, 3))
    cpu = W.schedule_cpu(n, sc.vcpus, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert e["last_exec"] == "jit"
    assert len(set(o["r0"].tolist())) > 100


def jit_kernels():
    ks = [kernel_of(Scenario(vcpus=4, progs=[_stack_window_prog(v)])) for v in range(4)]
    ks += [kernel_of(_inc_scenario(v)) for v in range(4)]
    ks += [kernel_of(sc) for sc in _escape_scenarios()]
    ks += [kernel_of(_hash_scenario(*c)) for c in HASH_CASES]
    ks += [kernel_of(_tail_scenario(b)) for b in (0, 3)]
    ks += [kernel_of(_ptr_scenario(g), ctx=1) for g in _ptr_groups()]
    ks += [kernel_of(Scenario(vcpus=4, progs=[_ldabs_prog(s)]), ctx=1) for s in (False, True)]
    return ks
