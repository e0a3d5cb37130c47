"""Spread launches on MI355X (jit.cpp analyze_spread, engine.cpp spread_build): a vCPU's packets
on many lanes, for program sets whose only per-CPU state is counters they increment.  Every run
is compared with the oracle running each vCPU's packets in order on one worker per vCPU
(processPool, vm.go:548-573): per packet R0 / status / steps / err_pc, every (cpu, key) counter,
the total step count.  V = 256 is the reference's default VirtualCPUs on a 256-thread host
(runtime.NumCPU(), vm.go:64)."""
import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, assert_same, build_engine, kernel_of, run_engine, run_oracle, spread_kernel_of
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _table_spread(monkeypatch):
    """This module tests the table spread kernel: the owned form (test_gpu_spread_own.py), which
    takes batches of up to 256 packets per vCPU by default, is kept off."""
    monkeypatch.setenv("MIMIC_SPREAD_OWN", "0")


def _sc(p, V):
    return Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def _counter_prog(size=8, leak=False):
    """Per-CPU counter[packet length & 3] += 1 (a 4-byte form with ALU32); leak=True returns the
    counter's value in R0 -- a program the analysis must refuse."""
    items = [A.mov64_reg(6, 1), A.ldx(4, 2, 6, 0), A.ldx(4, 3, 6, 4), A.mov64_reg(4, 3), A.alu64("sub", 4, 2, reg=True),
             A.alu64("and", 4, 3), A.stx(4, 10, -4, 4), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "c"),
             A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, "out")]
    if leak:
        items += [A.ldx(size, 7, 0, 0), A.alu64("add", 7, 1), A.stx(size, 0, 0, 7), A.mov64_reg(0, 7), A.exit_()]
    elif size == 4:
        items += [A.ldx(4, 7, 0, 0), A.alu32("add", 7, 1), A.stx(4, 0, 0, 7)]
    else:
        items += [A.ldx(8, 7, 0, 0), A.alu64("add", 7, 1), A.stx(8, 0, 0, 7)]
    items += ["out", A.mov64_imm(0, 2), A.exit_()]
    raw, rel = A.assemble(items)
    return W.Program(f"cnt{size}{'leak' if leak else ''}", raw, rel,
                     [dict(name="c", type=6, key_size=4, value_size=size, max_entries=4)])


def _peek_sc(V):
    """The classifier plus a program that bumps per-CPU counter[1], then reads the same counter back
    through a computed address: get_smp_processor_id * the row period + an LD_IMM64 constant (the
    addresses from the oracle's layout, which is the engine's: layout_* KATs).  Its R0 counts the
    vCPU's packets in order, so it is exact only when a vCPU's packets run in order."""
    from harness import build_oracle

    p = W.prog_classifier()
    base = Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    ovm, mids, _ = build_oracle(base)
    a0 = ovm.map_lookup(mids["verdicts"], (1).to_bytes(4, "little"), 0)[1]
    period = ovm.map_lookup(mids["verdicts"], (1).to_bytes(4, "little"), 1)[1] - a0
    ovm.close()
    assert a0 and period > 0
    raw, rel = A.assemble([
        A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "verdicts"),
        A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, 3), A.ldx(8, 1, 0, 0), A.alu64("add", 1, 1), A.stx(8, 0, 0, 1),
        A.call(A.FN_GET_SMP_PROCESSOR_ID), A.alu64("mul", 0, period), A.ld_imm64(3, a0), A.alu64("add", 3, 0, reg=True),
        A.ldx(8, 0, 3, 0), A.exit_()])
    return Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs), ("peek", raw, list(rel))])


def jit_kernels():
    out = []
    for V in (1, 7, 256, 1000, 4096):
        out.append(spread_kernel_of(_sc(W.prog_classifier(), V)))
    for V in (64, 256):
        out.append(spread_kernel_of(_sc(W.prog_parse5(), V)))
    out.append(spread_kernel_of(_sc(_counter_prog(4), 256)))
    out.append(spread_kernel_of(_sc(W.prog_classifier(), 128)))
    out.append(kernel_of(_sc(_counter_prog(8, leak=True), 1)))
    out.append(kernel_of(_peek_sc(128)))
    return out


def _check(o, e, sc):
    assert_same(o, e)
    assert e["steps_total"] == int(np.asarray(o["steps"]).astype(np.int64).sum())


def test_classifier_v256_one_million_packets(gpu):
    """cfg 2's classifier over 1 M x 64 B packets at V = 256 (4 096 packets per vCPU)."""
    p = W.prog_classifier()
    V, n = 256, 1 << 20
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "spread"
    _check(o, e, sc)
    assert sum(int(np.frombuffer(v, np.uint64).sum()) for v in e["maps"]["verdicts"]) == n


@pytest.mark.parametrize("V", [1, 7, 256, 1000, 4096])
@pytest.mark.parametrize("sched", ["interleaved", "chunked"])
def test_classifier_schedules_and_vcpu_counts(gpu, V, sched):
    """Blocks whose packets wrap around the vCPU lanes (V < 1024 packets per block), chunks that
    end inside a block, V not dividing n, one vCPU."""
    p = W.prog_classifier()
    n = 100003
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 40, 20), weights=(6, 1, 1), seed=V)
    cpu = W.schedule_cpu(n, V, sched)
    o = run_oracle(sc, buf, off, lens, cpu)
    mode = M.SCHED_INTERLEAVED if sched == "interleaved" else M.SCHED_CHUNKED
    e = run_engine(sc, buf, off, lens, None, schedule=mode, spread=1)
    assert e["last_exec"] == "spread"
    _check(o, e, sc)


@pytest.mark.parametrize("V", [64, 256])
def test_parse5_agent_atomics(gpu, V):
    """parse5's 2 KiB rows: no LDS table; every increment is an agent-scope atomic into the map."""
    p = W.prog_parse5()
    n = 300000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=V)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "spread"
    _check(o, e, sc)


def test_four_byte_counters(gpu):
    p = _counter_prog(4)
    V, n = 256, 200000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 65, 66, 67), weights=(1, 1, 1, 1), seed=4)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "spread"
    _check(o, e, sc)


def test_leaking_program_is_not_spread(gpu):
    """A program that returns the counter in R0 (its value depends on the vCPU's earlier packets):
    refused by the analysis, it runs one lane per vCPU even with spread forced, and stays exact."""
    p = _counter_prog(8, leak=True)
    V, n = 256, 100000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 65), weights=(1, 1), seed=8)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED, spread=1)
    assert e["last_exec"] == "jit"
    _check(o, e, sc)
    assert len(np.unique(e["r0"])) > 100   # the counters really reach R0


def test_shard_with_spread(gpu):
    """Two engines owning vCPUs [0, 128) and [128, 256) (VMOptShard), each spreading its packets:
    together one oracle run."""
    p = W.prog_classifier()
    V, n = 256, 200000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, seed=11)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    for r in range(2):
        b0 = 128 * r
        sel = np.nonzero((cpu >= b0) & (cpu < b0 + 128))[0]
        vm, maps, pids = build_engine(sc, shard=(b0, 128))
        batch = M.XDPBatch.from_numpy(buf, off[sel], lens[sel], device="cuda:0", schedule=M.SCHED_INTERLEAVED)
        e = vm.RunXDPBatch(pids[0], batch).numpy(len(sel))
        assert vm.LastExec() == "spread"
        for k in ("r0", "status", "steps"):
            assert np.array_equal(np.asarray(o[k])[sel].astype(np.int64), np.asarray(e[k]).astype(np.int64)), (r, k)
        for c in range(b0, b0 + 128):
            assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c], c
        vm.close()


def test_host_resident_sub_batches(gpu):
    """RunXDPHost's sub-batches continue the interleaved schedule (sched_shift) in spread launches."""
    p = W.prog_classifier()
    V, n = 128, 300000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, seed=12)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    vm, maps, pids = build_engine(sc)
    r0, st = vm.RunXDPHost(pids[0], buf, off, lens, schedule=M.SCHED_INTERLEAVED, chunks=5)
    assert vm.LastExec() == "spread"
    assert np.array_equal(np.asarray(o["r0"]).astype(np.uint64), r0)
    assert np.array_equal(np.asarray(o["status"]).astype(np.uint8), st)
    for c in range(V):
        assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c], c
    vm.close()


def test_computed_address_into_per_cpu_memory_runs_exact(gpu):
    """An address the program computes (an LD_IMM64 constant) into the per-CPU counters: the base
    has no provenance the spread analysis can place, so under the default policy the program set
    runs one lane per vCPU and the result is the oracle's (memory_controller.go:117-145 resolves any
    address); SPREAD_GUARD is never reached."""
    V = 128
    sc = _peek_sc(V)
    n = 50000
    buf, off, lens = W.make_packets(n, seed=13)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu, entry=1)
    e = run_engine(sc, buf, off, lens, None, entry=1, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "jit"
    assert_same(o, e)
    # R0 counts each vCPU's packets in order: 1, 2, 3 ... (a spread launch would interleave them)
    assert sorted(set(np.asarray(o["r0"]).tolist())) == list(range(1, -(-n // V) + 1))
