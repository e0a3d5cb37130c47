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


def jit_kernels():
    out = []
    for V in (1, 7, 256, 1000, 4096):
        out.append(spread_kernel_of(_sc(W.prog_classifier(), V)))
    for V in (64, 256):
        out.append(spread_kernel_of(_sc(W.prog_parse5(), V)))
    out.append(spread_kernel_of(_sc(_counter_prog(4), 256)))
    out.append(spread_kernel_of(_sc(W.prog_classifier(), 128)))
    out.append(kernel_of(_sc(_counter_prog(8, leak=True), 1)))
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


def test_computed_address_into_per_cpu_memory_fails_loudly(gpu):
    """An address the program computes (an LD_IMM64 constant) into the counters: the analysis
    cannot see it, the generic load reaches resolve(), and the launch is reported as an engine
    error instead of returning a result that depends on the lanes' interleaving."""
    p = W.prog_classifier()
    V = 128
    sc = _sc(p, V)
    vm, maps, pids = build_engine(sc)
    addr = maps["verdicts"].Lookup((1).to_bytes(4, "little"), 3)
    assert addr
    raw, rel = A.assemble([
        A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "verdicts"),
        A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, 3), A.ldx(8, 1, 0, 0), A.alu64("add", 1, 1), A.stx(8, 0, 0, 1),
        A.ld_imm64(3, addr), A.ldx(8, 0, 3, 0), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("peek", raw, list(rel)))
    n = 50000
    buf, off, lens = W.make_packets(n, seed=13)
    batch = M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", schedule=M.SCHED_INTERLEAVED)
    with pytest.raises(M.MimicError, match="spread launch"):
        vm.RunXDPBatch(pid, batch)
    vm.close()
