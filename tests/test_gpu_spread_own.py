"""Owned spread launches on MI355X (jit.cpp spread_own, engine.cpp spread_build_own): block b runs
every packet of vCPU lanes [b * 256 / P, +256 / P) (P = packets per vCPU, 2..256) at once, its fused
counter increments into an LDS table that it then adds into the rows only it touches.  For program
sets whose only per-CPU state is counters they increment (analyze_spread), every run is compared
with the oracle running each vCPU's packets in order (processPool, vm.go:548-573): per packet R0 /
status / steps / err_pc, every (cpu, key) counter, the total step count."""
import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, assert_same, build_engine, kernel_of, run_engine, run_oracle, spread_kernel_of
from mimic_amd import workloads as W
from test_gpu_spread import _check, _counter_prog, _peek_sc, _sc

pytestmark = pytest.mark.gpu


@pytest.fixture
def own(monkeypatch):
    monkeypatch.setenv("MIMIC_SPREAD_OWN", "1")


def jit_kernels():
    out = [spread_kernel_of(_sc(W.prog_classifier(), 4), own=True),
           spread_kernel_of(_sc(W.prog_parse5(), 4), own=True),
           spread_kernel_of(_sc(_counter_prog(4), 4), own=True),
           kernel_of(_sc(_counter_prog(8, leak=True), 1)), kernel_of(_peek_sc(128))]
    return out


@pytest.mark.parametrize("V,n", [(262144, 1 << 20), (50000, 100003), (4096, 100003), (1000, 256000), (1000, 100003),
                                 (65536, 131077), (7, 14)])
@pytest.mark.parametrize("sched", ["interleaved", "chunked"])
def test_classifier(gpu, own, V, n, sched):
    """P = 4 (cfg 2's shape), 3 (ragged), 25, 256, 101, 3 (two packets past 2 V) and 2."""
    p = W.prog_classifier()
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 40, 20), weights=(6, 1, 1), seed=V + n)
    cpu = W.schedule_cpu(n, V, sched)
    o = run_oracle(sc, buf, off, lens, cpu)
    mode = M.SCHED_INTERLEAVED if sched == "interleaved" else M.SCHED_CHUNKED
    e = run_engine(sc, buf, off, lens, None, schedule=mode)
    assert e["last_exec"] == "spread_own"
    _check(o, e, sc)
    assert sum(int(np.frombuffer(v, np.uint64).sum()) for v in e["maps"]["verdicts"]) == n


def test_parse5_two_kib_rows(gpu, own):
    """2 KiB rows: a 16-row table, so P >= 16 (here 74)."""
    p = W.prog_parse5()
    V, n = 4096, 300000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=5)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "spread_own"
    _check(o, e, sc)


def test_parse5_rows_too_long_for_few_packets(gpu, own):
    """P = 4 would need 64 rows of 2 KiB: the one-lane kernel runs it."""
    p = W.prog_parse5()
    V, n = 4096, 16384
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=6)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "jit"
    _check(o, e, sc)


def test_four_byte_counters(gpu, own):
    p = _counter_prog(4)
    V, n = 4096, 40000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 65, 66, 67), weights=(1, 1, 1, 1), seed=4)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "spread_own"
    _check(o, e, sc)


def test_refused_programs_run_one_lane_per_vcpu(gpu, own):
    """The counter leaked into R0, and a computed address into per-CPU memory: both keep one lane
    per vCPU and stay exact."""
    p = _counter_prog(8, leak=True)
    V, n = 4096, 16384
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 65), weights=(1, 1), seed=8)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "jit"
    _check(o, e, sc)
    sc = _peek_sc(128)
    n = 512
    buf, off, lens = W.make_packets(n, seed=13)
    cpu = W.schedule_cpu(n, 128, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu, entry=1)
    e = run_engine(sc, buf, off, lens, None, entry=1, schedule=M.SCHED_INTERLEAVED)
    assert e["last_exec"] == "jit"
    assert_same(o, e)


def test_shard(gpu, own):
    """Two engines owning vCPUs [0, 2048) and [2048, 4096) (VMOptShard): each block's rows are
    offset by the shard's first vCPU; together one oracle run."""
    p = W.prog_classifier()
    V, n = 4096, 20000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, seed=11)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    for r in range(2):
        b0 = 2048 * r
        sel = np.nonzero((cpu >= b0) & (cpu < b0 + 2048))[0]
        vm, maps, pids = build_engine(sc, shard=(b0, 2048))
        batch = M.XDPBatch.from_numpy(buf, off[sel], lens[sel], device="cuda:0", schedule=M.SCHED_INTERLEAVED)
        e = vm.RunXDPBatch(pids[0], batch).numpy(len(sel))
        assert vm.LastExec() == "spread_own"
        for k in ("r0", "status", "steps"):
            assert np.array_equal(np.asarray(o[k])[sel].astype(np.int64), np.asarray(e[k]).astype(np.int64)), (r, k)
        for c in range(b0, b0 + 2048):
            assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c], c
        vm.close()


def test_host_resident_sub_batches(gpu, own):
    """RunXDPHost's sub-batches continue the interleaved schedule (sched_shift): P of each sub-batch
    counts the shift."""
    p = W.prog_classifier()
    V, n = 4096, 300000
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, seed=12)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    vm, maps, pids = build_engine(sc)
    r0, st = vm.RunXDPHost(pids[0], buf, off, lens, schedule=M.SCHED_INTERLEAVED, chunks=5)
    assert vm.LastExec() == "spread_own"
    assert np.array_equal(np.asarray(o["r0"]).astype(np.uint64), r0)
    assert np.array_equal(np.asarray(o["status"]).astype(np.uint8), st)
    for c in range(V):
        assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c], c
    vm.close()


def test_repeated_launches_accumulate(gpu, own):
    """The rows a block adds into keep what earlier launches counted: three launches of one batch."""
    p = W.prog_classifier()
    V, n = 65536, 262144
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, seed=21)
    cpu = W.schedule_cpu(n, V, "interleaved")
    cpu3 = np.concatenate([cpu] * 3)
    buf3, off3, lens3 = buf, np.concatenate([off] * 3), np.concatenate([lens] * 3)
    o = run_oracle(sc, buf3, off3, lens3, cpu3)
    vm, maps, pids = build_engine(sc)
    batch = M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", schedule=M.SCHED_INTERLEAVED)
    for _ in range(3):
        vm.RunXDPBatch(pids[0], batch)
        assert vm.LastExec() == "spread_own"
    for c in range(0, V, 97):
        assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c], c
    vm.close()


@pytest.mark.parametrize("q", [2, 4, 8])
@pytest.mark.parametrize("sched", ["interleaved", "chunked"])
def test_packets_per_thread(gpu, own, monkeypatch, q, sched):
    """Q packets per thread (KParams::own_q; MIMIC_SPREAD_OWN_Q fixes it): R = 256 Q / P lanes per
    block, each thread its lane's packets j, j + P / Q, ... in order; P = 16, ragged last lanes."""
    monkeypatch.setenv("MIMIC_SPREAD_OWN_Q", str(q))
    p = W.prog_classifier()
    V, n = 4096, 65536 - 77
    sc = _sc(p, V)
    buf, off, lens = W.make_packets(n, sizes=(64, 40, 20), weights=(6, 1, 1), seed=q)
    cpu = W.schedule_cpu(n, V, sched)
    o = run_oracle(sc, buf, off, lens, cpu)
    mode = M.SCHED_INTERLEAVED if sched == "interleaved" else M.SCHED_CHUNKED
    e = run_engine(sc, buf, off, lens, None, schedule=mode)
    assert e["last_exec"] == "spread_own"
    _check(o, e, sc)
