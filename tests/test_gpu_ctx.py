"""Run(ctx) on MI355X (vm.go:343-360, vm.go:548-573): contexts given to a batch are read by the
kernels (JIT, interpreter, spread) before each process's first step; a done one ends that process
with ctx.Err() after its context Load.  Every run is replayed on the oracle with the per-packet
context states the device saw (orc_xdp_batch.ctx_done): r0 / status / steps / err_pc, packet
memory and every map agree.  In-flight cancellation and deadlines: a context marked while the
batch runs stops each vCPU's remaining processes (a suffix of its schedule).  Process.Run(ctx)
suspends a running process at a deadline and continues it afterwards."""
import threading
import time

import numpy as np
import pytest
import torch

import mimic_amd as M
from harness import (Scenario, assert_same, build_engine, kernel_of, packets_to_buffer, run_engine, run_engine_skb,
                     run_oracle, run_oracle_skb, spread_kernel_of)
from mimic_amd import _lib
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu
CANCELED, DEADLINE = _lib.STATUS["ERR_CANCELED"], _lib.STATUS["ERR_DEADLINE"]


def _count_sc(V=8):
    """c[0] += 1 (per-CPU), a byte stored into the packet, r0 = packet length."""
    raw, rel = A.assemble([A.mov64_reg(6, 1), A.ldx(4, 7, 6, 0), A.ldx(4, 8, 6, 4), A.st(1, 7, 0, 0x5a),
                           A.st(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "c"),
                           A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, "out"), A.ldx(8, 3, 0, 0),
                           A.alu64("add", 3, 1), A.stx(8, 0, 0, 3), "out", A.mov64_reg(0, 8),
                           A.alu64("sub", 0, 7, reg=True), A.exit_()])
    return Scenario(vcpus=V, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=1)],
                    progs=[("cnt", raw, rel)])


def _loop_sc(V, K):
    """r7 counts to K in a loop, then c[0] += 1 (per-CPU); r0 = r7."""
    raw, rel = A.assemble([A.mov64_imm(7, 0), "top", A.alu64("add", 7, 1), A.jmp("jlt", 7, K, "top"),
                           A.st(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "c"),
                           A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, "out"), A.ldx(8, 3, 0, 0),
                           A.alu64("add", 3, 1), A.stx(8, 0, 0, 3), "out", A.mov64_reg(0, 7), A.exit_()])
    return Scenario(vcpus=V, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=1)],
                    progs=[("loop", raw, rel)])


K_LOOP = 50000


def jit_kernels():
    return [kernel_of(_count_sc()), kernel_of(_loop_sc(64, K_LOOP)), kernel_of(_pkt_loop_sc(64)),
            spread_kernel_of(_sc_cls(7))]


def _sc_cls(V):
    p = W.prog_classifier()
    return Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def _packets(n, seed=3):
    rng = np.random.default_rng(seed)
    pkts = [bytes(rng.integers(1, 255, int(L), dtype=np.uint8)) for L in rng.integers(14, 300, n)]
    buf, off, lens = packets_to_buffer(pkts, headroom=8, tailroom=8)
    buf[:] = np.where(buf == 0, 0x77, buf)   # non-zero rooms: Load zeroes them
    return buf, off, lens


def _states(ctxs):
    return np.array([0 if c is None else {None: 0, "context canceled": 1, "context deadline exceeded": 2}[c.Err()]
                     for c in ctxs], np.uint8)


@pytest.mark.parametrize("mode", ["jit", "interp"])
def test_canceled_before_the_batch(gpu, mode):
    sc = _count_sc()
    buf, off, lens = _packets(512)
    cpu = W.schedule_cpu(len(lens), sc.vcpus, "chunked")
    ctx = M.WithCancel()
    ctx.Cancel()
    e = run_engine(sc, buf, off, lens, cpu, headroom=8, tailroom=8, exec_mode=mode, ctx=ctx)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=8, tailroom=8, ctx_done=np.ones(len(lens), np.uint8))
    assert (e["status"] == CANCELED).all() and (e["steps"] == 0).all()
    assert_same(o, e)
    ctx.close()


@pytest.mark.parametrize("mode", ["jit", "interp"])
def test_per_packet_contexts(gpu, mode):
    """Background (None), live WithCancel, canceled, and past-deadline contexts mixed in one batch."""
    sc = _count_sc()
    buf, off, lens = _packets(600, seed=4)
    cpu = np.random.default_rng(1).integers(0, sc.vcpus, len(lens)).astype(np.int32)
    live, gone, late = M.WithCancel(), M.WithCancel(), M.WithTimeout(0.0)
    gone.Cancel()
    pick = np.random.default_rng(2).integers(0, 4, len(lens))
    ctxs = [[None, live, gone, late][k] for k in pick]
    e = run_engine(sc, buf, off, lens, cpu, headroom=8, tailroom=8, exec_mode=mode, ctx_per_packet=ctxs)
    done = _states(ctxs)
    assert set(np.unique(done)) == {0, 1, 2}
    o = run_oracle(sc, buf, off, lens, cpu, headroom=8, tailroom=8, ctx_done=done)
    assert_same(o, e)
    for c in (live, gone, late):
        c.close()


def test_per_packet_contexts_spread(gpu):
    """A batch the spread kernel would run (a vCPU's packets on many lanes) runs with contexts on
    the one-lane-per-vCPU variant with the context check, exactly."""
    sc = _sc_cls(7)
    buf, off, lens = W.make_packets(20000, sizes=(64, 128), weights=(1, 1))
    gone = M.WithCancel()
    gone.Cancel()
    ctxs = [gone if i % 5 == 2 else None for i in range(len(lens))]
    e = run_engine(sc, buf, off, lens, None, schedule=M.SCHED_INTERLEAVED, spread=1, ctx_per_packet=ctxs)
    assert e["last_exec"] == "jit"
    cpu = W.schedule_cpu(len(lens), 7, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu, ctx_done=_states(ctxs))
    assert (e["status"][2::5] == CANCELED).all()
    assert_same(o, e)
    gone.close()


def test_skb_per_packet_contexts(gpu):
    """sk_buff batches: a done context's process still loads (its entries leak), as in the oracle."""
    buf, off, lens = W.make_skb_packets(2048, **W.IMIX, variety=0.2)
    progs, maps, pa = W.skb_programs()
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(buf, off, lens)]
    sc = Scenario(vcpus=32, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa, map_init=init)
    cpu = W.schedule_cpu(len(lens), 32, "chunked")
    gone, late = M.WithCancel(), M.WithTimeout(0.0)
    gone.Cancel()
    ctxs = [[None, gone, None, late][i % 4] for i in range(len(lens))]
    e = run_engine_skb(sc, buf, off, lens, cpu, ifindex=2, ctx_per_packet=ctxs)
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=2, ctx_done=_states(ctxs))
    assert_same(o, e)
    assert (e["status"][1::4] != 0).all()
    gone.close()
    late.close()


def _pkt_loop_sc(V):
    """r7 counts to the packet's first u32 in a loop, then c[0] += 1 (per-CPU); r0 = r7."""
    raw, rel = A.assemble([A.ldx(4, 2, 1, 0), A.ldx(4, 3, 2, 0), A.mov64_imm(7, 0), "top", A.alu64("add", 7, 1),
                           A.jmp("jlt", 7, 3, "top", reg=True), A.st(4, 10, -4, 0), A.mov64_reg(2, 10),
                           A.alu64("add", 2, -4), A.ld_map_fd(1, "c"), A.call(A.FN_MAP_LOOKUP_ELEM),
                           A.jmp("jeq", 0, 0, "out"), A.ldx(8, 3, 0, 0), A.alu64("add", 3, 1), A.stx(8, 0, 0, 3),
                           "out", A.mov64_reg(0, 7), A.exit_()])
    return Scenario(vcpus=V, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=1)],
                    progs=[("pktloop", raw, rel)])


K_SHORT, K_LONG = 100, (1 << 31) + 5   # a long process runs >= 2^31 loop iterations: seconds on any lane


@pytest.mark.parametrize("mode,kind", [("jit", "cancel"), ("jit", "deadline"), ("interp", "cancel")])
def test_done_while_the_batch_runs(gpu, mode, kind):
    """Each lane (chunked, P processes) first runs a short process, then long ones that cannot
    finish before the context is done (0.5 s after the launch).  Whatever the box's speed, the
    outcome is fixed: per lane the short process exits, the first long one stops inside its run
    (it re-reads its context every 4096 steps), every later one stops before its first step."""
    V, P = 64, 4
    sc = _pkt_loop_sc(V)
    vm, maps, pids = build_engine(sc, exec_mode=mode)
    dev = "cuda:0"
    k = np.full((V, P), K_LONG, np.uint32)
    k[:, 0] = K_SHORT
    buf, off, lens = packets_to_buffer([int(x).to_bytes(4, "little") + bytes(60) for x in k.ravel()])
    budget = 1 << 40
    # the context-checking kernel variant, built and loaded before the timed launch
    warm = M.XDPBatch.from_numpy(*packets_to_buffer([K_SHORT.to_bytes(4, "little") + bytes(60)] * V), device=dev,
                                 schedule=M.SCHED_CHUNKED, step_budget=budget)
    live = M.WithCancel()
    vm.RunXDPBatch(pids[0], warm, ctx=live)
    batch = M.XDPBatch.from_numpy(buf, off, lens, device=dev, schedule=M.SCHED_CHUNKED, step_budget=budget)
    if kind == "cancel":
        ctx = M.WithCancel()
        ctx.native()
        timer = threading.Timer(0.5, ctx.Cancel)
    else:
        ctx = M.WithTimeout(0.5)
        ctx.native()
        timer = None
    res = M.XDPResults.empty(V * P, dev)
    vm.RunXDPBatch(pids[0], batch, res, sync=False, ctx=ctx)
    if timer is not None:
        timer.start()
    torch.cuda.synchronize()
    e = res.numpy(V * P)
    want = CANCELED if kind == "cancel" else DEADLINE
    st = e["status"].reshape(V, P)
    steps = e["steps"].reshape(V, P).astype(np.int64)
    r0 = e["r0"].reshape(V, P)
    assert (st[:, 0] == 0).all() and (r0[:, 0] == K_SHORT).all()
    assert (steps[:, 0] == steps[0, 0]).all()
    assert (st[:, 1:] == want).all()
    assert ((steps[:, 1] > 2 * K_SHORT) & (steps[:, 1] < 2 * K_LONG)).all()   # stopped inside its run
    assert (steps[:, 2:] == 0).all() and (r0[:, 1:] == 0).all()
    # only the short processes counted
    assert all(int(np.frombuffer(maps["c"].Values(c), np.uint64)[0]) == 2 for c in range(V))
    vm.close()
    ctx.close()
    live.close()


def test_done_while_the_batch_runs_matches_the_oracle(gpu):
    """The same in-flight cancel replayed on the oracle with the states the device saw: per packet
    results and the per-CPU counters of exactly the processes that ran."""
    V, P = 32, 24
    sc = _loop_sc(V, K_LOOP)
    buf, off, lens = packets_to_buffer([bytes(64)] * (V * P))
    cpu = W.schedule_cpu(V * P, V, "chunked")
    vm, maps, pids = build_engine(sc)
    dev = "cuda:0"
    warm = M.XDPBatch.from_numpy(*packets_to_buffer([bytes(64)] * V), device=dev, schedule=M.SCHED_CHUNKED)
    live = M.WithCancel()
    vm.RunXDPBatch(pids[0], warm, ctx=live)
    t = time.monotonic()
    vm.RunXDPBatch(pids[0], warm, ctx=live)
    vm.RunXDPBatch(pids[0], warm, ctx=live)
    t1 = (time.monotonic() - t) / 2
    vm.close()
    vm, maps, pids = build_engine(sc)
    vm.RunXDPBatch(pids[0], M.XDPBatch.from_numpy(*packets_to_buffer([bytes(64)]), device=dev), ctx=live)   # (build)
    for c in range(V):   # the build run's count out of the way
        maps["c"].Update((0).to_bytes(4, "little"), bytes(8), 0, c)
    batch = M.XDPBatch.from_numpy(buf, off, lens, device=dev, schedule=M.SCHED_CHUNKED)
    ctx = M.WithTimeout(0.5 * P * t1)
    res = vm.RunXDPBatch(pids[0], batch, ctx=ctx)
    e = res.numpy(V * P)
    e["pkt"] = batch.pkt_data.cpu().numpy()
    e["maps"] = {"c": [maps["c"].Values(c) for c in range(V)]}
    e["hash"] = {}
    done = (e["status"] == DEADLINE).astype(np.uint8) * 2
    o = run_oracle(sc, buf, off, lens, cpu, ctx_done=done,
                   ctx_done_step=np.where(done > 0, e["steps"], 0).astype(np.uint32))
    assert_same(o, e)
    vm.close()
    ctx.close()


def test_process_run_ctx_deadline_then_continue(gpu):
    """Process.Run(ctx) with a deadline that passes mid-run: ctx.Err(), the process suspended with
    some steps done; Run with a live context finishes it exactly as one uninterrupted run."""
    K = 1_500_000
    sc = _loop_sc(1, K)
    vm, maps, pids = build_engine(sc)
    p = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=bytes(64)))
    p.SetCPUID(0)
    t = time.monotonic()
    with pytest.raises(M.MimicError, match="context deadline exceeded"):
        p.Run(ctx=M.WithTimeout(0.02))
    assert time.monotonic() - t < 5.0
    assert 0 < p.Steps < 2 * K and not p._exited
    p.Run(ctx=M.WithCancel())
    assert p._exited and p.Status == 0 and p.Registers.R0 == K
    b, o, l = packets_to_buffer([bytes(64)])
    ref = run_oracle(sc, b, o, l, np.zeros(1, np.int32))
    assert p.Steps == int(ref["steps"][0])
    assert np.frombuffer(maps["c"].Values(0), np.uint64)[0] == 1
    p.Cleanup()
    vm.close()


def test_process_run_ctx_canceled_takes_no_step(gpu):
    sc = _count_sc(2)
    vm, maps, pids = build_engine(sc)
    p = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=bytes(40)))
    p.SetCPUID(1)
    c = M.WithCancel()
    c.Cancel()
    with pytest.raises(M.MimicError, match="context canceled"):
        p.Run(ctx=c)
    assert p.Steps == 0 and not p._exited
    p.Run()
    assert p.Status == 0 and p.Registers.R0 == 40
    p.Cleanup()
    vm.close()
    c.close()


def test_pool_jobs_with_contexts(gpu):
    """ProcessPool jobs carry their own contexts into the launch: a job whose context is canceled
    is handed off with ctx.Err(), the others run."""
    sc = _count_sc(4)
    vm, maps, pids = build_engine(sc)
    pool = vm.GetProcessPool()
    pool.Start(64)
    got = {}
    ev = threading.Event()

    def handoff(k):
        def f(proc, err):
            got[k] = (proc.Registers.R0, None if err is None else str(err))
            if len(got) == 16:
                ev.set()
        return f

    live = M.WithCancel()
    for k in range(16):
        pool.Enqueue(M.ProcessPoolJob(vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=bytes(20 + k))), live,
                                      handoff(k)))
    assert ev.wait(60)
    pool.Stop()
    assert all(got[k] == (20 + k, None) for k in range(16))
    vm.close()
    live.close()


def test_context_freed_while_its_batch_runs(gpu):
    """Freeing a context (mimic_ctx_free, here through the garbage collector) while a launch that
    reads it runs waits for that launch: the kernel never reads freed host memory."""
    import gc

    V, P = 64, 16
    sc = _loop_sc(V, K_LOOP)
    vm, maps, pids = build_engine(sc)
    buf, off, lens = packets_to_buffer([bytes(64)] * (V * P))
    batch = M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", schedule=M.SCHED_CHUNKED)
    res = M.XDPResults.empty(V * P, "cuda:0")
    ctx = M.WithCancel()
    vm.RunXDPBatch(pids[0], batch, res, sync=False, ctx=ctx)
    del ctx
    gc.collect()
    torch.cuda.synchronize()
    e = res.numpy(V * P)
    assert (e["status"] == 0).all() and (e["r0"] == K_LOOP).all()
    vm.close()


@pytest.mark.parametrize("mode,K", [("jit", 20_000_000), ("interp", 2_000_000)])
def test_canceled_inside_running_processes(gpu, mode, K):
    """A cancel while processes run their loops: each running process reads its context again
    every 4096 steps (the JIT's context variant at block starts, the interpreter per 4096
    wave-steps) and stops before its next step.  Each of the 8 lanes runs 2 processes of 2 K steps
    (about a second each at this engine's rate for one wave), so a cancel 30 ms in lands inside
    every lane's first one; without the in-process check the batch would run to its end (bounded).
    The oracle replays the batch with each canceled process's context seen done before the step the
    device stopped at (orc ctx_done_step): R0, status, steps, err_pc, packet memory and the per-CPU
    counters agree."""
    V, P = 8, 2
    sc = _loop_sc(V, K)
    vm, maps, pids = build_engine(sc, exec_mode=mode)
    dev = "cuda:0"
    live = M.WithCancel()
    vm.RunXDPBatch(pids[0], M.XDPBatch.from_numpy(*packets_to_buffer([bytes(64)]), device=dev, step_budget=1 << 26),
                   ctx=live)   # builds the kernel variant (its count reset below)
    maps["c"].Update((0).to_bytes(4, "little"), bytes(8), 0, 0)
    buf, off, lens = packets_to_buffer([bytes(64)] * (V * P))
    batch = M.XDPBatch.from_numpy(buf, off, lens, device=dev, schedule=M.SCHED_CHUNKED, step_budget=1 << 26)
    ctx = M.WithCancel()
    ctx.native()
    res = M.XDPResults.empty(V * P, dev)
    t = time.monotonic()
    vm.RunXDPBatch(pids[0], batch, res, sync=False, ctx=ctx)
    threading.Timer(0.03, ctx.Cancel).start()
    torch.cuda.synchronize()
    wall = time.monotonic() - t
    e = res.numpy(V * P)
    e["pkt"] = batch.pkt_data.cpu().numpy()
    e["maps"] = {"c": [maps["c"].Values(c) for c in range(V)]}
    e["hash"] = {}
    st = e["status"].reshape(V, P)
    steps = e["steps"].reshape(V, P)
    assert (st == CANCELED).all(), (wall, st)
    assert (steps[:, 0] > 0).all() and (steps[:, 0] < 2 * K).all() and (steps[:, 1] == 0).all(), steps
    cpu = W.schedule_cpu(V * P, V, "chunked")
    done = np.ones(V * P, np.uint8)
    o = run_oracle(sc, buf, off, lens, cpu, step_budget=1 << 26, ctx_done=done,
                   ctx_done_step=e["steps"].astype(np.uint32))
    assert_same(o, e)
    vm.close()
    ctx.close()
    live.close()


def test_host_resident_batch_with_a_context(gpu):
    """mimic_run_xdp_host_ctx: every sub-batch's kernel reads the run's context -- a live one
    changes nothing, a canceled one ends every process before its first step."""
    sc = _count_sc()
    buf, off, lens = _packets(3000, seed=9)
    cpu = W.schedule_cpu(len(lens), sc.vcpus, "interleaved")
    results = []
    for state in (0, 1):
        vm, maps, pids = build_engine(sc)
        c = M.WithCancel()
        if state:
            c.Cancel()
        hbuf = buf.copy()
        r0, st = vm.RunXDPHost(pids[0], hbuf, off, lens, schedule=M.SCHED_INTERLEAVED, headroom=8, tailroom=8,
                               chunks=3, ctx=c)
        o = run_oracle(sc, buf, off, lens, cpu, headroom=8, tailroom=8,
                       ctx_done=np.full(len(lens), state, np.uint8))
        assert (r0 == o["r0"]).all() and (st == o["status"]).all()
        assert [maps["c"].Values(k) for k in range(sc.vcpus)] == o["maps"]["c"]
        results.append(st)
        vm.close()
        c.close()
    assert (results[0] == 0).all() and (results[1] == CANCELED).all()


@pytest.mark.parametrize("sched", ["interleaved", "explicit"])
def test_host_resident_per_packet_contexts(gpu, sched):
    """mimic_run_xdp_host_ctx_pp: Background, live, canceled and past-deadline contexts per packet
    (processPool's jobs each carry theirs, vm.go:548-573) across 5 sub-batches; the oracle replays
    the states, packet bytes (pkt_out) and counters included."""
    sc = _count_sc()
    buf, off, lens = _packets(3000, seed=10)
    n = len(lens)
    rng = np.random.default_rng(5)
    cpu = rng.integers(0, sc.vcpus, n).astype(np.int32) if sched == "explicit" else W.schedule_cpu(n, sc.vcpus, sched)
    live, gone, late = M.WithCancel(), M.WithCancel(), M.WithTimeout(0.0)
    gone.Cancel()
    ctxs = [[None, live, gone, late, M.Background()][k] for k in rng.integers(0, 5, n)]
    done = _states([None if c is not None and getattr(c, "_background", False) else c for c in ctxs])
    assert set(np.unique(done)) == {0, 1, 2}
    vm, maps, pids = build_engine(sc)
    hbuf, out = buf.copy(), np.zeros_like(buf)
    mode = M.SCHED_EXPLICIT if sched == "explicit" else M.SCHED_INTERLEAVED
    r0, st = vm.RunXDPHost(pids[0], hbuf, off, lens, schedule=mode, cpu=cpu if sched == "explicit" else None,
                           headroom=8, tailroom=8, chunks=5, pkt_out=out, ctx_per_packet=ctxs)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=8, tailroom=8, ctx_done=done)
    assert (r0 == o["r0"]).all() and (st == o["status"]).all()
    assert (st[done == 1] == CANCELED).all() and (st[done == 2] == DEADLINE).all()
    from harness import build_oracle

    ovm, _, opids = build_oracle(sc)   # the packet memory the oracle leaves (a process that ran stored a byte)
    obuf = buf.copy()
    ovm.run_xdp_batch(opids[0], obuf, off, lens, cpu, 8, 8, None, None, None, 0, ctx_done=done)
    ovm.close()
    for i in range(n):
        a, L = int(off[i]), int(lens[i])
        assert out[a:a + 16 + L].tobytes() == obuf[a:a + 16 + L].tobytes(), i
    assert [maps["c"].Values(k) for k in range(sc.vcpus)] == o["maps"]["c"]
    vm.close()
    for c in (live, gone, late):
        c.close()
