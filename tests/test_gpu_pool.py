"""ProcessPool (vm.go:468-583) on the device: jobs enqueued from the host run in micro-batches,
each a single launch; every job's R0 and status, and the per-CPU map state, equal the oracle
running the jobs in enqueue order on the vCPUs the pool gave them."""
import threading
import time

import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, build_engine, kernel_of, packets_to_buffer, run_oracle
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


def _sc(V):
    p = W.prog_classifier()
    return Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def _order_sc(V):
    def prog(name, op):
        return (name, *A.assemble([
            A.st(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "c"),
            A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, "out"),
            A.ldx(8, 1, 0, 0), op, A.stx(8, 0, 0, 1), A.mov64_reg(0, 1), A.exit_(),
            "out", A.mov64_imm(0, 0), A.exit_()]))

    return Scenario(vcpus=V, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=1)],
                    progs=[prog("inc", A.alu64("add", 1, 1)), prog("tri", A.alu64("mul", 1, 3))])


def jit_kernels():
    return [kernel_of(_sc(1)), kernel_of(_order_sc(2))]


def _addr_prog():
    """sk_buff program: R0 = flow_keys pointer << 32 | skb->data (the addresses its Load leaked)."""
    S = A.SKB
    raw, _ = A.assemble([A.mov64_reg(6, 1), A.ldx(4, 0, 6, S["data"]), A.ldx(4, 2, 6, S["flow_keys"]),
                         A.alu64("lsh", 2, 32), A.alu64("or", 0, 2, reg=True), A.exit_()])
    return raw


def test_pool_skb_jobs_run_on_their_own_load(gpu):
    """an sk_buff process's Load runs at NewProcess (its sock / flow keys / packet
    take the VM's next leak addresses then); the pool worker only calls Run (vm.go:570).  Pooled
    jobs must see the same addresses as the same processes run one at a time, and the VM's leak
    cursor must move once per process (a process made after the pool lands where it would)."""
    raw = _addr_prog()
    buf, off, lens = W.make_skb_packets(12, (64, 576, 1500), (1, 1, 1), seed=5)
    pk = [bytes(buf[int(o) + 32:int(o) + 32 + int(n)]) for o, n in zip(off, lens)]

    def fresh():
        vm = M.NewVM(M.VMOptEmulator(M.NewLinuxEmulator()), M.VMOptSetvCPUs(3))
        return vm, vm.AddProgram(M.ProgramSpec("addr", raw))

    vm1, pid1 = fresh()
    want = []
    for p in pk:
        proc = vm1.NewProcess(pid1, M.LinuxContextSKBuff(Packet=p))
        proc.Run()
        want.append(proc.Registers.R0)
        proc.Cleanup()
    after1 = vm1.NewProcess(pid1, M.LinuxContextSKBuff(Packet=pk[0]))
    after1.Run()

    vm2, pid2 = fresh()
    pool = vm2.GetProcessPool()
    pool.Start(64)
    got = {}
    mu = threading.Lock()

    def handoff(proc, err):
        with mu:
            got[proc.idx] = (proc.Registers.R0, err)

    for i, p in enumerate(pk):
        proc = vm2.NewProcess(pid2, M.LinuxContextSKBuff(Packet=p))
        proc.idx = i
        pool.Enqueue(M.ProcessPoolJob(proc, None, handoff))
    pool.Stop()
    t0 = time.time()
    while len(got) < len(pk) and time.time() - t0 < 30:
        time.sleep(0.01)
    assert [got[i][1] for i in range(len(pk))] == [None] * len(pk)
    assert [got[i][0] for i in range(len(pk))] == want
    assert len(set(want)) == len(pk)   # every process leaked its own addresses
    after2 = vm2.NewProcess(pid2, M.LinuxContextSKBuff(Packet=pk[0]))
    after2.Run()
    assert after2.Registers.R0 == after1.Registers.R0
    vm1.close()
    vm2.close()


@pytest.mark.parametrize("backlog", [16, 4096])
def test_pool_runs_jobs_like_the_oracle(gpu, backlog):
    V = 8
    sc = _sc(V)
    buf, off, lens = W.make_packets(1500, seed=17)
    pk = [bytes(buf[int(o):int(o) + int(n)]) for o, n in zip(off, lens)]
    vm, maps, pids = build_engine(sc)
    pool = vm.GetProcessPool()
    pool.Start(backlog)
    got = {}
    mu = threading.Lock()

    def handoff(proc, err):
        with mu:
            got[proc.idx] = (proc.Registers.R0, proc.CPUID(), proc.Status, err)
        proc.Cleanup()

    for i, p in enumerate(pk):
        proc = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=p))
        proc.idx = i
        pool.Enqueue(M.ProcessPoolJob(proc, None, handoff))
    pool.Stop()
    t0 = time.time()
    while len(got) < len(pk) and time.time() - t0 < 30:
        time.sleep(0.01)
    assert len(got) == len(pk)
    cpu = np.array([got[i][1] for i in range(len(pk))], np.int32)
    assert set(cpu.tolist()) == set(range(V))
    o = run_oracle(sc, *packets_to_buffer(pk), cpu)
    assert [got[i][0] for i in range(len(pk))] == [int(x) for x in o["r0"]]
    assert all(got[i][2] == 0 and got[i][3] is None for i in range(len(pk)))
    for c in range(V):
        assert maps["verdicts"].Values(c) == o["maps"]["verdicts"][c]
    vm.close()


def test_pool_api_rules_and_errors(gpu):
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(2))
    raw, _ = A.assemble([A.mov64_imm(0, 1), A.mov64_imm(2, 0), A.alu64("div", 0, 2, reg=True), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("div0", raw))
    pool = vm.GetProcessPool()
    with pytest.raises(M.MimicError, match="not yet running"):
        pool.Enqueue(M.ProcessPoolJob(vm.NewProcess(pid, M.LinuxContextXDP(Packet=bytes(8)))))
    with pytest.raises(M.MimicError, match="backlog"):
        pool.Start(0)
    pool.Start(2)
    with pytest.raises(M.MimicError, match="already running"):
        pool.Start(2)
    errs = []
    ev = threading.Event()

    def handoff(proc, err):
        errs.append(err)
        if len(errs) == 2:
            ev.set()

    pool.Enqueue(M.ProcessPoolJob(vm.NewProcess(pid, M.LinuxContextXDP(Packet=bytes(8))), None, handoff))
    pool.Enqueue(M.ProcessPoolJob(vm.NewProcess(pid, M.LinuxContextXDP(Packet=bytes(8))), M.Context(Cancelled=True),
                                  handoff))
    pool.Stop()
    assert ev.wait(10)
    msgs = sorted(str(e) for e in errs)
    assert "context canceled" in msgs[0] and "PANIC_DIV0" in msgs[1]
    vm.close()


def test_pool_keeps_enqueue_order_per_vcpu_across_programs(gpu):
    """Jobs of two programs that update one per-CPU counter non-commutatively (A: +1, B: *3),
    enqueued in a pattern that wraps the round-robin vCPU counter inside a micro-batch: every job's
    R0 (the counter after it) equals a sequential run of each vCPU's jobs in enqueue order."""
    V = 2
    sc = _order_sc(V)
    vm, maps, pids = build_engine(sc)
    pool = vm.GetProcessPool()
    pool.max_batch = 7
    pool.Start(64)
    got = {}
    mu = threading.Lock()

    def handoff(proc, err):
        with mu:
            got[proc.idx] = (proc.Registers.R0, proc.CPUID(), err)
        proc.Cleanup()

    pattern = [0, 0, 1, 0, 1, 1, 0, 1, 0, 0, 0, 1, 1, 1, 0, 1] * 4
    for i, k in enumerate(pattern):
        proc = vm.NewProcess(pids[k], M.LinuxContextXDP(Packet=bytes(64)))
        proc.idx = i
        pool.Enqueue(M.ProcessPoolJob(proc, None, handoff))
    pool.Stop()
    t0 = time.time()
    while len(got) < len(pattern) and time.time() - t0 < 30:
        time.sleep(0.01)
    assert len(got) == len(pattern) and all(g[2] is None for g in got.values())
    val = [0] * V
    for i, k in enumerate(pattern):
        c = got[i][1]
        val[c] = val[c] + 1 if k == 0 else val[c] * 3
        assert got[i][0] == val[c], (i, got[i], val)
    vm.close()


def test_pool_skb_chain_jobs_batched_like_the_oracle(gpu):
    """cfg 5's tail-call chain through the pool: 3 000 sk_buff jobs (NewProcess each, so every Load
    reserves its own leak addresses in enqueue order) run as micro-batched launches of the
    processes NewProcess made (mimic_process_run_many).  Every job's R0 / status / steps, its
    packet memory, and every per-CPU counter equal the oracle running the same jobs in order on the
    vCPUs the pool gave them (round robin); a few processes stepped before they are enqueued run
    on their own and still agree."""
    from harness import run_oracle_skb

    V = 16
    buf, off, lens = W.make_skb_packets(3000, **W.IMIX, variety=0.2, seed=8)
    progs, maps, pa = W.skb_programs()
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(buf, off, lens)]
    sc = Scenario(vcpus=V, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa, map_init=init)
    vm, mp, pids = build_engine(sc, ctx=1)
    procs, keep = [], []
    for i, (o_, n_) in enumerate(zip(off, lens)):
        try:   # NewProcess returns the context's Load error (vm.go:226-229): those jobs never exist
            procs.append(vm.NewProcess(pids[0], M.LinuxContextSKBuff(Packet=bytes(buf[int(o_) + 32:int(o_) + 32 + int(n_)]),
                                                                    Dev=M.NetDev(IFIndex=3))))
            keep.append(i)
        except M.MimicError as ex:
            assert "ERR_CTX_LOAD" in str(ex)
    assert 2500 < len(keep) < 3000
    off, lens = off[keep], lens[keep]
    pk = procs
    for k in (5, 77):   # stepped first: these continue on their own device process
        procs[k].SetCPUID(k % V)
        procs[k].Step()
    pool = vm.GetProcessPool()
    pool.max_batch = 1024
    pool.Start(len(pk))
    got = {}
    mu = threading.Lock()

    def handoff(proc, err):
        with mu:
            got[proc.idx] = (proc.Registers.R0, proc.CPUID(), proc.Status, proc.Steps, proc.Packet())
        proc.Cleanup()

    for i, p in enumerate(procs):
        p.idx = i
        pool.Enqueue(M.ProcessPoolJob(p, None, handoff))
    pool.Stop()
    t0 = time.time()
    while len(got) < len(pk) and time.time() - t0 < 60:
        time.sleep(0.01)
    assert len(got) == len(pk)
    cpu = np.array([got[i][1] for i in range(len(pk))], np.int32)
    assert (cpu == np.arange(len(pk)) % V).all()
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=3)
    assert [got[i][0] for i in range(len(pk))] == [int(x) for x in o["r0"]]
    assert [got[i][2] for i in range(len(pk))] == [int(x) for x in o["status"]]
    assert [got[i][3] for i in range(len(pk))] == [int(x) for x in o["steps"]]
    for i in range(0, len(pk), 7):
        o_ = int(off[i])
        assert got[i][4] == bytes(o["pkt"][o_:o_ + 32 + int(lens[i]) + 64]), i
    for c in range(V):
        assert mp["stats"].Values(c) == o["maps"]["stats"][c], c
    vm.close()
