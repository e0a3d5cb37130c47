"""Process.Step (vm.go:291-340) on the device, instruction by instruction, against the oracle's
Step: after every step the registers (PC, R0..R10), the current program and the exit / fatal
state must be identical -- for the cfg-2 classifier, a BPF-to-BPF + tail-call program, and the
error paths (fatal error, stepping a terminated process, Run after Step)."""
import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, build_engine, build_oracle, kernel_of
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


def jit_kernels():
    return []   # stepping runs on the interpreter


def _trace(sc, entry, pkt, cpu, H=0, T=0, max_steps=500):
    ovm, omids, opids = build_oracle(sc)
    evm, emaps, epids = build_engine(sc)
    from oracle.pyoracle import OracleProcess

    o = OracleProcess(ovm, opids[entry], xdp=(pkt, H, T, 1, 0, 0))
    if cpu >= 0:
        assert o.set_cpu(cpu) == 0
    e = evm.NewProcess(epids[entry], M.LinuxContextXDP(Packet=pkt, Headroom=H, Tailroom=T, IngessIfIndex=1))
    if cpu >= 0:
        e.SetCPUID(cpu)
    n = 0
    while True:
        n += 1
        rc, epc = o.step()
        try:
            exited = e.Step()
            err = None
        except M.MimicError as ex:
            exited, err = True, ex
        regs_o = [o.reg(r) for r in range(11)]
        regs_e = [e.Registers.Get(r) for r in range(11)]
        assert regs_e == regs_o, (n, regs_e, regs_o)
        if rc > 0:
            assert err is not None and M.STATUS_NAMES[e.Status] == M.STATUS_NAMES[rc], (n, e.Status, rc)
            assert e.Registers.PC == epc, (n, e.Registers.PC, epc)
            break
        assert err is None, (n, err)
        assert e.Registers.PC == o.pc(), (n, e.Registers.PC, o.pc())
        assert e.ProgramID == o.prog(), n
        if rc == -1:
            assert exited
            break
        assert not exited, n
        assert n < max_steps
    pk = e.Packet()
    o.cleanup()
    e.Cleanup()
    ovm.close()
    evm.close()
    return n, pk


def test_step_trace_classifier(gpu):
    p = W.prog_classifier()
    sc = Scenario(vcpus=4, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    buf, off, lens = W.make_packets(8, seed=5)
    for i in range(4):
        pkt = bytes(buf[int(off[i]):int(off[i]) + int(lens[i])])
        n, _ = _trace(sc, 0, pkt, cpu=i % 4)
        assert n > 20


def _calls_sc():
    PA = dict(name="progs", type=3, key_size=4, value_size=4, max_entries=2)
    main = [A.mov64_reg(6, 1), A.mov64_imm(1, 5), A.call_local("f"), A.mov64_reg(7, 0), A.mov64_reg(1, 6),
            A.ld_map_fd(2, "progs"), A.mov64_imm(3, 0), A.call(A.FN_TAIL_CALL), A.mov64_imm(0, 99), A.exit_(),
            "f", A.mov64_reg(0, 1), A.alu64("mul", 0, 3), A.st(8, 10, -8, 7), A.ldx(8, 2, 10, -8),
            A.alu64("add", 0, 2, reg=True), A.exit_()]
    leaf = [A.ldx(4, 2, 1, 0), A.ldx(1, 0, 2, 0), A.alu64("add", 0, 7, reg=True), A.exit_()]
    return Scenario(vcpus=2, maps=[PA], progs=[("main", *A.assemble(main)), ("leaf", *A.assemble(leaf))],
                    prog_array=[("progs", 0, 1)])


def test_step_trace_bpf2bpf_and_tailcall(gpu):
    n, _ = _trace(_calls_sc(), 0, bytes(range(1, 65)), cpu=1)
    assert n >= 14   # main 0-2, f (6 slots), main 3-8 with the LD_IMM64 pad, the leaf


def test_step_fatal_error_then_terminated(gpu):
    raw, _ = A.assemble([A.mov64_imm(0, 1), A.mov64_imm(2, 0), A.alu64("div", 0, 2, reg=True), A.exit_()])
    sc = Scenario(vcpus=1, progs=[("d", raw, [])])
    _trace(sc, 0, bytes(16), cpu=0)
    evm, _, pids = build_engine(sc)
    p = evm.NewProcess(pids[0], M.LinuxContextXDP(Packet=bytes(16)))
    p.SetCPUID(0)
    assert p.Step() is False and p.Step() is False
    with pytest.raises(M.MimicError, match="PANIC_DIV0"):
        p.Step()
    assert p.Registers.PC == 2
    with pytest.raises(M.MimicError, match="terminated"):
        p.Step()
    evm.close()


def test_step_then_run_and_exit_again(gpu):
    """A few Steps, then Run to the end: the same R0 and packet as one Run; stepping after a clean
    exit reports exited again (the exit leaves PC on the EXIT instruction, vm.go:318-325)."""
    p = W.prog_classifier()
    sc = Scenario(vcpus=2, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    buf, off, lens = W.make_packets(2, seed=11)
    pkt = bytes(buf[int(off[0]):int(off[0]) + int(lens[0])])
    evm, maps, pids = build_engine(sc)
    a = evm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pkt))
    a.SetCPUID(1)
    for _ in range(5):
        assert a.Step() is False
    a.Run()
    b = evm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pkt))
    b.SetCPUID(0)
    b.Run()
    assert a.Registers.R0 == b.Registers.R0 and a.Registers.R0 in (1, 2)
    pc = a.Registers.PC
    assert a.Step() is True and a.Registers.PC == pc
    assert a.Packet() == pkt
    evm.close()


def test_step_after_layout_change_is_refused(gpu):
    """A map loaded between two Steps moves the VM's next free address (and may move its map
    arena): the started process's saved R10 / packet pointers would point into the old layout, so
    the next Step is refused (ENOTSUP) instead of running on stale addresses.  A process that has
    not started yet picks up the new layout."""
    p = W.prog_classifier()
    sc = Scenario(vcpus=4, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    vm, maps, pids = build_engine(sc)
    pkt = bytes(W.make_packets(1)[0][:64])
    e = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pkt))
    e.SetCPUID(1)
    e.Step()
    e.Step()
    fresh = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pkt))
    fresh.SetCPUID(1)
    extra = M.LinuxArrayMap(M.MapSpec("late", M.MapType.Array, 4, 8, 1 << 16))
    vm.emulator.AddMap("late", extra)
    with pytest.raises(M.MimicError, match="layout changed"):
        e.Step()
    fresh.Run()
    assert fresh.Registers.R0 in (1, 2)
    e.Cleanup()
    fresh.Cleanup()
    vm.close()


def _skb_scenario(V=4):
    progs, maps, pa = W.skb_programs()
    buf, off, lens = W.make_skb_packets(64, **W.IMIX, variety=0.3, seed=21)
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(buf, off, lens, every=1)]
    sc = Scenario(vcpus=V, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa, map_init=init)
    pkts = [bytes(buf[int(off[i]) + 32:int(off[i]) + 32 + int(lens[i])]) for i in range(len(lens))]
    return sc, pkts


def test_skb_chain_step_trace_matches_oracle(gpu):
    """Process.Step on sk_buff processes (LinuxContextSKBuff, context_sk_buff.go:42-107) through
    the cfg-5 tail-call chain: after every step R0..R10, PC and the current program equal the
    oracle's Step, for packets taking every chain (IPv4 / IPv6 / other, header variants).  The
    processes are made and cleaned up in the same order on both sides, so their leaked sock /
    flow-keys / packet entries (and every address a program sees) agree too."""
    from oracle.pyoracle import OracleProcess

    sc, pkts = _skb_scenario()
    ovm, omids, opids = build_oracle(sc)
    evm, emaps, epids = build_engine(sc)
    seen_progs = set()
    for k, pkt in enumerate(pkts[:24]):
        try:
            o = OracleProcess(ovm, opids[0], skb=(pkt, 3))
        except Exception:
            with pytest.raises(M.MimicError):
                evm.NewProcess(epids[0], M.LinuxContextSKBuff(Packet=pkt, Dev=M.NetDev(3)))
            continue
        assert o.set_cpu(k % 4) == 0
        e = evm.NewProcess(epids[0], M.LinuxContextSKBuff(Packet=pkt, Dev=M.NetDev(3)))
        e.SetCPUID(k % 4)
        n = 0
        while True:
            n += 1
            rc, epc = o.step()
            try:
                exited, err = e.Step(), None
            except M.MimicError as ex:
                exited, err = True, ex
            regs_o = [o.reg(r) for r in range(11)]
            assert [e.Registers.Get(r) for r in range(11)] == regs_o, (k, n)
            if rc > 0:
                assert err is not None and M.STATUS_NAMES[e.Status] == M.STATUS_NAMES[rc], (k, n)
                break
            assert err is None, (k, n, err)
            assert e.Registers.PC == o.pc() and e.ProgramID == o.prog(), (k, n)
            seen_progs.add(o.prog())
            if rc == -1:
                assert exited
                break
            assert not exited and n < 2000
        o.cleanup()
        e.Cleanup()
    assert seen_progs >= {0, 1, 2, 4}, seen_progs
    for m in sc.maps:
        for c in range(4 if m["type"] == 6 else 1):
            assert emaps[m["name"]].Values(c) == ovm.map_values(omids[m["name"]], c), m["name"]
    ovm.close()
    evm.close()


def test_skb_process_run_exposes_every_register(gpu):
    """Process.Run on an sk_buff process: R0..R10 afterwards equal the oracle's registers at the
    exit (Readme.md:74-78 reads them after Run), and the leak addresses of consecutive processes
    follow the reference's."""
    from oracle.pyoracle import OracleProcess

    sc, pkts = _skb_scenario()
    ovm, _, opids = build_oracle(sc)
    evm, _, epids = build_engine(sc)
    for k, pkt in enumerate(pkts[:16]):
        try:
            o = OracleProcess(ovm, opids[0], skb=(pkt, 2))
        except Exception:
            continue
        o.set_cpu(1)
        while True:
            rc, _ = o.step()
            if rc != 0:
                break
        e = evm.NewProcess(epids[0], M.LinuxContextSKBuff(Packet=pkt, Dev=M.NetDev(2)))
        e.SetCPUID(1)
        if rc > 0:
            with pytest.raises(M.MimicError):
                e.Run()
        else:
            e.Run()
        assert [e.Registers.Get(r) for r in range(11)] == [o.reg(r) for r in range(11)], k
        o.cleanup()
        e.Cleanup()
    ovm.close()
    evm.close()


def test_xdp_process_run_exposes_every_register(gpu):
    """Run without any Step: R1..R10 are readable afterwards (not only R0)."""
    from oracle.pyoracle import OracleProcess

    p = W.prog_classifier()
    sc = Scenario(vcpus=2, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    buf, off, lens = W.make_packets(4, seed=3)
    ovm, _, opids = build_oracle(sc)
    evm, _, epids = build_engine(sc)
    for i in range(4):
        pkt = bytes(buf[int(off[i]):int(off[i]) + int(lens[i])])
        o = OracleProcess(ovm, opids[0], xdp=(pkt, 0, 0, 1, 0, 0))
        o.set_cpu(i % 2)
        while o.step()[0] == 0:
            pass
        e = evm.NewProcess(epids[0], M.LinuxContextXDP(Packet=pkt, IngessIfIndex=1))
        e.SetCPUID(i % 2)
        e.Run()
        assert [e.Registers.Get(r) for r in range(11)] == [o.reg(r) for r in range(11)]
        assert e.Registers.R2 != 0 and e.Registers.R10 != 0
        o.cleanup()
        e.Cleanup()
    ovm.close()
    evm.close()
