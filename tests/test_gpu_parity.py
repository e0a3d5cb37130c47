"""GPU parity: the HIP engine vs the CPU oracle on the same inputs (bit-exact)."""
import numpy as np
import pytest

from harness import (Scenario, assert_same, build_engine, build_oracle, kernel_of, packets_to_buffer, run_engine,
                     run_oracle, single)
import mimic_amd as M
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


def _prog_scenario(p: W.Program, vcpus: int) -> Scenario:
    return Scenario(vcpus=vcpus, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def jit_kernels():
    ks = [kernel_of(_prog_scenario(p, 1)) for p in (W.prog_pass8(), W.prog_classifier(), W.prog_parse5())]
    ks += [kernel_of(_fuzz(s)[0]) for s in range(40)]
    return ks + [kernel_of(_tailcall_sc()), kernel_of(_rewrite_sc()), kernel_of(_cpuid_sc()), kernel_of(_elf_sc())]


def test_pass8(gpu):
    p = W.prog_pass8()
    sc = _prog_scenario(p, 2)
    buf, off, lens, cpu = single(sc)
    e = run_engine(sc, buf, off, lens, cpu)
    assert int(e["r0"][0]) == 2 and int(e["status"][0]) == 0 and int(e["steps"][0]) == 8
    assert_same(run_oracle(sc, buf, off, lens, cpu), e)


@pytest.mark.parametrize("mode", ["chunked", "interleaved"])
def test_classifier_small(gpu, mode):
    p = W.prog_classifier()
    sc = _prog_scenario(p, 64)
    buf, off, lens = W.make_packets(4096)
    cpu = W.schedule_cpu(4096, 64, mode)
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert set(np.unique(o["r0"])) <= {1, 2}


def _fuzz(seed):
    rng = np.random.default_rng(1000 + seed)
    raw, rel = __import__("fuzz").random_program(rng, n_body=int(rng.integers(10, 80)), map_name="m")
    return Scenario(vcpus=8, maps=[dict(name="m", type=6, key_size=4, value_size=8, max_entries=4)],
                    progs=[("fz", raw, rel)]), rng


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_programs(gpu, seed):
    sc, rng = _fuzz(seed)
    pk = [bytes(rng.integers(0, 256, int(rng.choice([0, 14, 60, 64, 100])), dtype=np.uint8)) for _ in range(64)]
    buf, off, lens = packets_to_buffer(pk)
    cpu = rng.integers(0, 8, 64).astype(np.int32)
    o = run_oracle(sc, buf, off, lens, cpu, step_budget=5000)
    e = run_engine(sc, buf, off, lens, cpu, step_budget=5000)
    assert_same(o, e)


def test_classifier_full_size_exact(gpu):
    """BASELINE configs[1] at full size: 1 048 576 x 64 B, V = 262 144 vCPUs, exact per-packet
    parity with the oracle plus the size-independent property sum(counters) == packets."""
    p = W.prog_classifier()
    n, V = 1 << 20, 1 << 18
    sc = _prog_scenario(p, V)
    buf, off, lens = W.make_packets(n)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    import mimic_amd as M
    for spread, kernel in ((None, "spread_own"), (0, "jit")):   # the bench's owned spread form, and one lane per vCPU
        e = run_engine(sc, buf, off, lens, cpu, schedule=M.SCHED_INTERLEAVED, spread=spread)
        assert e["last_exec"] == kernel
        assert_same(o, e)
        tot = sum(int(np.frombuffer(v, np.uint64).sum()) for v in e["maps"]["verdicts"])
        assert tot == n
        assert e["steps_total"] == int(o["steps"].astype(np.int64).sum())


def test_parse5_imix_exact(gpu):
    p = W.prog_parse5()
    n, V = 1 << 16, 4096
    sc = _prog_scenario(p, V)
    buf, off, lens = W.make_packets(n, **W.IMIX)
    cpu = W.schedule_cpu(n, V, "chunked")
    import mimic_amd as M
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu, schedule=M.SCHED_CHUNKED)
    assert_same(o, e)
    assert set(np.unique(o["r0"]).tolist()) <= {1, 2}


@pytest.mark.parametrize("sched", ["chunked", "interleaved", "explicit"])
def test_schedules(gpu, sched):
    import mimic_amd as M
    p = W.prog_classifier()
    n, V = 5000, 96
    sc = _prog_scenario(p, V)
    buf, off, lens = W.make_packets(n, seed=7)
    if sched == "explicit":
        cpu = np.random.default_rng(3).integers(0, V, n).astype(np.int32)
        mode = M.SCHED_EXPLICIT
    else:
        cpu = W.schedule_cpu(n, V, sched)
        mode = M.SCHED_CHUNKED if sched == "chunked" else M.SCHED_INTERLEAVED
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu if mode == M.SCHED_EXPLICIT else None, schedule=mode)
    assert_same(o, e)


def _tailcall_sc():
    PA = dict(name="progs", type=3, key_size=4, value_size=4, max_entries=4)
    CNT = dict(name="cnt", type=6, key_size=4, value_size=8, max_entries=4)
    main = [A.mov64_reg(6, 1), A.ldx(4, 2, 6, 0), A.ldx(4, 3, 6, 4), A.mov64_reg(4, 2), A.alu64("add", 4, 1),
            A.jmp("jgt", 4, 3, "out", reg=True), A.ldx(1, 3, 2, 0), A.alu64("and", 3, 3), A.mov64_reg(1, 6),
            A.ld_map_fd(2, "progs"), A.call(A.FN_TAIL_CALL), "out", A.mov64_imm(0, 99), A.exit_()]

    def leaf(v):
        return [A.st(4, 10, -4, v), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "cnt"),
                A.call(1), A.jmp("jeq", 0, 0, 3), A.ldx(8, 1, 0, 0), A.alu64("add", 1, 1), A.stx(8, 0, 0, 1),
                A.mov64_imm(0, v), A.exit_()]

    progs = [("main", *A.assemble(main))] + [(f"l{v}", *A.assemble(leaf(v))) for v in range(3)]
    return Scenario(vcpus=32, maps=[PA, CNT], progs=progs, prog_array=[("progs", 0, 1), ("progs", 1, 2),
                                                                        ("progs", 2, 3)])


def test_tailcall_divergence(gpu):
    """Lanes of one wave tail-call into different programs (and some do not) -- the wave
    runs several programs at once (min-key scheduling over global instruction indices)."""
    sc = _tailcall_sc()
    rng = np.random.default_rng(11)
    pk = [bytes(rng.integers(0, 256, int(rng.choice([0, 8, 64])), dtype=np.uint8)) for _ in range(3000)]
    buf, off, lens = packets_to_buffer(pk)
    cpu = rng.integers(0, 32, len(pk)).astype(np.int32)
    assert_same(run_oracle(sc, buf, off, lens, cpu), run_engine(sc, buf, off, lens, cpu))


def _rewrite_sc():
    items = [A.ldx(4, 2, 1, 0), A.ldx(4, 3, 1, 4), A.mov64_reg(4, 2), A.alu64("add", 4, 12),
             A.jmp("jgt", 4, 3, "out", reg=True),
             A.ldx(4, 5, 2, 0), A.ldx(2, 6, 2, 4), A.ldx(4, 7, 2, 6), A.ldx(2, 8, 2, 10),
             A.stx(4, 2, 0, 7), A.stx(2, 2, 4, 8), A.stx(4, 2, 6, 5), A.stx(2, 2, 10, 6),
             A.ldx(1, 9, 2, -1), A.mov64_imm(0, A.XDP_TX), A.alu64("add", 0, 9, reg=True), A.exit_(),
             "out", A.mov64_imm(0, A.XDP_DROP), A.exit_()]
    raw, rel = A.assemble(items)
    return Scenario(vcpus=8, progs=[("tx", raw, rel)])


def test_packet_rewrite_and_room(gpu):
    """XDP_TX-style MAC swap written in place, per-packet headroom/tailroom arrays."""
    sc = _rewrite_sc()
    rng = np.random.default_rng(5)
    n = 700
    pk = [bytes(rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8)) for _ in range(n)]
    H = rng.integers(1, 40, n).astype(np.uint32)
    T = rng.integers(0, 17, n).astype(np.uint32)
    buf, off, lens = packets_to_buffer(pk, H, T)
    buf[:] = rng.integers(0, 256, len(buf), dtype=np.uint8)   # dirty room bytes: the engine must zero them
    for i, p_ in enumerate(pk):
        buf[int(off[i]) + int(H[i]):int(off[i]) + int(H[i]) + len(p_)] = np.frombuffer(p_, np.uint8)
    cpu = rng.integers(0, 8, n).astype(np.int32)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=H, tailroom=T)
    e = run_engine(sc, buf, off, lens, cpu, headroom=H, tailroom=T)
    for i in range(n):  # compare only packet memories (the gaps between them are not process memory)
        a, m = int(off[i]), int(H[i] + lens[i] + T[i])
        assert bytes(o["pkt"][a:a + m]) == bytes(e["pkt"][a:a + m]), i
    assert_same(o, e, check_pkt=False)


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_programs_interp(gpu, seed):
    """The same random programs on the batch interpreter."""
    sc, rng = _fuzz(seed)
    pk = [bytes(rng.integers(0, 256, int(rng.choice([0, 14, 60, 64, 100])), dtype=np.uint8)) for _ in range(64)]
    buf, off, lens = packets_to_buffer(pk)
    cpu = rng.integers(0, 8, 64).astype(np.int32)
    assert_same(run_oracle(sc, buf, off, lens, cpu, step_budget=5000),
                run_engine(sc, buf, off, lens, cpu, step_budget=5000, exec_mode="interp"))


def _cpuid_sc():
    """r6 = get_smp_processor_id(); then a per-CPU array lookup (fails for CPU IDs -1 and V,
    emulator_linux_map_array.go:236-238) unless the packet is empty."""
    items = [A.call(8), A.mov64_reg(6, 0), A.ldx(4, 2, 1, 0), A.ldx(4, 3, 1, 4), A.jmp("jeq", 2, 3, "out", reg=True),
             A.st(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "pc"), A.call(1),
             "out", A.mov64_reg(0, 6), A.exit_()]
    raw, rel = A.assemble(items)
    return Scenario(vcpus=4, maps=[dict(name="pc", type=6, key_size=4, value_size=8, max_entries=2)],
                    progs=[("cpuid", raw, rel)])


@pytest.mark.parametrize("exec_mode", ["jit", "interp"])
def test_unset_and_V_cpu_ids(gpu, exec_mode):
    """Processes whose CPU ID was never set (-1, vm.go:214) or equals V (SetCPUID accepts it,
    vm.go:273) run: helper 8 returns the ID as set, per-CPU map operations fail."""
    sc = _cpuid_sc()
    pk = [b"", bytes(64), b"", bytes(64), b"", bytes(64)]
    buf, off, lens = packets_to_buffer(pk)
    cpu = np.array([-1, -1, 4, 4, 1, 1], np.int32)
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu, exec_mode=exec_mode)
    assert_same(o, e)
    assert [int(x) for x in e["r0"][:3]] == [2 ** 64 - 1, 2 ** 64 - 1, 4]
    st = [M.STATUS_NAMES[int(x)] for x in e["status"]]
    assert st == ["OK", "ERR_HELPER_MAP_OP", "OK", "ERR_HELPER_MAP_OP", "OK", "OK"], st


def test_process_run_cpu_unset_and_V(gpu):
    """The Process.Run drop-in without SetCPUID, and with SetCPUID(V)."""
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(3))
    raw, _ = A.assemble([A.call(8), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("smp", raw))
    p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=bytes(64)))
    p.Run()
    assert p.Registers.R0 == 2 ** 64 - 1
    p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=bytes(64)))
    p.SetCPUID(3)
    p.Run()
    assert p.Registers.R0 == 3
    with pytest.raises(M.MimicError):
        p.SetCPUID(4)
    vm.close()


def _elf_sc(btf: bool = False):
    import os
    import sys

    from mimic_amd import elf

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from test_elf import OBJ, OBJ_BTF, scenario_of

    spec = elf.LoadCollectionSpec(OBJ_BTF if btf else OBJ)
    return scenario_of(spec, ["xdp_count", "xdp_pass"])


@pytest.mark.parametrize("btf", [False, True], ids=["legacy_maps", "btf_maps"])
@pytest.mark.parametrize("exec_mode", ["jit", "interp"])
def test_elf_object_on_the_engine(gpu, exec_mode, btf):
    """The committed ELF objects (tests/golden/xdp_count.o with a legacy "maps" section,
    xdp_count_btf.o with BTF-defined ".maps") loaded through mimic_amd.elf run on the engine
    exactly like the oracle: BPF-to-BPF calls (with Q12), per-CPU map, .data datasec."""
    sc = _elf_sc(btf)
    pk = [bytes([i % 256]) * (1 + i % 70) for i in range(300)] + [b""]
    buf, off, lens = packets_to_buffer(pk)
    cpu = (np.arange(len(pk)) % 4).astype(np.int32)
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu, exec_mode=exec_mode)
    assert_same(o, e)
    assert int(e["r0"][1]) == 0x1122334455667788 + 1


@pytest.mark.parametrize("V,E", [(1000, 4), (64, 300), (7, 1)])
def test_sum_u64_readout(gpu, V, E):
    """mimic_map_sum_u64 (the sum-over-CPUs readout the multi-GPU all-reduce starts from) equals
    the per-cpu Values summed on the host, for flat (E <= 256) and per-key (E > 256) layouts."""
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(V))
    m = M.LinuxPerCPUArrayMap(M.MapSpec("c", M.MapType.PerCPUArray, 4, 8, E))
    emu.AddMap("c", m)
    rng = np.random.default_rng(V * 7 + E)
    want = np.zeros(E, np.uint64)
    for _ in range(min(400, V * E)):
        k, c = int(rng.integers(0, E)), int(rng.integers(0, V))
        v = int(rng.integers(0, 1 << 62))
        assert m.Update(k.to_bytes(4, "little"), v.to_bytes(8, "little"), 0, c) == 0
    for c in range(V):
        want += np.frombuffer(m.Values(c), np.uint64)
    assert m.SumU64() == [int(x) for x in want]
    assert m.SumU64(1, V) == [int(x) for x in want - np.frombuffer(m.Values(0), np.uint64)]
    vm.close()


def test_batches_across_streams_and_parameter_slots(gpu):
    """Back-to-back asynchronous batches on three streams (the VM's own and two torch streams),
    each batch a different packet window (new launch parameters: the engine's 8 parameter slots
    are reused several times over).  A parameter slot's event is recorded when the slot is left,
    and a stream change waits for the device (engine.cpp kp_slot), so every batch must give the
    oracle's per-packet results and the per-CPU counters must add up over all batches in order."""
    import torch

    import mimic_amd as M

    p = W.prog_classifier()
    V = 64
    sc = _prog_scenario(p, V)
    n, chunk = 8192, 512
    buf, off, lens = W.make_packets(n, seed=11)
    vm, maps, pids = build_engine(sc)
    streams = [None, torch.cuda.Stream(), torch.cuda.Stream()]
    keep = []
    for k in range(24):
        a = (k * 331) % (n - chunk)
        sel = slice(a, a + chunk)
        batch = M.XDPBatch.from_numpy(buf, off[sel], lens[sel], device="cuda:0", schedule=M.SCHED_INTERLEAVED)
        res = vm.RunXDPBatch(pids[0], batch, stream=streams[(k // 2) % 3], sync=False)
        keep.append((sel, batch, res))
    torch.cuda.synchronize()
    total = 0
    ovm, _, opids = build_oracle(sc)
    for sel, batch, res in keep:
        cpu = W.schedule_cpu(chunk, V, "interleaved")
        o = ovm.run_xdp_batch(opids[0], buf.copy(), off[sel], lens[sel], cpu)
        got = res.numpy(chunk)
        assert np.array_equal(np.asarray(o["r0"], np.uint64), np.asarray(got["r0"], np.uint64))
        assert np.array_equal(np.asarray(o["status"]), np.asarray(got["status"]))
        total += chunk
    ovm.close()
    cnt = sum(int(np.frombuffer(maps["verdicts"].Values(c), np.uint64).sum()) for c in range(V))
    assert cnt == total
    vm.close()
