"""The GPU engine against the hand-derived KATs and the reference's own tests (through the
Python mirror of the reference API).

* Every KAT runs on the batch interpreter in a VM of its own (the KAT's exact address layout)
  and must give the expected R0 / status / steps / err_pc.
* The JIT runs the same single-program KATs in chunks: one VM (one generated kernel) holds a
  chunk's programs, each case runs as its own batch with its program as the entry, and every
  batch plus the final maps must equal the oracle running the same sequence on the same
  layout (the oracle is pinned to the KATs by tests/test_oracle_golden.py).  The multi-program
  KATs (tail calls) run on the JIT in VMs of their own against the expected values.
"""
import numpy as np
import pytest

import mimic_amd as M
from harness import (assert_same_sequence, kernel_of, run_engine, run_sequence_engine, run_sequence_oracle)
from kat import check, inputs, jit_groups, load_cases, multi_cases, scenario

pytestmark = pytest.mark.gpu

CASES = load_cases()
GROUPS = jit_groups(CASES)
MULTI = multi_cases(CASES)


def jit_kernels():
    """The JIT kernels this module runs (compiled in parallel before the session, conftest.py)."""
    return [kernel_of(sc) for sc, _, _ in GROUPS] + [kernel_of(scenario(c)) for c in MULTI]


def _run_kat(c, exec_mode):
    i = inputs(c)
    return run_engine(scenario(c), i["buf"], i["off"], i["lens"], i["cpu"], headroom=i["headroom"],
                      tailroom=i["tailroom"], ingress=np.array([c["ingress"]], np.int32),
                      rxq=np.array([c["rxq"]], np.int32), egress=np.array([c["egress"]], np.int32),
                      step_budget=i["step_budget"], exec_mode=exec_mode)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_engine_kat_interp(gpu, c):
    check(c, _run_kat(c, "interp"))


@pytest.mark.parametrize("g", range(len(GROUPS)), ids=[f"chunk{k}_{len(g[2])}" for k, g in enumerate(GROUPS)])
def test_engine_kat_jit_chunk(gpu, g):
    sc, runs, chunk = GROUPS[g]
    o = run_sequence_oracle(sc, runs)
    e = run_sequence_engine(sc, runs, exec_mode="jit")
    assert_same_sequence(o, e, tag=f"chunk {g}")
    assert any(r["last_exec"] == "jit" for r in e[0]), "no batch of the chunk ran on the JIT kernel"


@pytest.mark.parametrize("c", MULTI, ids=[c["name"] for c in MULTI])
def test_engine_kat_jit_multi(gpu, c):
    check(c, _run_kat(c, "jit"))


def _k(v):
    return int(v).to_bytes(4, "little")


def test_ref_TestLinuxPerCPUArray(gpu):
    """emulator_linux_map_array_test.go:10-103 against the device-resident map."""
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(2))
    m = M.LinuxPerCPUArrayMap(M.MapSpec("per-cpu-array", M.MapType.PerCPUArray, 4, 4, 5))
    emu.AddMap("per-cpu-array", m)
    assert m.Update(_k(1), _k(2), 0, 0) == 0
    assert m.Update(_k(1), _k(3), 0, 1) == 0
    a0, a1 = m.Lookup(_k(1), 0), m.Lookup(_k(1), 1)
    assert a0 != a1
    assert vm.MemoryController.Load(a0, 4) == 2
    assert vm.MemoryController.Load(a1, 4) == 3
    assert m.Update(_k(7), _k(1), 0, 0) == M.E2BIG
    vm.close()


def test_ref_TestLinuxHelperLookup_process_run(gpu):
    """emulator_linux_helpers_test.go:11-113 as a program run through Process.Run."""
    from mimic_amd import asm as A

    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(1))
    m = M.LinuxArrayMap(M.MapSpec("happy path", M.MapType.Array, 4, 4, 5))
    emu.AddMap("happy path", m)
    assert m.Update(_k(1), _k(2), 0, 0) == 0
    raw, rel = A.assemble([A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4),
                           A.ld_map_fd(1, "happy path"), A.call(1), A.ldx(4, 0, 0, 0), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("lookup", raw, rel))
    p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=b"\x00" * 64))
    p.SetCPUID(0)
    p.Run()
    assert p.Registers.R0 == 2
    p.Cleanup()
    vm.close()


def test_ref_TestLinuxHelperGetSmpProcessorID(gpu):
    from mimic_amd import asm as A

    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(2))
    raw, _ = A.assemble([A.call(8), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("pseudo", raw))
    for cpu in (0, 1):
        p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=b"\x00" * 64))
        p.SetCPUID(cpu)
        p.Run()
        assert p.Registers.R0 == cpu
    vm.close()


def test_process_run_reports_fatal_error(gpu):
    from mimic_amd import asm as A

    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(1))
    raw, _ = A.assemble([A.mov64_imm(0, 1), A.mov64_imm(2, 0), A.alu64("div", 0, 2, reg=True), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("div0", raw))
    p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=b"\x00" * 64))
    p.SetCPUID(0)
    with pytest.raises(M.MimicError, match="PANIC_DIV0"):
        p.Run()
    assert p.Steps == 3 and p.ErrPC == 2
    vm.close()


def test_context_json(gpu):
    """UnmarshalContextJSON (context.go:57-71) feeding Process.Run."""
    import base64
    import json

    from mimic_amd import asm as A

    pkt = bytes(range(64))
    js = json.dumps({"name": "c", "type": "xdp_md", "ctx": {"headroom": 8, "tailroom": 4,
                                                          "packet": base64.b64encode(pkt).decode(),
                                                          "ingress_ifidx": 7, "rx_queue_idx": 1}})
    ctx = M.UnmarshalContextJSON(js)
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(1))
    raw, _ = A.assemble([A.ldx(4, 2, 1, 0), A.ldx(1, 0, 2, 5), A.ldx(4, 3, 1, 12), A.alu64("lsh", 3, 8),
                         A.alu64("or", 0, 3, reg=True), A.exit_()])
    pid = vm.AddProgram(M.ProgramSpec("p", raw))
    p = vm.NewProcess(pid, ctx)
    p.SetCPUID(0)
    p.Run()
    assert p.Registers.R0 == 5 | (7 << 8)
    assert p.PacketAfter[8:72] == pkt and p.PacketAfter[:8] == b"\x00" * 8
    vm.close()
