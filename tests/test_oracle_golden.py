"""Pin the CPU oracle: the reference's own golden values and the hand-derived KATs."""
import numpy as np
import pytest

import oracle
from harness import run_oracle
from kat import check, inputs, load_cases, scenario
from mimic_amd import asm as A

CASES = load_cases()


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_kat(c):
    i = inputs(c)
    out = run_oracle(scenario(c), i["buf"], i["off"], i["lens"], i["cpu"], headroom=i["headroom"],
                     tailroom=i["tailroom"], ingress=np.array([c["ingress"]]), rxq=np.array([c["rxq"]]),
                     egress=np.array([c["egress"]]), step_budget=i["step_budget"])
    check(c, out)


def _k(v):
    return int(v).to_bytes(4, "little")


def test_ref_TestLinuxHelperLookup():
    """emulator_linux_helpers_test.go:11-113, restated against the oracle's helper entry point."""
    vm = oracle.OracleVM(4)
    pid = vm.prog_load("pseudo", b"")
    p = vm.new_process(pid)
    mid = vm.map_create("happy path", 2, 4, 4, 5)
    scratch = vm.mem_add_scratch(16)
    assert vm.mem_write(scratch, _k(1)) == 0
    assert vm.map_update(mid, _k(1), _k(2), 0, 0) == 0
    p.set_reg(1, vm.map_addr(mid))
    p.set_reg(2, scratch)
    assert p.call_helper(1) == 0
    r0 = p.reg(0)
    assert r0 < 1 << 63
    rc, val = vm.mem_load(r0, 4)
    assert rc == 0 and val == 2
    p.cleanup()


def test_ref_TestLinuxPerCPUArray():
    """emulator_linux_map_array_test.go:10-103."""
    vm = oracle.OracleVM(2)
    mid = vm.map_create("per-cpu-array", 6, 4, 4, 5)
    assert vm.map_update(mid, _k(1), _k(2), 0, 0) == 0
    assert vm.map_update(mid, _k(1), _k(3), 0, 1) == 0
    rc0, a0 = vm.map_lookup(mid, _k(1), 0)
    rc1, a1 = vm.map_lookup(mid, _k(1), 1)
    assert rc0 == rc1 == 0 and a0 != a1
    assert vm.mem_load(a0, 4) == (0, 2)
    assert vm.mem_load(a1, 4) == (0, 3)


def test_ref_TestLinuxHelperGetSmpProcessorID():
    """emulator_linux_helpers_test.go:185-220."""
    vm = oracle.OracleVM(2)
    pid = vm.prog_load("pseudo", b"")
    p = vm.new_process(pid)
    assert p.set_cpu(0) == 0
    assert p.call_helper(8) == 0 and p.reg(0) == 0
    assert p.set_cpu(1) == 0
    assert p.call_helper(8) == 0 and p.reg(0) == 1
    assert p.set_cpu(2) == 0      # Q18: SetCPUID accepts id == V (vm.go:273)
    assert p.set_cpu(3) != 0
    p.cleanup()


def test_memory_controller_first_fit_and_reuse():
    """memory_controller.go:58-112: entries from 0x10000 with one-byte gaps; Cleanup reopens the
    per-process hole so every process of a batch gets the same stack address."""
    vm = oracle.OracleVM(2)
    mid = vm.map_create("m", 6, 4, 8, 4)
    assert vm.map_addr(mid) == 0x10000
    pid = vm.prog_load("p", A.assemble([A.mov64_reg(0, 10), A.exit_()])[0])
    # map obj 8 + 2 x (sub obj 8 + backing 32 + 2 gaps) = 0x10009 + 2*42
    assert vm.prog_addr(pid) == 0x10009 + 2 * 42
    st = vm.next_free()
    bufs = np.zeros(4 * 64, np.uint8)
    out = vm.run_xdp_batch(pid, bufs, np.arange(4) * 64, np.full(4, 64), np.zeros(4, np.int32))
    assert (out["r0"] == st + 256).all()
    assert vm.next_free() == st


def test_prog_load_rejects_truncated_ld_imm64():
    vm = oracle.OracleVM(1)
    with pytest.raises(oracle.OracleError):
        vm.prog_load("bad", A.encode(0x18, 1, 0, 0, 5))
    bad2 = A.encode(0x18, 1, 0, 0, 5) + A.encode(0x07, 0, 0, 0, 1)
    with pytest.raises(oracle.OracleError):
        vm.prog_load("bad2", bad2)


def test_oracle_cpu_unset_and_V():
    """vm.go:214 (cpuID -1 until SetCPUID) and vm.go:273 (id == V accepted): the process runs,
    helper 8 returns the ID, a per-CPU array lookup is a fatal map error."""
    from harness import Scenario, packets_to_buffer, run_oracle

    raw, rel = A.assemble([A.call(8), A.mov64_reg(6, 0), A.st(4, 10, -4, 0), A.mov64_reg(2, 10),
                           A.alu64("add", 2, -4), A.ld_map_fd(1, "pc"), A.call(1), A.mov64_reg(0, 6), A.exit_()])
    sc = Scenario(vcpus=2, maps=[dict(name="pc", type=6, key_size=4, value_size=8, max_entries=2)],
                  progs=[("p", raw, rel)])
    buf, off, lens = packets_to_buffer([bytes(8)] * 4)
    o = run_oracle(sc, buf, off, lens, np.array([-1, 2, 1, 3], np.int32))
    from mimic_amd import STATUS_NAMES
    assert [STATUS_NAMES[int(s)] for s in o["status"]] == ["ERR_HELPER_MAP_OP", "ERR_HELPER_MAP_OP", "OK", "ERR_NO_CPU"]
    assert [int(x) for x in o["r0"][:3]] == [2 ** 64 - 1, 2, 1]
