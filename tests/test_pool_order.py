"""ProcessPool's micro-batch grouping on the host (no device): each (program, context kind) group
of a micro-batch is one launch, and a vCPU never gets jobs of two groups in one segment, so every
vCPU runs its jobs in enqueue order (vm.go:548-573).  The launches are recorded, not run."""
from types import SimpleNamespace

import mimic_amd as M
from mimic_amd.vm import ProcessPool


class _Proc:
    def __init__(self, pid, skb=False):
        self.prog_id = pid
        self.Context = M.LinuxContextSKBuff() if skb else M.LinuxContextXDP()
        self.cpuID = -1
        self.Status = 0
        self._started = False

    def SetCPUID(self, c):
        self.cpuID = c


def _pool(V):
    cleaned = []
    pool = ProcessPool(SimpleNamespace(settings=SimpleNamespace(vcpus=V), CleanupProcesses=cleaned.extend))
    launches = []
    pool._launch = lambda pid, skb, js: launches.append([(j.Process.prog_id, skb, j.Process.cpuID, j.idx) for j in js])
    pool._handoff = lambda job, err: None
    return pool, launches


def _jobs(pattern):
    out = []
    for i, (pid, skb) in enumerate(pattern):
        j = M.ProcessPoolJob(_Proc(pid, skb))
        j.idx = i
        out.append(j)
    return out


def test_groups_split_where_a_vcpu_would_see_a_second_group():
    pool, launches = _pool(2)
    pattern = [(0, False), (0, False), (1, False), (0, False), (1, True), (1, True), (0, False)]
    pool._run(_jobs(pattern))
    order = [x for L in launches for x in L]
    assert sorted(x[3] for x in order) == list(range(len(pattern)))   # every job once
    for cpu in range(2):   # per vCPU: launch order = enqueue order
        seen = [x[3] for x in order if x[2] == cpu]
        assert seen == sorted(seen), (cpu, launches)
    for L in launches:     # one group per launch
        assert len({(x[0], x[1]) for x in L}) == 1


def test_single_group_is_one_launch():
    pool, launches = _pool(4)
    pool._run(_jobs([(3, False)] * 11))
    assert len(launches) == 1 and [x[2] for x in launches[0]] == [0, 1, 2, 3] * 2 + [0, 1, 2]
