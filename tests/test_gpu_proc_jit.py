"""Process.Run tiering (engine.cpp process_advance, jit.cpp Gen::proc): once a VM has made
MIMIC_PROC_JIT Runs, a fresh xdp_md process on one of the engine's vCPUs runs on the program set's
single-process JIT form instead of the stepping interpreter.  Everything Run leaves readable must
not depend on which ran it (vm.go:343-360, Readme.md:74-78): every register R0..R10, PC, the
program, the step count, the fatal status, the packet memory, and the maps.

* every single-program KAT (tests/golden/kat.json, pinned to the reference's tests through the
  oracle) as a sequence of processes in one VM per setup chunk, interpreter VM against JIT VM;
* the multi-program KATs (tail calls, empty programs) likewise, one VM each;
* the bench programs over IMIX packets on many vCPUs (per-CPU counters, hash inserts, E2BIG);
* the tier-up point: the first N Runs on the interpreter, then the compiled form."""
import os

import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, build_engine, kernel_of, ncpus
from kat import jit_groups, load_cases, multi_cases, scenario
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu

CASES = load_cases()
GROUPS = jit_groups(CASES)
MULTI = multi_cases(CASES)
PROGS = ("prog_classifier", "prog_pass8", "prog_flowtrack", "prog_parse5")


def _wl(name):
    p = getattr(W, name)(max_entries=128) if name == "prog_flowtrack" else getattr(W, name)()
    return Scenario(vcpus=64, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def jit_kernels():
    scs = [sc for sc, _, _ in GROUPS] + [scenario(c) for c in MULTI] + [_wl(n) for n in PROGS]
    out = []
    for sc in scs:
        raws, ctx, vc = kernel_of(sc)
        out += [(raws, ctx, vc), (raws, ctx | 0x100, vc)]   # the batch kernel and the single-process form
    return out


def _engine(sc, after):
    old = os.environ.get("MIMIC_PROC_JIT")
    os.environ["MIMIC_PROC_JIT"] = str(after)
    try:
        return build_engine(sc)
    finally:
        if old is None:
            del os.environ["MIMIC_PROC_JIT"]
        else:
            os.environ["MIMIC_PROC_JIT"] = old


def _run(vm, pid, pkt, H=0, T=0, ingress=1, rxq=0, egress=0, cpu=0, budget=0):
    p = vm.NewProcess(pid, M.LinuxContextXDP(Packet=pkt, Headroom=H, Tailroom=T, IngessIfIndex=ingress,
                                             RxQueueIndex=rxq, EgressIfIndex=egress))
    if cpu >= 0:
        p.SetCPUID(cpu)
    err = None
    try:
        p.Run(budget)
    except M.MimicError as e:
        err = str(e)
    r = p.Registers
    out = dict(regs=[getattr(r, f"R{q}") for q in range(11)], pc=r.PC, prog=getattr(p, "ProgramID", None), steps=p.Steps,
               status=p.Status, err=err, pkt=p.Packet(), exec=vm.LastExec())
    p.Cleanup()
    return out


def _maps(sc, maps):
    out = {}
    for m in sc.maps:
        mm = maps[m["name"]]
        out[m["name"]] = [bytes(mm.Values(c)) for c in range(ncpus(sc, m))]
        if m["type"] in (1, 5):   # hash maps: which key is in which slot
            out[m["name"] + "/entries"] = sorted(mm.Entries())
    return out


def _compare(sc, seq, tag, want_jit=1):
    """seq: [(entry program, run kwargs)], run in order on an interpreter VM and a JIT VM."""
    res = []
    for after in (-1, 0):
        vm, maps, pids = _engine(sc, after)
        res.append(([_run(vm, pids[e], **kw) for e, kw in seq], _maps(sc, maps)))
        vm.close()
    (a, am), (b, bm) = res
    for k, (x, y) in enumerate(zip(a, b)):
        for f in ("regs", "pc", "prog", "steps", "status", "err", "pkt"):
            assert x[f] == y[f], f"{tag} run {k}: {f} interp {x[f]} jit {y[f]} (jit run on {y['exec']}; errors {x['err']} / {y['err']})"
        assert x["exec"] == "interp"
    assert am == bm, f"{tag}: maps differ"
    n_jit = sum(y["exec"] == "jit" for y in b)
    assert n_jit >= want_jit, f"{tag}: {n_jit} of {len(b)} Runs on the single-process form"
    return n_jit


@pytest.mark.parametrize("g", range(len(GROUPS)), ids=[f"chunk{k}_{len(g[2])}" for k, g in enumerate(GROUPS)])
def test_kat_chunk_interp_vs_proc_jit(gpu, g):
    sc, runs, chunk = GROUPS[g]
    seq = [(k, dict(pkt=bytes.fromhex(c["packet"]), H=c["headroom"], T=c["tailroom"], ingress=c["ingress"],
                    rxq=c["rxq"], egress=c["egress"], cpu=c["cpu"], budget=c["step_budget"]))
           for k, c in enumerate(chunk)]
    # (a KAT whose program loops, whose CPU ID is unset / V, or whose budget is below the
    # program's bound stays on the interpreter: the chunk as a whole must still use the form)
    _compare(sc, seq, f"chunk {g}", want_jit=0)


def test_kat_chunks_use_the_form(gpu):
    """Most single-program KATs are loop-free with a set CPU: the form must carry them."""
    total = 0
    for sc, runs, chunk in GROUPS[:3]:
        seq = [(k, dict(pkt=bytes.fromhex(c["packet"]), H=c["headroom"], T=c["tailroom"], ingress=c["ingress"],
                        rxq=c["rxq"], egress=c["egress"], cpu=c["cpu"], budget=c["step_budget"]))
               for k, c in enumerate(chunk)]
        total += _compare(sc, seq, "chunk", want_jit=0)
    assert total > 0


@pytest.mark.parametrize("c", MULTI, ids=[c["name"] for c in MULTI])
def test_kat_multi_interp_vs_proc_jit(gpu, c):
    seq = [(0, dict(pkt=bytes.fromhex(c["packet"]), H=c["headroom"], T=c["tailroom"], ingress=c["ingress"],
                    rxq=c["rxq"], egress=c["egress"], cpu=c["cpu"], budget=c["step_budget"]))]
    _compare(scenario(c), seq, c["name"], want_jit=0)


@pytest.mark.parametrize("name", PROGS)
def test_bench_programs_interp_vs_proc_jit(gpu, name):
    """300 IMIX processes on 64 vCPUs; flowtrack's 128-entry table fills (E2BIG packets)."""
    sc = _wl(name)
    buf, off, lens = W.make_packets(300, **W.IMIX, seed=W.SEED + 17)
    rng = np.random.default_rng(5)
    seq = [(0, dict(pkt=bytes(buf[int(o):int(o) + int(n)]), cpu=int(rng.integers(0, 64)),
                    H=int(rng.integers(0, 3)) * 8, T=int(rng.integers(0, 2)) * 16))
           for o, n in zip(off, lens)]
    assert _compare(sc, seq, name, want_jit=300) == 300


def test_tier_up_after_n_runs(gpu):
    sc = _wl("prog_classifier")
    vm, maps, pids = _engine(sc, 3)
    buf, off, lens = W.make_packets(1, seed=1)
    pkt = bytes(buf[int(off[0]):int(off[0]) + int(lens[0])])
    got = [_run(vm, pids[0], pkt, cpu=k)["exec"] for k in range(6)]
    assert got == ["interp"] * 3 + ["jit"] * 3
    assert _run(vm, pids[0], pkt, cpu=-1)["exec"] == "interp"   # no CPU ID: the interpreter
    vm.close()


def test_processes_from_many_threads(gpu):
    """processPool's pattern: NewProcess / SetCPUID / Run / Step / Cleanup from several
    threads on one VM at once -- the engine serialises them per VM and recycles process blocks
    behind fences.  Every process's R0 equals the oracle's for its packet, and the per-CPU counters
    equal the oracle's (sums: the interleaving of the threads does not change them)."""
    import threading

    from harness import build_oracle

    sc = _wl("prog_classifier")
    n, T = 1200, 4
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=W.SEED + 29)
    pk = [bytes(buf[int(o):int(o) + int(m)]) for o, m in zip(off, lens)]
    cpus = [k % 64 for k in range(n)]
    ovm, omids, opids = build_oracle(sc)
    want = ovm.run_xdp_batch(opids[0], buf.copy(), off, lens, np.array(cpus, np.int32), ingress=np.ones(n, np.int32),
                             write_back=False)
    wmap = [ovm.map_values(omids[sc.maps[0]["name"]], c) for c in range(64)]
    ovm.close()
    vm, maps, pids = _engine(sc, 8)
    got = [None] * n
    errs = []

    def work(t):
        try:
            for k in range(t, n, T):
                p = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pk[k], IngessIfIndex=1))
                p.SetCPUID(cpus[k])
                if k % 7 == 0:   # a few stepped first: those stay on the interpreter
                    p.Step()
                p.Run()
                got[k] = p.Registers.R0
                p.Cleanup()
        except Exception as e:   # noqa: BLE001 (reported below)
            errs.append(repr(e))

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:3]
    assert got == [int(v) for v in np.asarray(want["r0"])]
    assert [bytes(maps[sc.maps[0]["name"]].Values(c)) for c in range(64)] == [bytes(v) for v in wmap]
    vm.close()
