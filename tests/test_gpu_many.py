"""mimic_run_xdp_many (VM.RunXDPMany): several device batches of one program as ONE launch of the
owned spread kernel -- every vCPU runs its packets of batch 0, then batch 1, ... (a processPool
draining a backlog of batches, vm.go:548-573) -- against the oracle running the same batches one
after another on one VM: per packet R0 / status / steps / err_pc of every batch, every packet byte,
and the per-CPU counters at the end."""
import numpy as np
import pytest

from harness import Scenario, build_engine, build_oracle, ncpus, spread_kernel_of
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


def _sc(p, V):
    return Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def jit_kernels():
    return [spread_kernel_of(_sc(W.prog_classifier(), V), own=True) for V in (4096, 1000)] + \
        [spread_kernel_of(_sc(W.prog_parse5(), 1024), own=True)]


def _run(sc, batches, sched, expect_exec):
    import mimic_amd as M

    ovm, omids, opids = build_oracle(sc)
    outs = []
    for buf, off, lens in batches:
        cpu = W.schedule_cpu(len(lens), sc.vcpus, sched)
        b = buf.copy()
        o = ovm.run_xdp_batch(opids[0], b, off, lens, cpu, 0, 0, 1, 0, 0)
        o["pkt"] = b
        outs.append(o)
    omaps = {m["name"]: [ovm.map_values(omids[m["name"]], c) for c in range(ncpus(sc, m))] for m in sc.maps}
    ovm.close()
    vm, maps, pids = build_engine(sc)
    s = M.SCHED_INTERLEAVED if sched == "interleaved" else M.SCHED_CHUNKED
    dev = [M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", ingress=1, schedule=s) for buf, off, lens in batches]
    res = vm.RunXDPMany(pids[0], dev)
    assert vm.LastExec() == expect_exec
    for k, (o, r, d) in enumerate(zip(outs, res, dev)):
        e = r.numpy(len(batches[k][2]))
        for f in ("r0", "status", "steps", "err_pc"):
            a, b = np.asarray(o[f]).astype(np.int64), np.asarray(e[f]).astype(np.int64)
            bad = np.nonzero(a != b)[0]
            assert len(bad) == 0, f"batch {k} {f} differs at {bad[:6]}"
        assert np.array_equal(o["pkt"], d.pkt_data.cpu().numpy()), f"batch {k} packet memory"
    for m in sc.maps:
        for c in range(ncpus(sc, m)):
            assert maps[m["name"]].Values(c) == omaps[m["name"]][c], f"map {m['name']} cpu {c}"
    vm.close()


@pytest.mark.parametrize("sched", ["interleaved", "chunked"])
def test_five_rotated_batches_one_launch(gpu, sched):
    """cfg 2's shape scaled down: 5 batches of 16 384 x 64 B at V = 4 096 (4 packets per vCPU per
    batch), the classifier, one owned launch."""
    sc = _sc(W.prog_classifier(), 4096)
    batches = [W.make_packets(16384, seed=W.SEED + 31 * k) for k in range(5)]
    _run(sc, batches, sched, "spread_own")


@pytest.mark.parametrize("sched", ["interleaved", "chunked"])
def test_eight_rotated_batches_one_launch(gpu, sched):
    """The bench's default: 8 batches (MIMIC_MANY_MAX) in one owned launch, cfg 2's shape scaled down."""
    sc = _sc(W.prog_classifier(), 4096)
    batches = [W.make_packets(16384, seed=W.SEED + 17 * k) for k in range(8)]
    _run(sc, batches, sched, "spread_own")


def test_eight_batches_at_bench_size(gpu):
    """cfg 2 at bench size, as the default bench line runs it: 8 batches of 1 048 576 x 64 B at
    V = 262 144 in one launch, every packet and every counter row exact."""
    sc = _sc(W.prog_classifier(), 1 << 18)
    batches = [W.make_packets(1 << 20, seed=W.SEED + k) for k in range(8)]
    _run(sc, batches, "interleaved", "spread_own")


def test_ragged_batches_and_more_than_eight(gpu):
    """10 batches (two launches: 8 + 2) of 3 001 packets at V = 1 000 (3-4 packets per vCPU)."""
    sc = _sc(W.prog_classifier(), 1000)
    batches = [W.make_packets(3001, seed=W.SEED + 7 * k) for k in range(10)]
    _run(sc, batches, "interleaved", "spread_own")


def test_parse5_imix_batches(gpu):
    """parse5's 2 KiB counter rows over 3 IMIX batches at V = 1 024 (16 packets per vCPU)."""
    sc = _sc(W.prog_parse5(), 1024)
    batches = [W.make_packets(16384, **W.IMIX, seed=W.SEED + k) for k in range(3)]
    _run(sc, batches, "interleaved", "spread_own")


def test_programs_without_the_owned_form_run_batch_by_batch(gpu):
    """flowtrack (a hash map) has no spread form: the call runs one launch per batch, same results."""
    p = W.prog_flowtrack(max_entries=1 << 15)
    sc = _sc(p, 64)
    batches = [W.make_packets(2000, **W.IMIX, seed=W.SEED + k) for k in range(3)]
    # one vCPU lane each for 64 vCPUs, interleaved: the engine and the oracle insert in the same
    # order per vCPU, but vCPUs race -- compare per key through the maps' contents instead of slots
    import mimic_amd as M

    ovm, omids, opids = build_oracle(sc)
    vm, maps, pids = build_engine(sc)
    dev = [M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", ingress=1, schedule=M.SCHED_INTERLEAVED)
           for buf, off, lens in batches]
    res = vm.RunXDPMany(pids[0], dev)
    assert vm.LastExec() == "jit"
    for (buf, off, lens), r in zip(batches, res):
        o = ovm.run_xdp_batch(opids[0], buf.copy(), off, lens, W.schedule_cpu(len(lens), 64, "interleaved"), 0, 0, 1, 0, 0)
        e = r.numpy(len(lens))
        assert np.array_equal(np.asarray(o["r0"]).astype(np.int64), np.asarray(e["r0"]).astype(np.int64))
    want = {bytes(k): ovm.map_values(omids["flows"], 0)[s * 8:(s + 1) * 8] for k, s in ovm.map_entries(omids["flows"])}
    got = {k: v[0] for k, v in maps["flows"].Contents().items()}
    assert want == got
    ovm.close()
    vm.close()
