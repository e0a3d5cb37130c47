"""The engine's multi-GPU shard path, on one GPU: two engines own vCPUs [0, Vr) and [Vr, 2Vr)
of one V = 2Vr VM (VMOptShard, vcpu_begin != 0 addressing) and each runs its own packets.
Together they must equal ONE oracle run of all packets in order: per-packet R0 / status /
steps, every vCPU's per-CPU map bytes, and (cfg 4) the merged hash replicas' key -> value map."""
import numpy as np
import pytest

from harness import Scenario, build_engine, build_oracle, kernel_of, run_oracle
from mimic_amd import dist as D
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu

VR = 96


def _sc(p, vcpus):
    return Scenario(vcpus=vcpus, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def jit_kernels():
    return [kernel_of(_sc(W.prog_classifier(), 1)), kernel_of(_sc(W.prog_flowtrack(max_entries=65536), 1)),
            kernel_of(_sc(W.prog_flowtrack(), 1))]


def _run_shards(sc, buf, off, lens, cpu, nshards):
    import mimic_amd as M

    V = sc.vcpus
    vr = V // nshards
    outs = []
    for r in range(nshards):
        b0 = r * vr
        sel = np.nonzero((cpu >= b0) & (cpu < b0 + vr))[0]
        vm, maps, pids = build_engine(sc, shard=(b0, vr))
        batch = M.XDPBatch.from_numpy(buf, off[sel], lens[sel], device="cuda:0", schedule=M.SCHED_EXPLICIT,
                                      cpu=cpu[sel])
        res = vm.RunXDPBatch(pids[0], batch).numpy(len(sel))
        vals = {m["name"]: {c: maps[m["name"]].Values(c) for c in range(b0, b0 + vr)}
                for m in sc.maps if m["type"] in (5, 6)}
        hashes = {m["name"]: maps[m["name"]].Contents() for m in sc.maps if m["type"] in (1,)}
        outs.append((sel, res, vals, hashes))
        vm.close()
    return outs


def test_cfg4_bench_size_two_engines_merge_to_oracle(gpu):
    """cfg 4 exactly as `bench.py --gpus 2 --config flowtrack` shards it, on one GPU: two engines
    own vCPUs [0, 262144) and [262144, 524288) (VMOptShard) and each runs its 2M-packet shard of
    the ONE batch (workloads.flowtrack_shard) into its own E = 131 072 replica.  The merged
    replicas (MaxEntries checked) equal one oracle VM running both shards on one table, key by
    key, and the per-packet verdicts are the single table's."""
    import mimic_amd as M

    n, vr, ws = 1 << 21, 1 << 18, 2
    p = W.prog_flowtrack()
    assert p.maps[0]["max_entries"] == 131072
    sc = _sc(p, vr * ws)
    ovm, mids, pids = build_oracle(sc)
    blobs = []
    for r in range(ws):
        buf, off, lens = W.flowtrack_shard(n, r, ws)
        b0 = r * vr
        vm, maps, epids = build_engine(sc, shard=(b0, vr))
        batch = M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", ingress=1, schedule=M.SCHED_INTERLEAVED)
        e = vm.RunXDPBatch(epids[0], batch).numpy(n)
        mine = {k: v[0] for k, v in maps["flows"].Contents().items()}
        vm.close()
        del batch
        o = ovm.run_xdp_batch(pids[0], buf, off, lens, b0 + W.schedule_cpu(n, vr, "interleaved"), ingress=1,
                              write_back=False)
        assert np.array_equal(np.asarray(o["r0"]).astype(np.uint64), np.asarray(e["r0"]).astype(np.uint64)), r
        assert np.array_equal(np.asarray(o["status"]).astype(np.int64), np.asarray(e["status"]).astype(np.int64)), r
        assert 110000 < len(mine) <= 131072
        blobs.append(D.replica_blob(mine))
    vals = ovm.map_values(mids["flows"], 0)
    want = {k: vals[s * 8:(s + 1) * 8] for k, s in ovm.map_entries(mids["flows"])}
    ovm.close()
    merged = D.merge_records(blobs, 16, 8, max_entries=131072)
    assert merged == want and len(want) > 120000


def _merge_results(n, outs):
    r = {k: np.zeros(n, dt) for k, dt in (("r0", np.uint64), ("status", np.int64), ("steps", np.int64),
                                           ("err_pc", np.int64))}
    for sel, res, _, _ in outs:
        for k in r:
            r[k][sel] = np.asarray(res[k]).astype(r[k].dtype)
    return r


@pytest.mark.parametrize("nshards", [2, 3])
def test_classifier_shards_equal_one_run(gpu, nshards):
    p = W.prog_classifier()
    V = VR * nshards
    sc = _sc(p, V)
    n = 20000
    buf, off, lens = W.make_packets(n, seed=3)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    outs = _run_shards(sc, buf, off, lens, cpu, nshards)
    e = _merge_results(n, outs)
    for k in e:
        assert np.array_equal(np.asarray(o[k]).astype(e[k].dtype), e[k]), k
    for _, _, vals, _ in outs:
        for c, v in vals["verdicts"].items():
            assert v == o["maps"]["verdicts"][c], c
    tot = sum(int(np.frombuffer(v, np.uint64).sum()) for _, _, vals, _ in outs for v in vals["verdicts"].values())
    assert tot == n


def test_flowtrack_replicas_merge_to_one_table(gpu):
    """cfg 4: a shared hash map as one replica per shard, merged (first shard wins) -- the same
    key -> value map and the same verdicts as the one shared table of a single run."""
    p = W.prog_flowtrack(max_entries=65536)
    V = 2 * VR
    sc = _sc(p, V)
    n = 30000
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=9)
    cpu = W.schedule_cpu(n, V, "interleaved")
    o = run_oracle(sc, buf, off, lens, cpu)
    outs = _run_shards(sc, buf, off, lens, cpu, 2)
    e = _merge_results(n, outs)
    assert np.array_equal(np.asarray(o["r0"]).astype(np.uint64), e["r0"])
    assert np.array_equal(np.asarray(o["status"]).astype(np.int64), e["status"])
    blobs = [D.replica_blob({k: v[0] for k, v in h["flows"].items()}) for _, _, _, h in outs]
    merged = D.merge_records(blobs, 16, 8, max_entries=65536)
    want = {k: v[0] for k, v in o["hash"]["flows"].items()}
    assert merged == want
    assert len(merged) > 1000

