"""world_size-2 gloo rehearsal of the multi-GPU path on CPU: program broadcast, vCPU sharding
with per-rank packets, and the all-reduced per-CPU counter readout -- checked against one
process running every packet (the oracle stands in for the engine on CPU)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from mimic_amd import dist as D
from mimic_amd import workloads as W

VPR = 16          # vCPUs per rank
N = 2048          # packets per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counters(vm, mid, cpus, E):
    tot = np.zeros(E, np.uint64)
    for c in cpus:
        tot += np.frombuffer(vm.map_values(mid, c), np.uint64)
    return tot


def _rank_main(rank, ws, port, q):
    import torch.distributed as dist

    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    prog = W.prog_classifier()
    raw = D.broadcast_bytes(prog.raw if rank == 0 else None, "cpu")
    assert raw == prog.raw
    b0, cnt = D.shard(VPR, rank)
    vm = oracle.OracleVM(VPR * ws)
    mid = vm.map_create("verdicts", 6, 4, 8, 4)
    pid = vm.prog_load("p", raw, [(s, mid) for s, _ in prog.relocs])
    buf, off, lens = W.make_packets(N, seed=W.SEED + rank)
    cpu = b0 + W.schedule_cpu(N, cnt, "interleaved")
    vm.run_xdp_batch(pid, buf, off, lens, cpu, write_back=False)
    local = _counters(vm, mid, range(b0, b0 + cnt), 4)
    total = D.allreduce_sum_u64(local.tolist(), "cpu")
    mx = D.allreduce_max_f64(float(rank), "cpu")
    q.put((rank, total, mx))
    dist.destroy_process_group()


def test_two_rank_shard_matches_single_process():
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import oracle

    # one process, every packet of both ranks on the same vCPUs
    prog = W.prog_classifier()
    vm = oracle.OracleVM(VPR * ws)
    mid = vm.map_create("verdicts", 6, 4, 8, 4)
    pid = vm.prog_load("p", prog.raw, [(s, mid) for s, _ in prog.relocs])
    for r in range(ws):
        buf, off, lens = W.make_packets(N, seed=W.SEED + r)
        cpu = D.shard(VPR, r)[0] + W.schedule_cpu(N, VPR, "interleaved")
        vm.run_xdp_batch(pid, buf, off, lens, cpu, write_back=False)
    want = _counters(vm, mid, range(VPR * ws), 4).tolist()
    for rank, total, mx in res:
        assert total == want, (rank, total, want)
        assert mx == ws - 1
    assert sum(want) == N * ws


def _hash_rank_main(rank, ws, port, q):
    import torch.distributed as dist

    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    prog = W.prog_flowtrack(max_entries=8192)
    vm = oracle.OracleVM(VPR * ws)
    mid = vm.map_create("flows", 1, 16, 8, 8192)
    pid = vm.prog_load("p", prog.raw, [(s, mid) for s, _ in prog.relocs])
    buf, off, lens = W.make_packets(N, W.IMIX["sizes"], W.IMIX["weights"], seed=W.SEED + rank)
    b0, cnt = D.shard(VPR, rank)
    vm.run_xdp_batch(pid, buf, off, lens, b0 + W.schedule_cpu(N, cnt, "interleaved"), write_back=False)
    vals = vm.map_values(mid, 0)
    mine = {k: vals[s * 8:(s + 1) * 8] for k, s in vm.map_entries(mid)}
    merged = D.merge_hash_replicas(mine, 16, 8, "cpu")
    q.put((rank, sorted(merged.items())))
    dist.destroy_process_group()


def test_two_rank_hash_replicas_merge_to_single_process():
    """cfg 4 over 2 ranks: one hash-map replica per rank, all-gathered and merged, equals one
    process inserting every rank's packets (values are a function of the key)."""
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hash_rank_main, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import oracle

    prog = W.prog_flowtrack(max_entries=8192)
    vm = oracle.OracleVM(VPR * ws)
    mid = vm.map_create("flows", 1, 16, 8, 8192)
    pid = vm.prog_load("p", prog.raw, [(s, mid) for s, _ in prog.relocs])
    for r in range(ws):
        buf, off, lens = W.make_packets(N, W.IMIX["sizes"], W.IMIX["weights"], seed=W.SEED + r)
        vm.run_xdp_batch(pid, buf, off, lens, D.shard(VPR, r)[0] + W.schedule_cpu(N, VPR, "interleaved"),
                         write_back=False)
    vals = vm.map_values(mid, 0)
    want = sorted((k, vals[s * 8:(s + 1) * 8]) for k, s in vm.map_entries(mid))
    assert len(want) > 1000
    for rank, got in res:
        assert got == want, rank


CFG4_N = 1 << 21        # bench.py's cfg-4 packets per GPU
CFG4_VPR = 1 << 18      # and vCPUs per GPU
CFG4_E = 131072


def _flowtrack_oracle(V):
    import oracle

    prog = W.prog_flowtrack()
    assert prog.maps[0]["max_entries"] == CFG4_E
    vm = oracle.OracleVM(V)
    mid = vm.map_create("flows", 1, 16, 8, CFG4_E)
    pid = vm.prog_load("p", prog.raw, [(s, mid) for s, _ in prog.relocs])
    return vm, mid, pid


def _contents(vm, mid):
    vals = vm.map_values(mid, 0)
    return {k: vals[s * 8:(s + 1) * 8] for k, s in vm.map_entries(mid)}


def _cfg4_rank_main(rank, ws, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    buf, off, lens = W.flowtrack_shard(CFG4_N, rank, ws)   # what bench.py's rank r runs
    vm, mid, pid = _flowtrack_oracle(CFG4_VPR * ws)
    b0, cnt = D.shard(CFG4_VPR, rank)
    o = vm.run_xdp_batch(pid, buf, off, lens, b0 + W.schedule_cpu(CFG4_N, cnt, "interleaved"), write_back=False)
    mine = _contents(vm, mid)
    merged = D.merge_hash_replicas(mine, 16, 8, "cpu", CFG4_E)   # raises ReplicaOverflow past E
    q.put((rank, len(mine), sorted(merged.items()), np.bincount(o["r0"].astype(np.int64), minlength=3).tolist()))
    dist.destroy_process_group()


def test_cfg4_bench_size_shards_merge_to_one_oracle_run():
    """cfg 4 as bench.py shards it over 2 ranks (workloads.flowtrack_shard: packets [r*2M,
    (r+1)*2M) of ONE batch, E = 131 072, 262 144 vCPUs per rank): each rank's replica, merged
    over gloo with the MaxEntries check, equals ONE oracle VM running both shards on one shared
    table, key by key; and every rank's verdicts are the single table's (no E2BIG anywhere)."""
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cfg4_rank_main, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    vm, mid, pid = _flowtrack_oracle(CFG4_VPR * ws)
    verdicts = []
    for r in range(ws):
        buf, off, lens = W.flowtrack_shard(CFG4_N, r, ws)
        o = vm.run_xdp_batch(pid, buf, off, lens, D.shard(CFG4_VPR, r)[0] + W.schedule_cpu(CFG4_N, CFG4_VPR, "interleaved"),
                             write_back=False)
        verdicts.append(np.bincount(o["r0"].astype(np.int64), minlength=3).tolist())
    want = sorted(_contents(vm, mid).items())
    assert 120000 < len(want) <= CFG4_E
    for rank, nmine, got, vr in sorted(res):
        assert 110000 < nmine < len(want)       # each replica holds only its own shard's keys
        assert got == want, rank
        assert vr == verdicts[rank], rank        # XDP_DROP only for non-IP frames, never E2BIG


def test_cfg4_keys_of_eight_shards_fit_max_entries():
    """The bound that makes the replica merge exact at 8 GPUs: the 8 bench-size shards of the one
    cfg-4 batch (16M packets) insert at most MaxEntries distinct keys in total."""
    keys = []
    for r in range(8):
        buf, off, lens = W.flowtrack_shard(CFG4_N, r, 8)
        keys.append(W.flow_keys_np(buf, off, lens))
    assert W.distinct_keys(*keys) <= CFG4_E
    assert W.distinct_keys(*keys) > 131000


def test_flow_keys_np_matches_the_program():
    """flow_keys_np / flowtrack_value (bench.py's --launch-selftest readout) against the oracle
    running prog_flowtrack on a shard: the same (key, value) records."""
    buf, off, lens = W.flowtrack_shard(30000, 1, 3)
    vm, mid, pid = _flowtrack_oracle(64)
    vm.run_xdp_batch(pid, buf, off, lens, W.schedule_cpu(30000, 64, "interleaved"), write_back=False)
    want = _contents(vm, mid)
    keys = W.flow_keys_np(buf, off, lens)
    vals = W.flowtrack_value(keys)
    got = {bytes(k): int(v).to_bytes(8, "little") for k, v in zip(np.ascontiguousarray(keys).view(np.uint8).reshape(-1, 16), vals)}
    assert got == want and len(want) > 10000


def test_shard_ranges_are_one_batch():
    """make_packet_range: a packet has the same length and bytes whichever range holds it."""
    whole = W.make_packet_range(0, 3 * 70000, **W.IMIX)
    for lo, hi in ((0, 70000), (70000, 140000), (123, 70123), (200000, 210000)):
        part = W.make_packet_range(lo, hi, **W.IMIX)
        assert np.array_equal(part[2], whole[2][lo:hi])
        for j in range(0, hi - lo, 997):
            a, b, n = int(whole[1][lo + j]), int(part[1][j]), int(part[2][j])
            assert np.array_equal(whole[0][a:a + n], part[0][b:b + n])


def test_replica_overflow_is_detected():
    import pytest

    blobs = [D.replica_blob({bytes([i]) * 4: bytes(8) for i in range(3)}),
             D.replica_blob({bytes([i]) * 4: bytes(8) for i in range(2, 6)})]
    assert len(D.merge_records(blobs, 4, 8, max_entries=6)) == 6
    with pytest.raises(D.ReplicaOverflow):
        D.merge_records(blobs, 4, 8, max_entries=5)
