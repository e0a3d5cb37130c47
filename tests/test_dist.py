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


def test_replica_overflow_is_detected():
    import pytest

    blobs = [D.replica_blob({bytes([i]) * 4: bytes(8) for i in range(3)}),
             D.replica_blob({bytes([i]) * 4: bytes(8) for i in range(2, 6)})]
    assert len(D.merge_records(blobs, 4, 8, max_entries=6)) == 6
    with pytest.raises(D.ReplicaOverflow):
        D.merge_records(blobs, 4, 8, max_entries=5)
