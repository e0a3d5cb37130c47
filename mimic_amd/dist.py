"""Multi-GPU plumbing (one process per GPU, torch.distributed; backend "nccl" = RCCL on ROCm).

The hot path shards with no exchange: rank r owns vCPUs [r*Vr, (r+1)*Vr) of one VM whose
address layout is that of the full V = world*Vr machine, and its own packets.  The only
collectives are setup/readout ones: the program bytes are broadcast from rank 0, and the
per-CPU counters' per-key sums are all-reduced (the "sum over CPUs" view of a per-CPU map);
a shared hash map is one replica per GPU whose (key, value) records are all-gathered and
merged for the readout.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple


def shard(vcpus_per_rank: int, rank: int) -> Tuple[int, int]:
    """(first vCPU, count) owned by `rank`."""
    return rank * vcpus_per_rank, vcpus_per_rank


def broadcast_bytes(data: Optional[bytes], device, src: int = 0) -> bytes:
    import torch
    import torch.distributed as dist

    n = torch.tensor([len(data) if data is not None else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8, device=device)
    if dist.get_rank() == src and data:
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    if buf.numel():
        dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def allreduce_sum_u64(values: Sequence[int], device) -> List[int]:
    import numpy as np
    import torch
    import torch.distributed as dist

    t = torch.tensor(np.asarray(values, dtype=np.uint64).view(np.int64), device=device)
    dist.all_reduce(t)
    return [int(v) & ((1 << 64) - 1) for v in t.cpu().numpy().tolist()]


def allreduce_max_f64(value: float, device) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_records(records: bytes, rec_size: int, device) -> List[bytes]:
    """All-gather variable-length byte blobs of fixed-size records (one per rank)."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size()
    n = torch.tensor([len(records)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(ws)]
    dist.all_gather(sizes, n)
    mx = max(int(s.item()) for s in sizes)
    buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=device)
    if records:
        buf[:len(records)].copy_(torch.frombuffer(bytearray(records), dtype=torch.uint8))
    outs = [torch.zeros(max(mx, 1), dtype=torch.uint8, device=device) for _ in range(ws)]
    dist.all_gather(outs, buf)
    return [bytes(o[:int(s.item())].cpu().numpy().tobytes()) for o, s in zip(outs, sizes)]


class ReplicaOverflow(RuntimeError):
    """The replicas together hold more keys than the map's MaxEntries: the reference's one shared
    table would have answered E2BIG to some of these inserts, so the sharded run is not exact."""


def merge_records(blobs: Sequence[bytes], key_size: int, value_size: int,
                  max_entries: Optional[int] = None) -> Dict[bytes, bytes]:
    """Merge per-replica (key, value) record blobs in rank order; the first rank's value wins.
    With max_entries, more distinct keys than the map holds raise ReplicaOverflow."""
    rs = key_size + value_size
    merged: Dict[bytes, bytes] = {}
    for blob in blobs:
        for o in range(0, len(blob), rs):
            merged.setdefault(blob[o:o + key_size], blob[o + key_size:o + rs])
    if max_entries is not None and len(merged) > max_entries:
        raise ReplicaOverflow(f"{len(merged)} keys over the replicas, MaxEntries {max_entries}")
    return merged


def replica_blob(contents: Dict[bytes, bytes]) -> bytes:
    return b"".join(k + v for k, v in sorted(contents.items()))


def merge_hash_replicas(contents: Dict[bytes, bytes], key_size: int, value_size: int, device,
                        max_entries: Optional[int] = None) -> Dict[bytes, bytes]:
    """Shared hash map over N GPUs kept as one replica per GPU (SURVEY 8(e) option 1): gather
    every replica's (key, value) records and keep the first rank's value for each key.  Exact
    for insert-if-absent programs whose values are a function of the key (cfg 4) as long as the
    replicas together stay within MaxEntries (checked when max_entries is given).  A rank does
    not see the keys other ranks inserted during the batch."""
    blobs = allgather_records(replica_blob(contents), key_size + value_size, device)
    return merge_records(blobs, key_size, value_size, max_entries)
