"""Multi-GPU plumbing (one process per GPU, torch.distributed; backend "nccl" = RCCL on ROCm).

The hot path shards with no exchange: rank r owns vCPUs [r*Vr, (r+1)*Vr) of one VM whose
address layout is that of the full V = world*Vr machine, and its own packets.  The only
collectives are setup/readout ones: the program bytes are broadcast from rank 0, and the
per-CPU counters' per-key sums are all-reduced (the "sum over CPUs" view of a per-CPU map).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple


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
