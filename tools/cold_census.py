"""Diagnostics: how many slow-path (cold_*) calls each packet of a bench workload makes in the JIT
kernel.  MIMIC_JIT_CENSUS=1 makes the kernel store, in place of each packet's step count, one
4-bit counter per slow-path kind.
    python tools/cold_census.py [config] [packets]"""
import os
import sys

os.environ["MIMIC_JIT_CENSUS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import mimic_amd as M  # noqa: E402
from mimic_amd import workloads as W  # noqa: E402

KINDS = ["load", "store", "lookup", "update", "delete", "tailcall", "ldabs", "adjust_tail"]
cfg_name = sys.argv[1] if len(sys.argv) > 1 else "skb"
cfg = bench.CONFIGS[cfg_name]
n = int(sys.argv[2]) if len(sys.argv) > 2 else min(cfg["packets"], 1 << 18)
vpg = cfg.get("vcpus") or max(64, n // 4)
dev = torch.device("cuda:0")
wl = bench.Workload(cfg_name, n, W.SEED)
vm, maps, pids = wl.build_vm(M, vpg, 0, (0, vpg), [p.raw for p in wl.progs])
if wl.skb:
    batch = M.SKBBatch.from_numpy(wl.buf, wl.off, wl.lens, device=dev, ifindex=1, schedule=M.SCHED_INTERLEAVED)
    res = vm.RunSKBBatch(pids[0], batch)
else:
    batch = M.XDPBatch.from_numpy(wl.buf, wl.off, wl.lens, device=dev, ingress=1, schedule=M.SCHED_INTERLEAVED)
    res = vm.RunXDPBatch(pids[0], batch)
print("engine", vm.LastExec())
c = res.steps.cpu().numpy().astype(np.uint32)
print(f"{cfg_name}: {n} packets, status ok {float((res.status.cpu().numpy() == 0).mean()):.3f}")
tot = 0
for k, name in enumerate(KINDS):
    v = (c >> (4 * k)) & 15
    tot += int(v.sum())
    if v.any():
        print(f"  {name:12s} mean {v.mean():.3f} per packet, max {v.max()}, packets with any {float((v > 0).mean()):.3f}")
print(f"  total        mean {tot / n:.3f} slow-path calls per packet")
