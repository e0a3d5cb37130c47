#!/usr/bin/env python3
"""Where the time of one cfg-2 launch goes (measurement only).

Runs the bench workload (1 M x 64 B, classifier, V = 262 144, interleaved, rotating batches) on a
JIT kernel built with MIMIC_JIT_MEMTIME=1: every packet's process stores s_memrealtime (100 MHz)
when its lane reaches it (err_pc) and when its results are stored (steps).  From the last launch's
stamps: when lanes start (dispatch ramp), how long each of a lane's 4 packets takes, and when lanes
finish (tail).  Prints one JSON object.

    MIMIC_JIT_MEMTIME=1 python tools/memtime.py [--config classifier] [--launches 30]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="classifier")
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--batches", type=int, default=5)
    args = ap.parse_args()
    assert os.environ.get("MIMIC_JIT_MEMTIME") == "1", "run with MIMIC_JIT_MEMTIME=1"
    os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
    import torch

    import bench
    import mimic_amd as M
    from mimic_amd import workloads as W

    cfg = bench.CONFIGS[args.config]
    n = cfg["packets"]
    V = cfg.get("vcpus") or n // 4
    wl = bench.Workload(args.config, n, W.SEED)
    vm, maps, pids = wl.build_vm(M, V, 0, (0, V), [p.raw for p in wl.progs])
    dev = "cuda:0"
    batches = []
    for b in range(args.batches):
        w = wl if b == 0 else bench.Workload(args.config, n, W.SEED + 1000 * b)
        batches.append((M.XDPBatch.from_numpy(w.buf, w.off, w.lens, device=dev, ingress=1,
                                               schedule=M.SCHED_INTERLEAVED), M.XDPResults.empty(n, dev)))
    st = torch.cuda.Stream(device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in range(args.launches):
        if k == args.launches - 1:
            e0.record(st)
        b, r = batches[k % len(batches)]
        vm.RunXDPBatch(pids[0], b, r, stream=st, sync=False)
    e1.record(st)
    torch.cuda.synchronize()
    last = batches[(args.launches - 1) % len(batches)][1].numpy(n)
    start = last["err_pc"].astype(np.int64) & 0xFFFFFFFF
    end = last["steps"].astype(np.int64) & 0xFFFFFFFF
    t0 = start.min()
    start, end = (start - t0) * 10, (end - t0) * 10   # ns (100 MHz)
    # interleaved schedule: packet i is packet j = i // V of lane i % V
    P = -(-n // V)
    pad = P * V - n
    S = np.concatenate([start, np.full(pad, -1)]).reshape(P, V)
    E = np.concatenate([end, np.full(pad, -1)]).reshape(P, V)

    def pct(x):
        x = x[x >= 0]
        return {q: round(float(np.percentile(x, q)) / 1000, 2) for q in (0, 10, 50, 90, 99, 100)}

    out = {
        "config": args.config, "packets": n, "vcpus": V, "packets_per_lane": P,
        "launch_us_events": round(e0.elapsed_time(e1) * 1000, 2),
        "span_us_stamps": round(float(end.max()) / 1000, 2),
        "lane_start_us": pct(S[0]),
        "lane_end_us": pct(E[P - 1] if pad == 0 else np.maximum(E[P - 1], E[P - 2])),
        "packet_us": {str(j): pct(E[j] - S[j]) for j in range(P)},
        "gap_to_next_packet_us": {str(j): pct(S[j + 1] - E[j]) for j in range(P - 1)},
        "wave_span_us": pct(E.max(axis=0) - S[0]),
        "status_ok": float((last["status"] == 0).mean()),
    }
    print(json.dumps(out))
    vm.close()


if __name__ == "__main__":
    main()
