#!/usr/bin/env python3
"""Shared hash table across two engines: per-shard DROP counts against the oracle, run concurrently
(two streams) and one after the other, to isolate a concurrency effect from a sharding one."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch

    import mimic_amd as M
    from harness import Scenario, build_engine, build_oracle
    from mimic_amd import workloads as W

    E, V, n = 65536, 64, 20000
    p = W.prog_flowtrack(max_entries=E)
    sc = Scenario(vcpus=2 * V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    sa = W.make_packets(n, **W.IMIX, seed=W.SEED + 3)
    sb = W.make_packets(n, **W.IMIX, seed=W.SEED + 4)
    ca = W.schedule_cpu(n, V, "interleaved").astype(np.int32)
    cb = (W.schedule_cpu(n, V, "interleaved") + V).astype(np.int32)
    ovm, omids, opids = build_oracle(sc)
    oa = ovm.run_xdp_batch(opids[0], sa[0].copy(), sa[1], sa[2], ca, write_back=False)
    ob = ovm.run_xdp_batch(opids[0], sb[0].copy(), sb[1], sb[2], cb, write_back=False)
    ovm.close()
    out = {"oracle_drop": [int((np.asarray(o["r0"]) == 1).sum()) for o in (oa, ob)]}
    for mode in ("concurrent", "sequential", "a_only", "unshared_concurrent"):
        a = build_engine(sc, shard=(0, V))
        b = build_engine(sc, shard=(V, V))
        if mode != "unshared_concurrent":
            b[1]["flows"].Share(a[1]["flows"])
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        mk = lambda s, c: M.XDPBatch.from_numpy(*s, device="cuda:0", schedule=M.SCHED_EXPLICIT, cpu=c)
        ba, bb = mk(sa, ca), mk(sb, cb)
        torch.cuda.synchronize()
        ra = a[0].RunXDPBatch(a[2][0], ba, stream=s1, sync=False)
        if mode == "sequential":
            torch.cuda.synchronize()
        rb = b[0].RunXDPBatch(b[2][0], bb, stream=s2, sync=False) if mode != "a_only" else None
        torch.cuda.synchronize()
        ea = ra.numpy(n)
        rec = {"a_drop": int((np.asarray(ea["r0"]) == 1).sum()),
               "a_mismatch": int((np.asarray(ea["r0"]).astype(np.int64) != np.asarray(oa["r0"]).astype(np.int64)).sum()),
               "a_status": np.unique(np.asarray(ea["status"]), return_counts=True)[1].tolist(),
               "entries_a": len(a[1]["flows"].Entries())}
        if rb is not None:
            eb = rb.numpy(n)
            rec["b_drop"] = int((np.asarray(eb["r0"]) == 1).sum())
            rec["b_mismatch"] = int((np.asarray(eb["r0"]).astype(np.int64) != np.asarray(ob["r0"]).astype(np.int64)).sum())
            rec["entries_b"] = len(b[1]["flows"].Entries())
        rec["exec"] = a[0].LastExec()
        out[mode] = rec
        b[0].close()
        a[0].close()
        print(json.dumps({mode: rec}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
