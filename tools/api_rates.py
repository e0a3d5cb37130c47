#!/usr/bin/env python3
"""Rates of the reference-shaped API (vm.go:198-235, 343-360, 500-573) on MI355X -- what a Go caller
that binds NewProcess / Run / ProcessPool one process at a time gets, next to the batch entry points
(DESIGN.md 6.5).  Prints one JSON object.

  process_run_xdp   NewProcess + SetCPUID + Run + Cleanup per call, classifier, 64 B packets
  process_run_skb   the same for an sk_buff process of the cfg-5 chain (NewProcess runs the Load)
  pool_xdp          ProcessPool: N xdp_md jobs (NewProcess + Enqueue each, handoff counts them)
  pool_skb          ProcessPool: N sk_buff jobs of the cfg-5 chain, processes made beforehand
                    (NewProcess timed separately): one launch per micro-batch (mimic_process_run_many)
  pool_skb_per_job  the same jobs run one Process.Run each (what round 4's pool did)
  oracle_*          the C oracle (the reference restated) on one host thread, per process

    python tools/api_rates.py [--xdp-jobs 1048576] [--skb-jobs 65536]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--xdp-jobs", type=int, default=1 << 20)
    ap.add_argument("--skb-jobs", type=int, default=1 << 16)
    ap.add_argument("--per-job", type=int, default=2048, help="sk_buff jobs timed through Process.Run one by one")
    ap.add_argument("--calls", type=int, default=300)
    args = ap.parse_args()
    os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
    import mimic_amd as M
    import oracle
    from harness import Scenario, build_engine, build_oracle
    from mimic_amd import workloads as W

    out = {}
    p = W.prog_classifier()
    V = 256
    sc = Scenario(vcpus=V, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    vm, maps, pids = build_engine(sc)
    buf, off, lens = W.make_packets(max(args.calls, 4096), seed=3)
    pk = [bytes(buf[int(o):int(o) + int(n)]) for o, n in zip(off, lens)]

    # ---- Process.Run per call (xdp_md) ----------------------------------------------------------
    def one_xdp(k):
        pr = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pk[k]))
        pr.SetCPUID(k % V)
        pr.Run()
        r0 = pr.Registers.R0
        pr.Cleanup()
        return r0

    for k in range(64):   # past the Run tier-up (MIMIC_PROC_JIT, 32 Runs) and its one hipRTC build
        one_xdp(k)
    t0 = time.perf_counter()
    for k in range(args.calls):
        one_xdp(k)
    dt = time.perf_counter() - t0
    out["process_run_xdp"] = {"us_per_call": round(dt / args.calls * 1e6, 1), "calls": args.calls,
                              "what": "NewProcess + SetCPUID + Run + Cleanup, classifier, 64 B"}

    # ---- the same four calls straight through the C ABI (what a cgo binding calls; the Python
    # mirror's Run also reads the packet back and fills its register fields) ----------------------
    import ctypes as C
    from mimic_amd import _lib as L
    pr0 = vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=pk[0]))
    pr0._ensure_native()
    prog_id, c0 = pr0.prog_id, pr0.Context
    pr0.Cleanup()
    lib, hv, regs = vm.lib, vm.h, L.ProcessRegs()

    def one_cabi(k):
        h = C.c_void_p()
        if lib.mimic_process_new(hv, prog_id, pk[k], len(pk[k]), c0.Headroom, c0.Tailroom, c0.IngessIfIndex,
                                 c0.RxQueueIndex, c0.EgressIfIndex, C.byref(h)) != 0:
            raise RuntimeError("mimic_process_new")
        if lib.mimic_process_set_cpu(h, k % V) != 0 or lib.mimic_process_run(h, 0, C.byref(regs)) != 0:
            raise RuntimeError("mimic_process_set_cpu / _run")
        r0 = int(regs.r[0])
        lib.mimic_process_free(h)
        return r0

    for k in range(20):
        assert one_cabi(k) == one_xdp(k)
    t0 = time.perf_counter()
    for k in range(args.calls):
        one_cabi(k)
    dt = time.perf_counter() - t0
    out["process_run_xdp_cabi"] = {"us_per_call": round(dt / args.calls * 1e6, 1), "calls": args.calls,
                                   "what": "mimic_process_new + _set_cpu + _run + _free through ctypes, classifier, 64 B"}
    # where a call's time goes: each C-ABI call timed alone (medians), next to a torch op + sync
    parts = {"new": [], "set_cpu": [], "run": [], "free": []}
    for k in range(args.calls):
        h = C.c_void_p()
        t0 = time.perf_counter()
        lib.mimic_process_new(hv, prog_id, pk[k], len(pk[k]), c0.Headroom, c0.Tailroom, c0.IngessIfIndex,
                              c0.RxQueueIndex, c0.EgressIfIndex, C.byref(h))
        t1 = time.perf_counter()
        lib.mimic_process_set_cpu(h, k % V)
        t2 = time.perf_counter()
        lib.mimic_process_run(h, 0, C.byref(regs))
        t3 = time.perf_counter()
        lib.mimic_process_free(h)
        t4 = time.perf_counter()
        for key, d in zip(parts, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            parts[key].append(d * 1e6)
    import torch
    x = torch.zeros(16, device="cuda:0")
    lat = []
    for _ in range(args.calls):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t0) * 1e6)
    out["process_run_xdp_cabi_split_us"] = {k: round(float(np.median(v)), 1) for k, v in parts.items()}
    out["process_run_xdp_cabi_split_us"]["torch_op_plus_sync"] = round(float(np.median(lat)), 1)
    out["process_run_xdp_cabi_split_us"]["run_exec"] = vm.LastExec()
    # the same C-ABI calls on a VM that never tiers up (every Run on the stepping interpreter)
    os.environ["MIMIC_PROC_JIT"] = "-1"
    vmi, _, pidsi = build_engine(sc)
    del os.environ["MIMIC_PROC_JIT"]
    hvi = vmi.h
    runs = []
    for k in range(args.calls):
        h = C.c_void_p()
        lib.mimic_process_new(hvi, pidsi[0], pk[k], len(pk[k]), 0, 0, c0.IngessIfIndex, 0, 0, C.byref(h))
        lib.mimic_process_set_cpu(h, k % V)
        t0 = time.perf_counter()
        lib.mimic_process_run(h, 0, C.byref(regs))
        runs.append((time.perf_counter() - t0) * 1e6)
        lib.mimic_process_free(h)
    out["process_run_xdp_cabi_split_us"]["run_interp"] = round(float(np.median(runs[32:])), 1)
    vmi.close()

    # ---- ProcessPool, xdp_md jobs ------------------------------------------------------------------
    n = args.xdp_jobs
    bufx, offx, lensx = W.make_packets(n, seed=5)
    pool = vm.GetProcessPool()
    pool.Start(1 << 16)
    done = [0]
    mu = threading.Lock()
    ev = threading.Event()

    def handoff(proc, err):
        with mu:
            done[0] += 1
            if done[0] == n:
                ev.set()

    t0 = time.perf_counter()
    for k in range(n):
        o = int(offx[k])
        pool.Enqueue(M.ProcessPoolJob(vm.NewProcess(pids[0], M.LinuxContextXDP(Packet=bytes(bufx[o:o + int(lensx[k])]))),
                                      None, None))
    pool.Stop()
    dt = time.perf_counter() - t0
    out["pool_xdp"] = {"jobs": n, "seconds": round(dt, 2), "jobs_per_s": round(n / dt, 1),
                       "what": "NewProcess + Enqueue per job from one Python thread, Stop() waits for all"}
    vm.close()

    # ---- host map operations between launches (launch -> Update -> launch) ---------------
    # cfg 4's table (E = 131 072, 16-byte keys): every launch may write it, so the host image pages in
    # on demand after each (engine.cpp HashMirror); the host ops themselves are timed
    fp = W.prog_flowtrack()
    fsc = Scenario(vcpus=4096, maps=fp.maps, progs=[(fp.name, fp.raw, fp.relocs)])
    fvm, fmaps, fpids = build_engine(fsc)
    fb, fo, fl = W.make_packets(65536, **W.IMIX, seed=17)
    fbatch = M.XDPBatch.from_numpy(fb, fo, fl, device="cuda:0", schedule=M.SCHED_INTERLEAVED)
    fvm.RunXDPBatch(fpids[0], fbatch)
    ops = {"update_new_key": [], "lookup": [], "update_then_lookup_4": []}
    rng = np.random.default_rng(23)
    for it in range(60):
        fvm.RunXDPBatch(fpids[0], fbatch)   # may write the table: the host image is stale after it
        key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        t0 = time.perf_counter()
        fmaps["flows"].Update(key, (it).to_bytes(8, "little"), 0)
        ops["update_new_key"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        fmaps["flows"].Lookup(key)
        ops["lookup"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        for q in range(4):
            k2 = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            fmaps["flows"].Update(k2, b"\0" * 8, 0)
            fmaps["flows"].Lookup(k2)
        ops["update_then_lookup_4"].append(time.perf_counter() - t0)
    out["host_ops_after_launch"] = {k: {"median_us": round(float(np.median(v[5:])) * 1e6, 1),
                                        "p90_us": round(float(np.percentile(v[5:], 90)) * 1e6, 1)} for k, v in ops.items()}
    out["host_ops_after_launch"]["what"] = ("cfg-4 table (E = 131 072, 16-byte keys) written by a 65 536-packet launch "
                                            "before each round: the first Update after the launch, a Lookup, then 4 more "
                                            "Update + Lookup pairs (Python calls through the C ABI)")
    fvm.close()

    # ---- sk_buff processes of the cfg-5 chain ------------------------------------------------------
    progs, smaps, pa = W.skb_programs()
    ns = args.skb_jobs
    bs, os_, ls = W.make_skb_packets(ns, **W.IMIX, variety=0.05, seed=9)
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(bs, os_[:4096], ls[:4096])]
    ssc = Scenario(vcpus=V, maps=smaps, progs=[(q.name, q.raw, q.relocs) for q in progs], prog_array=pa, map_init=init)
    svm, _, spids = build_engine(ssc, ctx=1)
    spk = [bytes(bs[int(o) + 32:int(o) + 32 + int(L)]) for o, L in zip(os_, ls)]

    def make(k):
        try:
            return svm.NewProcess(spids[0], M.LinuxContextSKBuff(Packet=spk[k], Dev=M.NetDev(IFIndex=1)))
        except M.MimicError:
            return None

    for k in range(10):   # warm
        pr = make(k)
        if pr is not None:
            pr.SetCPUID(0)
            pr.Run()
            pr.Cleanup()
    t0 = time.perf_counter()
    c = 0
    for k in range(args.calls):
        pr = make(k)
        if pr is None:
            continue
        pr.SetCPUID(k % V)
        pr.Run()
        pr.Cleanup()
        c += 1
    dt = time.perf_counter() - t0
    out["process_run_skb"] = {"us_per_call": round(dt / max(c, 1) * 1e6, 1), "calls": c,
                              "what": "NewProcess (its Load: prep launch + sync) + SetCPUID + Run + Cleanup, cfg-5 chain"}

    def pool_run(procs, per_job):
        pool = svm.GetProcessPool()
        pool.Start(len(procs))
        t0 = time.perf_counter()
        if per_job:   # round 4's pool: one Process.Run each, then the process's Cleanup
            for k, pr in enumerate(procs):
                pr.SetCPUID(k % V)
                try:
                    pr.Run()
                except M.MimicError:
                    pass
                pr.Cleanup()
        else:
            for pr in procs:
                pool.Enqueue(M.ProcessPoolJob(pr, None, None))
        pool.Stop()
        return time.perf_counter() - t0

    # the batched launches run the chain's JIT kernel: built (or read from the cache) before timing
    warm = [q for q in (make(k) for k in range(64)) if q is not None]
    svm.RunProcesses(warm, None, [k % V for k in range(len(warm))])
    svm.CleanupProcesses(warm)
    t0 = time.perf_counter()
    procs = [q for q in (make(k) for k in range(ns)) if q is not None]
    t_new = time.perf_counter() - t0
    dt = pool_run(procs, False)
    out["pool_skb"] = {"jobs": len(procs), "seconds": round(dt, 3), "jobs_per_s": round(len(procs) / dt, 1),
                       "newprocess_us_each": round(t_new / max(len(procs), 1) * 1e6, 1),
                       "what": "Enqueue + micro-batched launches (mimic_process_run_many); NewProcess timed apart"}
    # the same kind of jobs through the C ABI call a Go pool would make per micro-batch
    # (mimic_process_run_many + mimic_process_free_many), without the Python pool's per-job work
    rates = []
    for _ in range(3):   # three rounds of fresh processes: the median
        procs = [q for q in (make(k) for k in range(ns)) if q is not None]
        cpus = [k % V for k in range(len(procs))]
        t0 = time.perf_counter()
        for b in range(0, len(procs), 1 << 16):
            svm.RunProcesses(procs[b:b + (1 << 16)], None, cpus[b:b + (1 << 16)])
            svm.CleanupProcesses(procs[b:b + (1 << 16)])
        rates.append(len(procs) / (time.perf_counter() - t0))
    out["abi_run_many_skb"] = {"jobs": len(procs), "jobs_per_s": round(sorted(rates)[1], 1),
                               "rounds_jobs_per_s": [round(r, 1) for r in rates],
                               "what": "mimic_process_run_many + mimic_process_free_many per 65 536 processes (median of 3)"}
    procs = [q for q in (make(k) for k in range(args.per_job)) if q is not None]
    dt = pool_run(procs, True)
    out["pool_skb_per_job"] = {"jobs": len(procs), "seconds": round(dt, 3), "jobs_per_s": round(len(procs) / dt, 1),
                               "what": "one Process.Run (single-lane launch + sync) + Cleanup per job"}
    out["pool_skb_batched_over_per_job"] = round(out["pool_skb"]["jobs_per_s"] / out["pool_skb_per_job"]["jobs_per_s"], 1)
    out["abi_run_many_over_per_job"] = round(out["abi_run_many_skb"]["jobs_per_s"] / out["pool_skb_per_job"]["jobs_per_s"], 1)
    svm.close()

    # ---- the oracle, one thread, per process -------------------------------------------------------
    ovm, omids, opids = build_oracle(sc)
    m = min(n, 1 << 18)
    t0 = time.perf_counter()
    ovm.run_xdp_batch(opids[0], bufx, offx[:m], lensx[:m], W.schedule_cpu(m, V, "interleaved"), write_back=False)
    dt = time.perf_counter() - t0
    out["oracle_xdp"] = {"processes_per_s": round(m / dt, 1), "processes": m, "threads": 1}
    ovm.close()
    ovm, omids, opids = build_oracle(ssc)
    m = min(ns, 4096)
    t0 = time.perf_counter()
    ovm.run_skb_batch(opids[0], bs, os_[:m], ls[:m], W.schedule_cpu(m, V, "interleaved"), 1, 0, write_back=False)
    dt = time.perf_counter() - t0
    out["oracle_skb"] = {"processes_per_s": round(m / dt, 1), "processes": m, "threads": 1,
                         "note": "one fresh VM per 4 096 processes (the leaked entries make AddEntry's scan grow)"}
    ovm.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
