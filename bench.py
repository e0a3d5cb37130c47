#!/usr/bin/env python3
"""bench.py -- Mpkts/s (and eBPF insns/s) of the MI355X batch-eBPF engine, device-resident.

A *step* is one pass of the hot path over one batch: for every packet of the batch,
NewProcess + SetCPUID + Run + read R0 + Cleanup (vm.go:198-374), i.e. one mimic_run_xdp launch.
Default workload = BASELINE.json configs[1]: 1 048 576 x 64 B xdp_md packets, the ~36-slot
parse+hash DROP/PASS classifier, per-CPU array map (E=4, S=8), one MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config classifier|pass8|parse5]

With N > 1 run under torch.distributed.run: every rank owns its own vCPUs and its own packet
shard (weak scaling, no data-path collective); RCCL broadcasts the program bytes at setup and
all-reduces the per-CPU verdict counters after the timed region (the sum-over-CPUs readout).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip table

CONFIGS = {
    "pass8": dict(prog="prog_pass8", packets=1 << 20, sizes=(64,), weights=(1,),
                  workload="cfg1-shape: 8-insn XDP_PASS over 1M x 64B xdp_md"),
    "classifier": dict(prog="prog_classifier", packets=1 << 20, sizes=(64,), weights=(1,),
                       workload="cfg2: 1M x 64B xdp_md, 36-slot parse+hash DROP/PASS classifier, "
                                "per-CPU array E=4 S=8"),
    "parse5": dict(prog="prog_parse5", packets=1 << 24, sizes=(64, 576, 1500), weights=(7, 4, 1), vcpus=1 << 18,
                   workload="cfg3: 16M IMIX 7:4:1 (64/576/1500B) xdp_md, L2/L3/L4 parse + 5-tuple hash, "
                            "per-CPU array E=256 S=8"),
    "flowtrack": dict(prog="prog_flowtrack", packets=1 << 21, sizes=(64, 576, 1500), weights=(7, 4, 1), vcpus=1 << 18,
                      workload="cfg4 per-GPU shard: 2M IMIX xdp_md (16M over 8 GPUs), 5-tuple parse + "
                               "insert-if-absent into a shared hash map K=16 S=8 E=131072"),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def algorithmic_bytes(lens: np.ndarray, vcpus: int, maps) -> int:
    """per packet L + 8 (descriptor) + 8 (r0); per batch 2*V*E*S of per-CPU array
    state, 2*E*(K+S) of hash-map state (K + V*S for a per-CPU hash).
    (The engine's actual descriptor is 12 B and it also writes a 1-B status; not counted.)"""
    b = int(lens.astype(np.int64).sum()) + 16 * len(lens)
    for m in maps:
        if m["type"] in (1, 5):
            ncpu = vcpus if m["type"] == 5 else 1
            b += 2 * m["max_entries"] * (m["key_size"] + ncpu * m["value_size"])
        else:
            ncpu = vcpus if m["type"] == 6 else 1
            b += 2 * ncpu * m["max_entries"] * m["value_size"]
    return b


def cpu_baseline(cfg_name: str, min_seconds: float, vcpus_cpu: int = 8):
    """The oracle (C restatement of the reference algorithm, 1 thread) on a bounded sample."""
    import oracle
    from mimic_amd import workloads as W

    cfg = CONFIGS[cfg_name]
    prog = getattr(W, cfg["prog"])()
    n = min(cfg["packets"], 1 << 18)
    buf, off, lens = W.make_packets(n, cfg["sizes"], cfg["weights"], seed=W.SEED)
    vm = oracle.OracleVM(vcpus_cpu)
    mids = {m["name"]: vm.map_create(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"])
            for m in prog.maps}
    pid = vm.prog_load(prog.name, prog.raw, [(s, mids[nm]) for s, nm in prog.relocs])
    cpu = W.schedule_cpu(n, vcpus_cpu, "chunked")
    done = 0
    steps = 0
    t0 = time.perf_counter()
    while True:
        o = vm.run_xdp_batch(pid, buf, off, lens, cpu, write_back=False)
        done += n
        steps += int(o["steps"].astype(np.int64).sum())
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    vm.close()
    return dict(value=done / dt / 1e6, unit="Mpkts/s", cores=1, kind="port",
                insns_per_s=steps / dt,
                sample=f"{done} packets ({done // n} passes over the first {n} packets of the {cfg_name} workload, "
                       f"{vcpus_cpu} vCPUs, chunked), C oracle single-threaded, {dt:.1f} s")


def read_pmc_traffic(cfg_name: str, kernel: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/*pmc*.json) of the
    same workload and kernel (mimic_jit_kernel / mimic_xdp_kernel)."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("config") == cfg_name and d.get("kernel") == kernel and d.get("bytes_per_launch"):
            best = d
    return best


def host_resident_rate(vm, M, pid, buf, off, lens, sched, dev, chunks: int = 0, reps: int = 5):
    """Packets start and end in host memory: mimic_run_xdp_host pipelines sub-batches (H2D of
    packet bytes + descriptors, the kernel, D2H of r0 + status) on separate streams.  The host
    arrays are pinned once (hipHostRegister) like NIC / capture buffers would be."""
    n = len(lens)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    r0 = np.empty(n, np.uint64)
    st = np.empty(n, np.uint8)
    arrs = (buf, off, lens, r0, st)
    for a in arrs:
        vm.HostRegister(a)
    try:
        vm.RunXDPHost(pid, buf, off, lens, schedule=sched, ingress=1, chunks=chunks, r0=r0, status=st)
        t0 = time.perf_counter()
        for _ in range(reps):
            vm.RunXDPHost(pid, buf, off, lens, schedule=sched, ingress=1, chunks=chunks, r0=r0, status=st)
        dt = time.perf_counter() - t0
    finally:
        for a in arrs:
            vm.HostUnregister(a)
    moved = int(buf.nbytes) + 12 * n + 9 * n
    return {"value": round(n * reps / dt / 1e6, 3), "unit": "Mpkts/s", "chunks": chunks,
            "pcie_bytes_per_batch": moved, "pcie_GBps": round(moved * reps / dt / 1e9, 2),
            "ok_frac": float((st == 0).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="classifier", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--vcpus", type=int, default=0, help="vCPUs per GPU (default: packets/4)")
    ap.add_argument("--sched", default="interleaved", choices=["chunked", "interleaved"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-resident", action="store_true", help="skip the PCIe-inclusive rate")
    args = ap.parse_args()
    # compiled JIT kernels persist here across runs (tools/jit_prewarm.py fills it on a CPU host)
    os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(os.path.dirname(os.path.abspath(__file__)), ".jitcache"))
    os.makedirs(os.environ["MIMIC_JIT_CACHE"], exist_ok=True)

    import torch

    ws, rank, local = dist_env()
    if ws > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    import mimic_amd as M
    from mimic_amd import dist as D
    from mimic_amd import workloads as W

    cfg = CONFIGS[args.config]
    n = args.packets or cfg["packets"]
    vpg = args.vcpus or cfg.get("vcpus") or max(64, n // 4)
    V = vpg * ws

    # program bytes: built on rank 0, broadcast over RCCL (the setup-time exchange)
    prog = getattr(W, cfg["prog"])()
    raw_bytes = D.broadcast_bytes(prog.raw if rank == 0 else None, dev) if ws > 1 else prog.raw

    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(V), M.VMOptDevice(local), M.VMOptShard(*D.shard(vpg, rank)))
    maps = {}
    for m in prog.maps:
        mm = M.MapSpecToLinuxMap(M.MapSpec(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"]))
        emu.AddMap(m["name"], mm)
        maps[m["name"]] = mm
    pid = vm.AddProgram(M.ProgramSpec(prog.name, raw_bytes, prog.relocs))

    buf, off, lens = W.make_packets(n, cfg["sizes"], cfg["weights"], seed=W.SEED + rank)
    sched = M.SCHED_INTERLEAVED if args.sched == "interleaved" else M.SCHED_CHUNKED
    batch = M.XDPBatch.from_numpy(buf, off, lens, device=dev, ingress=1, schedule=sched)
    res = M.XDPResults.empty(n, dev, full=False)  # R0 + status per packet; steps via per-lane counters
    stream = torch.cuda.Stream(device=dev)

    def step():
        vm.RunXDPBatch(pid, batch, res, stream=stream, sync=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    steps_per_batch = vm.LastSteps()
    st = res.status[:n].cpu().numpy()
    if ws > 1:
        elapsed = D.allreduce_max_f64(elapsed, dev)
        steps_total_batch = float(D.allreduce_sum_u64([steps_per_batch], dev)[0])
    else:
        steps_total_batch = float(steps_per_batch)

    # sum-over-CPUs readout of the verdict counters (RCCL all-reduce across ranks)
    counters = None
    hash_keys = None
    if prog.maps:
        m0 = prog.maps[0]
        if m0["type"] == 1:  # shared hash map: one replica per GPU, (key, value) records merged
            mine = {k: v[0] for k, v in maps[m0["name"]].Contents().items()}
            merged = D.merge_hash_replicas(mine, m0["key_size"], m0["value_size"], dev) if ws > 1 else mine
            hash_keys = len(merged)
        else:
            b0, cnt = D.shard(vpg, rank)
            local_sum = maps[m0["name"]].SumU64(b0, b0 + cnt)
            counters = D.allreduce_sum_u64(local_sum, dev) if ws > 1 else local_sum

    if rank == 0:
        total_pkts = n * ws * args.steps
        value = total_pkts / elapsed / 1e6
        avg_launch_s = float(np.mean(kern_ms)) / 1e3
        alg = algorithmic_bytes(lens, vpg, prog.maps)
        achieved = alg / avg_launch_s
        pmc = read_pmc_traffic(args.config, "mimic_jit_kernel" if vm.LastExec() == "jit" else "mimic_xdp_kernel")
        out = {
            "metric": "Mpkts/s (device-resident, one XDP program over 64-1500B batches)",
            "value": round(value, 3),
            "unit": "Mpkts/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded PCG64 packet mix, SURVEY.md 8(d))",
            "config": {"workload": cfg["workload"], "packets_per_gpu": n, "vcpus_per_gpu": vpg,
                       "schedule": args.sched, "parallelism": f"dp{ws}", "program_slots": len(prog.raw) // 8,
                       "engine": vm.LastExec()},
            "insns_per_s": round(steps_total_batch * args.steps / elapsed, 1),
            "mean_insns_per_packet": round(steps_total_batch / (n * ws), 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 3), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 5),
                         "traffic": pmc["bytes_per_launch"] if pmc else None,
                         "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(avg_launch_s * 1e3, 4)},
            "status_ok_frac": float((st == 0).mean()),
            "counters_sum": counters,
            "hash_keys": hash_keys,
        }
        if not args.no_host_resident and ws == 1:
            out["host_resident"] = host_resident_rate(vm, M, pid, buf, off, lens, sched, dev)
        if not args.no_cpu_baseline and ws == 1:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()
    vm.close()


if __name__ == "__main__":
    main()
