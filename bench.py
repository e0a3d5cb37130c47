#!/usr/bin/env python3
"""bench.py -- Mpkts/s (and eBPF insns/s) of the MI355X batch-eBPF engine, device-resident.

A *step* is one pass of the hot path over one batch: for every packet of the batch,
NewProcess + SetCPUID + Run + read R0 + Cleanup (vm.go:198-374), i.e. one mimic_run_xdp (or
mimic_run_skb) launch.  Default workload = BASELINE.json configs[1]: 1 048 576 x 64 B xdp_md
packets, the ~36-slot parse+hash DROP/PASS classifier, per-CPU array map (E=4, S=8), one MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config classifier|pass8|parse5|flowtrack|skb]

With N > 1 run under torch.distributed.run: every rank owns its own vCPUs and its own packet
shard (weak scaling, no data-path collective); RCCL broadcasts the program bytes at setup and
all-reduces the per-CPU verdict counters after the timed region (the sum-over-CPUs readout).

roofline.traffic / valu_busy come from a committed rocprofv3 summary (profiles/*_pmc_*.json,
written by tools/pmc_summary.py) whose kernel-source hash, workload and vCPU count match this
run exactly; with no such profile they are null.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip table

CONFIGS = {
    "pass8": dict(prog="prog_pass8", packets=1 << 20, sizes=(64,), weights=(1,), reads_packet=False,
                  workload="cfg1-shape: 8-insn XDP_PASS over 1M x 64B xdp_md (reads ctx fields, no packet bytes)"),
    # many: batches per launch by default (mimic_run_xdp_many: a processPool draining its backlog,
    # vm.go:548-573; every batch's packets all run, ms_per_step stays per 1M-packet batch); --many 1
    # is the one-batch-per-launch line
    "classifier": dict(prog="prog_classifier", packets=1 << 20, sizes=(64,), weights=(1,), many=8,
                       workload="cfg2: 1M x 64B xdp_md, 36-slot parse+hash DROP/PASS classifier, "
                                "per-CPU array E=4 S=8"),
    "parse5": dict(prog="prog_parse5", packets=1 << 24, sizes=(64, 576, 1500), weights=(7, 4, 1), vcpus=1 << 18,
                   workload="cfg3: 16M IMIX 7:4:1 (64/576/1500B) xdp_md, L2/L3/L4 parse + 5-tuple hash, "
                            "per-CPU array E=256 S=8"),
    "flowtrack": dict(prog="prog_flowtrack", packets=1 << 21, sizes=(64, 576, 1500), weights=(7, 4, 1), vcpus=1 << 18,
                      one_batch=True,
                      workload="cfg4 per-GPU shard: packets [r*2M, (r+1)*2M) of ONE 2M*N IMIX xdp_md batch (16M over "
                               "8 GPUs), 5-tuple parse + insert-if-absent into a shared hash map K=16 S=8 E=131072"),
    "flowtrack_insert": dict(prog="prog_flowtrack", packets=1 << 21, sizes=(64, 576, 1500), weights=(7, 4, 1),
                             vcpus=1 << 18, reset_maps=True, one_batch=True,
                             workload="cfg4 per-GPU shard, inserting: 2M IMIX xdp_md into a FRESH shared hash map "
                                      "K=16 S=8 E=131072 every step (map reset in the timed region), ~118K inserts "
                                      "per batch"),
    # V = 128K: the chain kernel holds 2 waves per SIMD (242 VGPRs), so 131 072 lanes fill the 1 024
    # SIMDs once (64K: 1 wave, 0.553 ms; 256K: two rounds, 0.428 ms; 128K: 0.409 ms per step)
    "skb": dict(kind="skb", packets=1 << 20, sizes=(64, 576, 1500), weights=(7, 4, 1), vcpus=1 << 17,
                workload="cfg5: 1M IMIX sk_buff contexts, 5-program tail-call chain (~230 slots): __sk_buff "
                         "fields, LD_ABS/IND parse, hash flow lookups, per-CPU counters"),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def reach_kind(cfg_name: str) -> str:
    return {"flowtrack_insert": "flowtrack"}.get(cfg_name, cfg_name)


def algorithmic_bytes(wl, vcpus: int) -> int:
    """Bytes one launch must move, SURVEY.md 8(d) with the packet term made exact: per packet the
    32-byte sectors holding the frame bytes the programs can read (workloads.packet_reach: the
    headers they parse, with their bounds checks; never more than L) + 8 (descriptor) + 8 (r0);
    sk_buff contexts also the 96 room bytes Load hands over zeroed and the sector the verdict
    program's one-byte packet store writes; per batch 2*V*E*S of per-CPU array state, 2*E*(K+S) of
    hash-map state (K + V*S for a per-CPU hash), 2*E*S of plain arrays.  (SURVEY's L per packet
    charged the 1500-byte packets' payloads no program reads: cfg 3 came out at frac 1.25.)"""
    from mimic_amd import workloads as W

    reach = wl.reach if wl.reach is not None else W.packet_reach(reach_kind(wl.name), wl.buf, wl.off, wl.lens)
    wl.reach = reach
    maps = wl.maps
    n = len(wl.lens)
    b = int(W.read_sector_bytes(reach).sum()) + 16 * n
    if wl.skb:
        b += (W.SKB_HEADROOM + W.SKB_TAILROOM + W.SECTOR) * n
    for m in maps:
        if m["type"] in (1, 5):
            ncpu = vcpus if m["type"] == 5 else 1
            b += 2 * m["max_entries"] * (m["key_size"] + ncpu * m["value_size"])
        else:
            ncpu = vcpus if m["type"] == 6 else 1
            b += 2 * ncpu * m["max_entries"] * m["value_size"]
    return b


# ---------------------------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------------------------
class Workload:
    """The programs, maps and input batch of one config (host side).

    Configs with a shared hash map (cfg 4: "one_batch") shard ONE batch: rank r of N takes
    packets [r*n, (r+1)*n) of an N*n batch drawn from one flow pool (workloads.flowtrack_shard),
    so the ranks' replicas together hold the keys of that one batch (<= MaxEntries).  The
    per-CPU configs draw each rank's packets from its own seed (their vCPUs are disjoint)."""

    def __init__(self, cfg_name: str, n: int, seed: int, rank: int = 0, world: int = 1, batch: int = 0):
        from mimic_amd import workloads as W

        self.cfg = CONFIGS[cfg_name]
        self.name = cfg_name
        self.skb = self.cfg.get("kind") == "skb"
        if self.cfg.get("one_batch"):
            p = getattr(W, self.cfg["prog"])()
            self.progs, self.maps, self.prog_array = [p], p.maps, []
            self.buf, self.off, self.lens = W.flowtrack_shard(n, rank, world, batch, W.SEED)
            self.map_init = []
        elif self.skb:
            self.progs, self.maps, self.prog_array = W.skb_programs()
            self.buf, self.off, self.lens = W.make_skb_packets(n, self.cfg["sizes"], self.cfg["weights"], seed=seed,
                                                               variety=0.05)
            m = min(n, 1 << 16)
            self.map_init = [("flows", k, v) for k, v in W.skb_flow_keys(self.buf, self.off[:m], self.lens[:m])]
        else:
            p = getattr(W, self.cfg["prog"])()
            self.progs, self.maps, self.prog_array = [p], p.maps, []
            self.buf, self.off, self.lens = W.make_packets(n, self.cfg["sizes"], self.cfg["weights"], seed=seed)
            self.map_init = []
        self.ctx = 1 if self.skb else 0
        self.reach = None   # per-packet read reach (algorithmic_bytes), computed once

    def kernel_src_hash(self, spread_vcpus: int = 0, own: bool = False) -> str:
        return kernel_src_hash_of(self.name, spread_vcpus, own)

    def build_vm(self, M, V, device, shard, raws):
        emu = M.NewLinuxEmulator()
        vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(V), M.VMOptDevice(device), M.VMOptShard(*shard))
        maps = {}
        for m in self.maps:
            mm = M.MapSpecToLinuxMap(M.MapSpec(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"]))
            emu.AddMap(m["name"], mm)
            maps[m["name"]] = mm
        pids = [vm.AddProgram(M.ProgramSpec(p.name, raw, p.relocs)) for p, raw in zip(self.progs, raws)]
        for mname, key, pi in self.prog_array:
            assert maps[mname].UpdateProgram(key.to_bytes(4, "little"), pids[pi]) == 0
        for mname, key, val in self.map_init:
            assert maps[mname].Update(key, val, 0, 0) == 0
        return vm, maps, pids


def kernel_src_hash_of(cfg_name: str, spread_vcpus: int = 0, own: bool = False) -> str:
    """sha256 (16 hex) of the JIT kernel source the config's programs generate (spread_vcpus > 0:
    the spread kernel a VM of that many vCPUs per engine builds; own: its owned form): the key that
    ties a committed rocprofv3 summary to the exact kernel it measured."""
    from mimic_amd import jit as J
    from mimic_amd import workloads as W

    cfg = CONFIGS[cfg_name]
    if cfg.get("kind") == "skb":
        progs, ctx = W.skb_programs()[0], 1
    else:
        progs, ctx = [getattr(W, cfg["prog"])()], 0
    if spread_vcpus:
        maps = progs[0].maps
        src = J.kernel_source([p.raw for p in progs], ctx, (),
                              J.spread_spec([(p.raw, p.relocs) for p in progs], maps, spread_vcpus, own=own))
    else:
        src = J.kernel_source([p.raw for p in progs], ctx)
    h = hashlib.sha256(src.encode())
    for f in ("mimic_amd/csrc/layout.h", "mimic_amd/csrc/hashmap.h", "mimic_amd/csrc/skb.h", "mimic_amd/csrc/runtime.h",
              "include/mimic_amd.h"):   # the headers embedded into every JIT kernel
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def cpu_baseline(wl: Workload, min_seconds: float, threads: int = 1):
    """The oracle (C restatement of the reference algorithm) on a bounded sample of the same
    workload: `threads` host threads, each one vCPU of a V = threads VM running its own chunk of
    the sample in order (processPool's one-worker-per-vCPU shape, vm.go:521-573); ctypes releases
    the GIL for every batch call, so the threads run the C code in parallel."""
    import oracle

    n = min(len(wl.lens), 1 << 18)
    chunk = (n + threads - 1) // threads
    if wl.skb:
        # every sk_buff process leaks three memory-controller entries and AddEntry's first-fit scan
        # walks them (memory_controller.go:58-112): the reference's per-packet cost grows with the
        # batch.  Batches of 4096 per fresh VM keep that term small (the rate is an upper bound).
        n = min(n, 4096 * threads)
        chunk = 4096
    done = [0] * threads
    steps = [0] * threads
    stop = threading.Event()

    def make_vm():
        vm = oracle.OracleVM(threads)
        mids = {m["name"]: vm.map_create(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"])
                for m in wl.maps}
        pids = [vm.prog_load(p.name, p.raw, [(s, mids[nm]) for s, nm in p.relocs]) for p in wl.progs]
        for mname, key, pi in wl.prog_array:
            vm.map_update(mids[mname], key.to_bytes(4, "little"), vm.prog_addr(pids[pi]).to_bytes(4, "little"))
        for mname, key, val in wl.map_init:
            vm.map_update(mids[mname], key, val, 0, 0)
        return vm, pids[0]

    def worker(t):
        a, b = t * chunk, min(n, (t + 1) * chunk)
        off, lens = wl.off[a:b], wl.lens[a:b]
        cpu = np.full(b - a, t, np.int32)
        vm, pid = make_vm()
        while not stop.is_set():
            if wl.skb:
                o = vm.run_skb_batch(pid, wl.buf, off, lens, cpu, 1, 0, write_back=False)
                # sk_buff processes leak their entries (context_sk_buff.go:110-119): a fresh VM per
                # pass keeps the 32-bit address space from running out
                vm.close()
                vm, pid = make_vm()
            else:
                o = vm.run_xdp_batch(pid, wl.buf, off, lens, cpu, write_back=False)
            done[t] += b - a
            steps[t] += int(o["steps"].astype(np.int64).sum())
        vm.close()

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(min_seconds)
    stop.set()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    tot = sum(done)
    return dict(value=tot / dt / 1e6, unit="Mpkts/s", cores=threads, kind="port",
                insns_per_s=sum(steps) / dt,
                sample=f"{tot} packets of the first {n} packets of the {wl.name} workload, {threads} thread(s) x "
                       f"1 vCPU chunk each (V = {threads}), C oracle, {dt:.1f} s")


def host_threads() -> int:
    """Host threads this job may use: the affinity mask, capped at the 16-CPU share of one GPU."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))


def default_batches(cfg_name: str, n: int) -> int:
    """Batches the timed region rotates over by default: enough that their packets, descriptors
    and results exceed ROTATE_BYTES (mean packet size of the config's mix)."""
    cfg = CONFIGS[cfg_name]
    w = np.asarray(cfg["weights"], np.float64)
    mean = float((np.asarray(cfg["sizes"], np.float64) * w).sum() / w.sum())
    return max(1, -(-ROTATE_BYTES // int(n * (mean + 21))))


def read_profile(cfg_name: str, kernel: str, src_hash: str, n: int, vcpus: int, batches: int = 1,
                 sched: str = "interleaved", per_launch: int = 1):
    """The committed rocprofv3 summary of exactly this kernel (source hash) on this workload."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if (d.get("config") == cfg_name and d.get("kernel") == kernel and d.get("kernel_src_hash") == src_hash
                and d.get("packets") == n and d.get("vcpus") == vcpus and d.get("batches", 1) == batches
                and d.get("schedule", "interleaved") == sched and d.get("batches_per_launch", 1) == per_launch):
            best = dict(d, file=os.path.relpath(f, ROOT))
    return best


def host_resident_rate(vm, pid, wl, sched, chunks: int = 0, reps: int = 5):
    """Packets start and end in host memory: mimic_run_xdp_host pipelines sub-batches (H2D of
    packet bytes + descriptors, the kernel, D2H of r0 + status) on separate streams.  The host
    arrays are pinned once (hipHostRegister) like NIC / capture buffers would be."""
    buf = wl.buf
    n = len(wl.lens)
    off = np.ascontiguousarray(wl.off, dtype=np.uint64)
    lens = np.ascontiguousarray(wl.lens, dtype=np.uint32)
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps: the barrier + synchronize around the region cost ~35 us once, 6 % of 20
    # cfg-2 steps (26 us each) but 1 % of 100
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="classifier", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: the config's)")
    ap.add_argument("--vcpus", type=int, default=0, help="vCPUs per GPU (default: the config's, else packets/4)")
    ap.add_argument("--sched", default="interleaved", choices=["chunked", "interleaved"])
    ap.add_argument("--batches", type=int, default=0,
                    help="distinct input batches the timed launches rotate over (default: enough that the "
                         f"working set exceeds {ROTATE_BYTES >> 20} MiB, so no batch is served from the "
                         "256 MiB Infinity Cache)")
    ap.add_argument("--many", type=int, default=0,
                    help="batches per launch (mimic_run_xdp_many, up to 8: one owned-spread launch runs K of the "
                         "rotated batches back to back); --steps counts launches, ms_per_step stays per batch "
                         "(0: the config's default, 5 for the classifier, else 1)")
    ap.add_argument("--digest", action="store_true",
                    help="add sha256 digests of every rank's per-packet R0 (batch 0, after the timed region) and "
                         "of the merged hash map's (key, value) records to the line (tests/test_gpu_bench_dist.py)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-resident", action="store_true", help="skip the PCIe-inclusive rate")
    ap.add_argument("--rccl", action="store_true",
                    help="run the multi-GPU setup / readout collectives over RCCL even at world size 1 "
                         "(a one-GPU rehearsal of the N-rank path: program broadcast, counter all-reduce, "
                         "hash replica merge)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend of the N-rank path: nccl (= RCCL, tensors on the rank's GPU) or "
                         "gloo (CPU tensors): with --one-device, N engine ranks share GPU 0, so the whole "
                         "N-rank sequence runs on a one-GPU box")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank runs its engine on GPU 0 (a rehearsal of the N-rank path on one GPU; "
                         "value is then not a scaling number)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="CPU rehearsal of the --gpus N launcher: gloo ranks run the setup / readout "
                         "collectives with no engine and rank 0 prints the launch facts")
    return ap.parse_args(argv)


# Working set the timed region must exceed: MI355X_MICROARCH.md's 256 MiB Infinity Cache (MALL)
# serves re-read lines and FETCH_SIZE counts those hits, so a batch re-launched from cache would
# report a cache rate as an HBM rate.
ROTATE_BYTES = 384 << 20


def launch_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) outside torch.distributed: start N ranks with torch.distributed.run,
    one process per GPU, and exit with its status.  Nothing here touches the GPU (counting
    devices does not initialise HIP on this image); the ranks are children, not an exec."""
    import socket
    import subprocess

    if not args.launch_selftest and not args.one_device:
        import torch

        have = torch.cuda.device_count()
        if have < args.gpus:
            sys.stderr.write(f"bench.py --gpus {args.gpus}: only {have} GPU(s) visible on this node; "
                             f"one rank per GPU needs {args.gpus}\n")
            return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    return subprocess.call(cmd, env=env)


def selftest_rank(args, ws, rank, local) -> None:
    """--launch-selftest: what a rank does around the engine, on gloo/CPU -- program broadcast,
    max-over-ranks time, counter all-reduce, hash-replica merge -- then rank 0 reports."""
    import torch.distributed as dist

    from mimic_amd import dist as D
    from mimic_amd import workloads as W

    dist.init_process_group("gloo")
    p = getattr(W, CONFIGS[args.config].get("prog", "prog_classifier"))()
    raw = D.broadcast_bytes(p.raw if rank == 0 else None, "cpu")
    ranks = D.allgather_records(bytes([rank, local]), 2, "cpu")
    elapsed = D.allreduce_max_f64(0.001 * (rank + 1), "cpu")
    counters = D.allreduce_sum_u64([rank + 1, 1], "cpu")
    cfg = CONFIGS[args.config]
    if cfg.get("one_batch"):
        # cfg 4: this rank's shard of the one batch, the (key, value) records its replica would
        # hold (what the program inserts, computed from the headers), merged over the ranks with
        # the map's MaxEntries check -- the readout the engine ranks run, at bench size
        n = args.packets or cfg["packets"]
        wl = Workload(args.config, n, W.SEED, rank, ws)
        keys = W.flow_keys_np(wl.buf, wl.off, wl.lens)
        vals = W.flowtrack_value(keys)
        kb = np.ascontiguousarray(keys).view(np.uint8).reshape(-1, 16)
        mine = {bytes(k): int(v).to_bytes(8, "little") for k, v in zip(kb, vals)}
        m0 = wl.maps[0]
        merged = D.merge_hash_replicas(mine, m0["key_size"], m0["value_size"], "cpu", m0["max_entries"])
    else:
        merged = D.merge_hash_replicas({bytes([rank]) * 4: bytes(8)}, 4, 8, "cpu")
    if rank == 0:
        print(json.dumps({"n_gpus": ws, "gpus_flag": args.gpus, "program_ok": raw == p.raw,
                          "ranks": [b[0] for b in ranks], "local_ranks": [b[1] for b in ranks],
                          "elapsed_max": elapsed, "counters": counters, "hash_keys": len(merged)}), flush=True)
    dist.destroy_process_group()


def make_batches(wl, args, n, rank, dev, sched):
    """The timed launches rotate over `nb` distinct seeded batches of the config's workload (each
    its own packets, descriptors and results)."""
    import mimic_amd as M
    from mimic_amd import workloads as W

    # (a config that runs several batches per launch rotates over at least that many: no batch twice
    # in one launch)
    nb = args.batches or max(default_batches(args.config, n), 1 if args.many else CONFIGS[args.config].get("many", 1))
    ws = dist_env()[0]
    out = []
    for b in range(nb):
        # a one-batch config rotates over further shards of the same batch (same flow pool)
        w = wl if b == 0 else Workload(args.config, n, W.SEED + rank + 1000 * b, rank, ws, b)
        if wl.skb:
            batch = M.SKBBatch.from_numpy(w.buf, w.off, w.lens, device=dev, ifindex=1, schedule=sched)
        else:
            batch = M.XDPBatch.from_numpy(w.buf, w.off, w.lens, device=dev, ingress=1, schedule=sched)
        out.append((w, batch, M.XDPResults.empty(n, dev, full=False)))
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    ws, rank, local = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    if ws != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}; launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop --gpus\n")
        return 2
    if args.launch_selftest:
        selftest_rank(args, ws, rank, local)
        return 0
    # compiled JIT kernels persist here across runs
    os.environ.setdefault("MIMIC_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
    os.makedirs(os.environ["MIMIC_JIT_CACHE"], exist_ok=True)

    import torch

    gpu = 0 if args.one_device else local   # the device this rank's engine runs on
    if torch.cuda.device_count() <= gpu:
        sys.stderr.write(f"bench.py rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} "
                         f"GPU(s) visible\n")
        return 2
    use_dist = ws > 1 or args.rccl   # the collective paths; at world size 1 only with --rccl
    gloo = args.dist_backend == "gloo"
    if gloo and args.rccl:
        sys.stderr.write("bench.py: --rccl and --dist-backend gloo exclude each other\n")
        return 2
    json_out = sys.stdout
    if use_dist:
        # RCCL writes its banner to file descriptor 1 when a communicator starts: native writes to
        # stdout go to stderr from here on, the one JSON line to the original stdout
        json_out = os.fdopen(os.dup(1), "w")
        sys.stdout.flush()
        os.dup2(2, 1)
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(ws))
        torch.cuda.set_device(gpu)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
    dev = torch.device(f"cuda:{gpu}")
    torch.cuda.set_device(dev)
    cdev = "cpu" if gloo else dev   # where the collectives' tensors live

    import mimic_amd as M
    from mimic_amd import dist as D
    from mimic_amd import workloads as W

    cfg = CONFIGS[args.config]
    n = args.packets or cfg["packets"]
    vpg = args.vcpus or cfg.get("vcpus") or max(64, n // 4)
    V = vpg * ws
    wl = Workload(args.config, n, W.SEED + rank, rank, ws)

    # program bytes: built on rank 0, broadcast over RCCL (the setup-time exchange)
    raws = [D.broadcast_bytes(p.raw if rank == 0 else None, cdev) if use_dist else p.raw for p in wl.progs]
    vm, maps, pids = wl.build_vm(M, V, gpu, D.shard(vpg, rank), raws)
    pid = pids[0]

    sched = M.SCHED_INTERLEAVED if args.sched == "interleaved" else M.SCHED_CHUNKED
    batches = make_batches(wl, args, n, rank, dev, sched)
    nb = len(batches)
    stream = torch.cuda.Stream(device=dev)

    reset = [maps[m["name"]] for m in wl.maps] if cfg.get("reset_maps") else []

    K = max(1, args.many or min(cfg.get("many", 1), nb))   # (the default never repeats a batch in a launch)
    if K > 1 and (wl.skb or reset or nb % K and nb > K):
        sys.stderr.write("bench.py: --many needs an xdp_md config without map resets and a batch count K divides\n")
        return 2

    def launch_many(k):   # batches k*K .. k*K + K - 1 (mod nb) in one mimic_run_xdp_many call
        sel = [batches[(k * K + q) % nb] for q in range(K)]
        vm.RunXDPMany(pid, [b for _, b, _ in sel], [r for _, _, r in sel], stream=stream, sync=False)

    def launch(k):
        if K > 1:
            launch_many(k)
            return
        w, batch, res = batches[k % nb]
        for m in reset:   # a fresh map per step: every flow of the batch is inserted again
            m.Reset(stream)
        if wl.skb:
            vm.RunSKBBatch(pid, batch, res, stream=stream, sync=False)
            vm.SKBRelease()   # the batch's leaked sk_buff entries: a long run would exhaust 32-bit addresses
        else:
            vm.RunXDPBatch(pid, batch, res, stream=stream, sync=False)

    for k in range(args.warmup):
        launch(k)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    # device time of the timed region: two HIP events on the stream the kernels run on, around the
    # K back-to-back launches (an event pair per launch would itself sit between the kernels)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        launch(args.warmup + k)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    region_ms = ev0.elapsed_time(ev1)
    st = np.concatenate([res.status[:n].cpu().numpy() for _, _, res in batches])
    timed = [((args.warmup + k) * K + q) % nb for k in range(args.steps) for q in range(K)]
    if use_dist:
        elapsed = D.allreduce_max_f64(elapsed, cdev)

    # sum-over-CPUs readout of the per-CPU counters (RCCL all-reduce across ranks); shared hash
    # maps: one replica per GPU, (key, value) records merged
    counters = None
    hash_keys = None
    pcm = [m for m in wl.maps if m["type"] == 6 and m["value_size"] == 8]
    hm = [m for m in wl.maps if m["type"] == 1]
    if hm and not wl.skb:
        m0 = hm[0]
        mine = {k: v[0] for k, v in maps[m0["name"]].Contents().items()}
        merged = D.merge_hash_replicas(mine, m0["key_size"], m0["value_size"], cdev, m0["max_entries"]) if use_dist else mine
        hash_keys = len(merged)
    if pcm:
        b0, cnt = D.shard(vpg, rank)
        local_sum = maps[pcm[0]["name"]].SumU64(b0, b0 + cnt)
        counters = D.allreduce_sum_u64(local_sum, cdev) if use_dist else local_sum
    digests = None
    if args.digest:   # per-packet and per-key evidence for the N-rank tests (nothing timed)
        import hashlib

        h = hashlib.sha256(batches[0][2].r0[:n].cpu().numpy().astype(np.uint64).tobytes()).digest()
        digests = {"r0": [d.hex() for d in (D.allgather_records(h, 32, cdev) if use_dist else [h])]}
        if hm and not wl.skb:
            digests["hash"] = hashlib.sha256(b"".join(k + v for k, v in sorted(merged.items()))).hexdigest()

    # eBPF instructions per batch (exact per-lane step counts): one more untimed launch of each
    # batch after the readout above
    steps_of = []
    for b in range(nb):
        if K > 1:   # one batch per launch here: LastSteps of exactly this batch
            vm.RunXDPBatch(pid, batches[b][1], batches[b][2], stream=stream, sync=False)
        else:
            launch(b)
        torch.cuda.synchronize(dev)
        steps_of.append(vm.LastSteps())
    steps_timed = float(sum(steps_of[b] for b in timed))
    if use_dist:
        steps_timed = float(D.allreduce_sum_u64([int(steps_timed)], cdev)[0])

    if rank == 0:
        total_pkts = n * ws * args.steps * K
        value = total_pkts / elapsed / 1e6
        avg_launch_s = region_ms / (args.steps * K) / 1e3   # per batch (a launch runs K), gaps included
        alg_of = {b: algorithmic_bytes(batches[b][0], vpg) for b in set(timed)}
        alg = sum(alg_of[b] for b in timed) / len(timed)
        achieved = alg / avg_launch_s
        kernel = "mimic_jit_kernel" if vm.LastExec() in ("jit", "spread", "spread_own") else "mimic_xdp_kernel"
        src_hash = wl.kernel_src_hash(vpg if vm.LastExec() in ("spread", "spread_own") else 0, vm.LastExec() == "spread_own")
        prof = read_profile(args.config, kernel, src_hash, n, vpg, nb, args.sched, K)
        # a profiled launch ran K batches: its bytes and time per batch, like alg and avg_launch_s
        prof_ns = (prof.get("kernel_stats") or {}).get("avg_ns") / K if prof and (prof.get("kernel_stats") or {}).get("avg_ns") else None
        prof_bytes = prof["bytes_per_launch"] / K if prof and prof.get("bytes_per_launch") else None
        out = {
            "metric": "Mpkts/s (device-resident, one XDP program over 64-1500B batches)",
            "value": round(value, 3),
            "unit": "Mpkts/s",
            "n_gpus": ws,
            "steps": args.steps * K,   # batches (a step is one pass over one batch); launches below
            "warmup": args.warmup,
            "launches": args.steps,
            "ms_per_step": round(elapsed / (args.steps * K) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded PCG64 packet mix, SURVEY.md 8(d))",
            "config": {"workload": cfg["workload"], "packets_per_gpu": n, "vcpus_per_gpu": vpg,
                       "schedule": args.sched, "parallelism": f"dp{ws}", "batches_rotated": nb,
                       "working_set_bytes": sum(int(w.buf.nbytes) + 21 * n for w, _, _ in batches),
                       "program_slots": sum(len(p.raw) // 8 for p in wl.progs), "engine": vm.LastExec(),
                       "kernel_src_hash": src_hash, "batches_per_launch": K},
            "insns_per_s": round(steps_timed / elapsed, 1),
            "mean_insns_per_packet": round(steps_timed / (n * ws * args.steps * K), 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 3), "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK, 5),
                         "traffic": prof_bytes,
                         "traffic_over_algorithmic": round(prof_bytes / alg, 3) if prof_bytes else None,
                         # the profile's measured bytes over the profile's own kernel time (one rocprofv3
                         # session: traffic and time from the same runs, not from this line's)
                         "frac_on_traffic": round(prof_bytes / (prof_ns * 1e-9) / HBM_PEAK, 5)
                                            if prof_ns and prof_bytes else None,
                         "profile_kernel_ms": round(prof_ns * 1e-6, 4) if prof_ns else None,
                         "valu_busy": prof.get("valu_busy") if prof else None,
                         "profile": prof["file"] if prof else None,
                         "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(avg_launch_s * 1e3, 4)},
            "status_ok_frac": float((st == 0).mean()),
            "counters_sum": counters,
            "hash_keys": hash_keys,
        }
        if digests:
            out["digests"] = digests
        if use_dist:
            out["collectives"] = f"{'gloo' if gloo else 'rccl'}, world size {ws}"
        if args.one_device and ws > 1:
            out["one_device"] = True   # N engine ranks shared GPU 0: a rehearsal, not a scaling point
        if not args.no_host_resident and ws == 1 and not wl.skb:
            out["host_resident"] = host_resident_rate(vm, pid, wl, sched)
        if not args.no_cpu_baseline and ws == 1:
            one = cpu_baseline(wl, args.cpu_seconds, 1)
            T = host_threads()
            allc = cpu_baseline(wl, args.cpu_seconds, T) if T > 1 else one
            out["cpu_baseline"] = dict(one, all_cores=allc)
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.destroy_process_group()
    vm.close()


if __name__ == "__main__":
    sys.exit(main())
