"""Host-resident pipeline probe: mimic_run_xdp_host with registered vs hipHostMalloc'd host memory.
    python tools/host_probe.py [modes] [chunk counts]     e.g.  registered,pinned 0,4,8,16"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import mimic_amd as M  # noqa: E402
from mimic_amd import workloads as W  # noqa: E402

modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["pinned", "registered"]
chunk_list = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 4, 8, 16, 32]
reps = 5
p = W.prog_classifier()
n = 1 << 20
emu = M.NewLinuxEmulator()
vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(n // 4))
for m in p.maps:
    emu.AddMap(m["name"], M.MapSpecToLinuxMap(M.MapSpec(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"])))
pid = vm.AddProgram(M.ProgramSpec(p.name, p.raw, p.relocs))
buf, off, lens = W.make_packets(n)
for mode in modes:
    if mode == "pinned":
        tb = torch.from_numpy(buf).pin_memory(); b = tb.numpy()
        to = torch.from_numpy(off.view(np.int64)).pin_memory(); o = to.numpy().view(np.uint64)
        tl = torch.from_numpy(lens.view(np.int32)).pin_memory(); l_ = tl.numpy().view(np.uint32)
        tr = torch.empty(n, dtype=torch.int64).pin_memory(); r0 = tr.numpy().view(np.uint64)
        ts = torch.empty(n, dtype=torch.uint8).pin_memory(); st = ts.numpy()
    else:
        b, o, l_ = buf, off, lens
        r0, st = np.empty(n, np.uint64), np.empty(n, np.uint8)
        for a in (b, o, l_, r0, st):
            vm.HostRegister(a)
    for chunks in chunk_list:
        vm.RunXDPHost(pid, b, o, l_, schedule=M.SCHED_INTERLEAVED, ingress=1, chunks=chunks, r0=r0, status=st)
        ts_ = []
        for _ in range(reps):
            t = time.perf_counter()
            vm.RunXDPHost(pid, b, o, l_, schedule=M.SCHED_INTERLEAVED, ingress=1, chunks=chunks, r0=r0, status=st)
            ts_.append(time.perf_counter() - t)
        dt = float(np.median(ts_))
        print(mode, chunks, f"median {n / dt / 1e6:.1f} Mpkts/s  {(buf.nbytes + 21 * n) / dt / 1e9:.1f} GB/s  "
              f"(per call ms: {' '.join(f'{x * 1e3:.2f}' for x in ts_)})", flush=True)
vm.close()
