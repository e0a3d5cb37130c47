"""Host cost of one RunXDPBatch call (tiny batches: launch-bound) and the gap it leaves."""
import sys
import time

import torch

sys.path.insert(0, ".")
import mimic_amd as M  # noqa: E402
from mimic_amd import workloads as W  # noqa: E402

p = W.prog_classifier()
for V in (256, 262144):
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(V))
    for m in p.maps:
        emu.AddMap(m["name"], M.MapSpecToLinuxMap(M.MapSpec(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"])))
    pid = vm.AddProgram(M.ProgramSpec(p.name, p.raw, p.relocs))
    buf, off, lens = W.make_packets(256)
    batch = M.XDPBatch.from_numpy(buf, off, lens, device="cuda:0", schedule=M.SCHED_INTERLEAVED)
    res = M.XDPResults.empty(256, "cuda:0", full=False)
    s = torch.cuda.Stream()
    for _ in range(10):
        vm.RunXDPBatch(pid, batch, res, stream=s, sync=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2000):
        vm.RunXDPBatch(pid, batch, res, stream=s, sync=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"V={V} engine={vm.LastExec()} host per call {(t1 - t) / 2000 * 1e6:.1f} us, wall per call {(t2 - t) / 2000 * 1e6:.1f} us", flush=True)
    vm.close()
