#!/usr/bin/env python3
"""Process.Run per call through the C ABI for a few programs (run under rocprofv3 --kernel-trace to
split kernel time from host time): classifier (36 slots, packet + map), pass8 (8 slots, no memory),
loops (the interpreter's per-step cost).  Each on the stepping interpreter (MIMIC_PROC_JIT=-1) and
on the single-process JIT form (MIMIC_PROC_JIT=0; loop programs stay on the interpreter)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import mimic_amd as M
    from harness import Scenario, build_engine
    from mimic_amd import _lib as L
    from mimic_amd import workloads as W

    out = {}
    buf, off, lens = W.make_packets(4096, seed=3)
    pk = [bytes(buf[int(o):int(o) + int(n)]) for o, n in zip(off, lens)]
    from mimic_amd import asm as A

    def loop_prog(n):   # n iterations of a 3-slot loop: the per-step cost once the code is warm
        raw, rel = A.assemble([A.mov64_imm(1, n), A.mov64_imm(0, 0), "l", A.alu64("add", 0, 1, reg=True),
                               A.alu64("add", 1, -1), A.jmp("jne", 1, 0, "l"), A.exit_()])
        return W.Program(f"loop{n}", raw, rel, [])

    for name, mode in [(n, m) for n in ("prog_pass8", "prog_classifier", "prog_flowtrack", "loop100", "loop2000")
                       for m in ("interp", "jit")]:
        if name.startswith("loop") and mode == "jit":
            continue
        p = getattr(W, name)() if name.startswith("prog_") else loop_prog(int(name[4:]))
        sc = Scenario(vcpus=256, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
        os.environ["MIMIC_PROC_JIT"] = "-1" if mode == "interp" else "0"
        vm, maps, pids = build_engine(sc)
        os.environ.pop("MIMIC_PROC_JIT")
        lib, hv, regs = vm.lib, vm.h, L.ProcessRegs()
        ts = {"new": [], "run": [], "free": []}
        for k in range(400):
            h = C.c_void_p()
            t0 = time.perf_counter()
            assert lib.mimic_process_new(hv, pids[0], pk[k], len(pk[k]), 0, 0, 1, 0, 0, C.byref(h)) == 0
            assert lib.mimic_process_set_cpu(h, k % 256) == 0
            t1 = time.perf_counter()
            assert lib.mimic_process_run(h, 0, C.byref(regs)) == 0
            t2 = time.perf_counter()
            lib.mimic_process_free(h)
            t3 = time.perf_counter()
            if k >= 100:
                for key, d in zip(ts, (t1 - t0, t2 - t1, t3 - t2)):
                    ts[key].append(d * 1e6)
        key = f"{name}_{mode}"
        out[key] = {k: round(float(np.median(v)), 1) for k, v in ts.items()}
        out[key]["steps"] = int(regs.steps)
        out[key]["exec"] = vm.LastExec()
        vm.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
