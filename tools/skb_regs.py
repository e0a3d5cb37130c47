#!/usr/bin/env python3
"""Register census of the cfg-5 chain kernel under generator knobs (CPU only: hipRTC builds,
code-object metadata).  Each variant compiles in its own worker process.
  python tools/skb_regs.py [VAR=VAL[,VAR=VAL...] ...]"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(spec):
    env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
    os.environ.update(env)
    from mimic_amd import _lib
    from mimic_amd import jit as J
    from mimic_amd import workloads as W
    progs, maps, _ = W.skb_programs()
    vc = J.vc_slots([(p.raw, p.relocs) for p in progs], maps) if os.environ.get("VC", "1") == "1" else []
    src = J.kernel_source([p.raw for p in progs], _lib.CTX_SKB, vc)
    return spec or "default", J.kernel_resources(J.code_object(src))


if __name__ == "__main__":
    specs = sys.argv[1:] or ["", "MIMIC_JIT_NOCOLD=1", "MIMIC_JIT_DEFER_NOREGS=1"]
    with ProcessPoolExecutor(min(8, len(specs))) as ex:
        for name, r in ex.map(one, specs):
            print(f"{name:50s} vgpr {r['vgpr_total']:4d} sgpr {r.get('sgpr', 0):4d} waves {r['waves_per_simd']} "
                  f"spill {r['vgpr_spill']}/{r['sgpr_spill']} scratch {r['scratch']} lds {r['lds']}")
