"""Known-answer vectors (tests/golden/kat.json) -> harness scenarios."""
import json
import os

import numpy as np

from harness import Scenario, packets_to_buffer

KAT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat.json")


def load_cases():
    with open(KAT_PATH) as f:
        return json.load(f)["cases"]


def scenario(c):
    progs = [(p["name"], bytes.fromhex(p["raw"]), [tuple(r) for r in p["relocs"]]) for p in c["progs"]]
    map_init = [(m, bytes.fromhex(kk), bytes.fromhex(v), cpu) for m, kk, v, cpu in c["map_init"]]
    return Scenario(vcpus=c["vcpus"], maps=c["maps"], progs=progs, prog_array=[tuple(x) for x in c["prog_array"]],
                    map_init=map_init, max_tail_calls=c["max_tail_calls"])


def inputs(c):
    buf, off, lens = packets_to_buffer([bytes.fromhex(c["packet"])], c["headroom"], c["tailroom"])
    return dict(buf=buf, off=off, lens=lens, cpu=np.array([c["cpu"]], dtype=np.int32), headroom=c["headroom"],
                tailroom=c["tailroom"], step_budget=c["step_budget"])


def check(c, out):
    ex = c["expect"]
    got = {"status": int(out["status"][0]), "err_pc": int(out["err_pc"][0]), "r0": int(out["r0"][0]) & ((1 << 64) - 1),
           "steps": int(out["steps"][0])}
    for k, v in ex.items():
        assert got[k] == v, f"{c['name']} ({c['ref']}): {k} = {got[k]:#x} expected {v:#x}  (got {got})"


def _setup_key(c):
    return json.dumps([c["vcpus"], c["maps"], c["max_tail_calls"], c["map_init"]], sort_keys=True)


def jit_groups(cases, max_progs: int = 40):
    """Single-program KATs with the same VM setup (vCPUs, maps, MaxTailCalls, map init), chunked
    into VMs of up to max_progs programs: one JIT kernel runs a whole chunk, each case with its own
    entry program.  Returns [(scenario, runs, cases)]; multi-program cases are left out."""
    groups = {}
    for c in cases:
        if len(c["progs"]) != 1 or c["prog_array"]:
            continue
        groups.setdefault(_setup_key(c), []).append(c)
    out = []
    for key in sorted(groups):
        cs = groups[key]
        for a in range(0, len(cs), max_progs):
            chunk = cs[a:a + max_progs]
            base = scenario(chunk[0])
            progs = []
            runs = []
            for k, c in enumerate(chunk):
                p = c["progs"][0]
                progs.append((f"k{k}", bytes.fromhex(p["raw"]), [tuple(r) for r in p["relocs"]]))
                i = inputs(c)
                runs.append(dict(entry=k, buf=i["buf"], off=i["off"], lens=i["lens"], cpu=i["cpu"],
                                 headroom=i["headroom"], tailroom=i["tailroom"],
                                 ingress=np.array([c["ingress"]], np.int32), rxq=np.array([c["rxq"]], np.int32),
                                 egress=np.array([c["egress"]], np.int32), step_budget=i["step_budget"]))
            out.append((Scenario(vcpus=base.vcpus, maps=base.maps, progs=progs, prog_array=[],
                                 map_init=base.map_init, max_tail_calls=base.max_tail_calls), runs, chunk))
    return out


def multi_cases(cases):
    return [c for c in cases if len(c["progs"]) != 1 or c["prog_array"]]
