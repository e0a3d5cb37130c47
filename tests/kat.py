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
