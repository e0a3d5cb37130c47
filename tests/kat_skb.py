"""sk_buff known-answer vectors (tests/golden/kat_skb.json) -> harness scenarios."""
import json
import os

import numpy as np

from harness import Scenario, skb_packets_to_buffer

KAT_SKB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat_skb.json")


def load_cases():
    with open(KAT_SKB_PATH) as f:
        return json.load(f)["cases"]


def scenario(c):
    return Scenario(vcpus=1, progs=[("main", bytes.fromhex(c["raw"]), [])])


def custom_table(contexts):
    """The mimic_skb_custom table of a vector's contexts (sock / flowKeys JSON, parsed as
    UnmarshalContextJSON parses them), or None."""
    if not contexts:
        return None
    from mimic_amd import vm as V

    ctxs = []
    for cj in contexts:
        cj = cj or {}
        sk = V.SK.FromJSON(cj["sock"]) if cj.get("sock") is not None else None
        if sk is not None and cj.get("nilIPs"):
            sk.ips = None   # a Go SK literal: UnmarshalJSON never set its net.IP fields
        fk = V.FlowKeys.FromJSON(cj["flowKeys"]) if cj.get("flowKeys") is not None else None
        ctxs.append(V.LinuxContextSKBuff(SK=sk, FlowKeys=fk))
    return V.SKBBatch.custom_array(ctxs)


def inputs(c):
    buf, off, lens = skb_packets_to_buffer([bytes.fromhex(p) for p in c["packets"]])
    return dict(buf=buf, off=off, lens=lens, cpu=np.zeros(len(lens), dtype=np.int32), ifindex=c["ifindex"],
                custom=custom_table(c.get("contexts")))


def check(c, out):
    for i, ex in enumerate(c["expect"]):
        got = {"status": int(out["status"][i]), "err_pc": int(out["err_pc"][i]),
               "r0": int(out["r0"][i]) & ((1 << 64) - 1), "steps": int(out["steps"][i])}
        for k, v in ex.items():
            assert got[k] == v, f"{c['name']} ({c['ref']}) packet {i}: {k} = {got[k]:#x} expected {v:#x} (got {got})"


def jit_groups(cases, max_progs: int = 40):
    """All vectors share one setup (1 vCPU, no maps): chunks of max_progs programs per VM, each
    case a batch of its own (sk_buff leaks carry over between the batches, as in the oracle)."""
    out = []
    for a in range(0, len(cases), max_progs):
        chunk = cases[a:a + max_progs]
        progs, runs = [], []
        for k, c in enumerate(chunk):
            progs.append((f"k{k}", bytes.fromhex(c["raw"]), []))
            i = inputs(c)
            runs.append(dict(skb=True, entry=k, buf=i["buf"], off=i["off"], lens=i["lens"], cpu=i["cpu"],
                             ifindex=i["ifindex"], custom=i["custom"]))
        out.append((Scenario(vcpus=1, progs=progs), runs, chunk))
    return out
