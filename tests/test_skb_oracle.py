"""The CPU oracle's sk_buff path (oracle/mimic_oracle.c, restating context_sk_buff.go and
emulator_linux_sk_buff.go) against the hand-derived vectors of tests/golden/kat_skb.json, plus
host-side checks of the engine's sk_buff workload generators.  No GPU."""
import numpy as np
import pytest

import kat_skb
from harness import run_oracle_skb

CASES = kat_skb.load_cases()


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_skb_kat(c):
    inp = kat_skb.inputs(c)
    out = run_oracle_skb(kat_skb.scenario(c), inp["buf"], inp["off"], inp["lens"], inp["cpu"], ifindex=inp["ifindex"])
    kat_skb.check(c, out)


def test_kat_skb_fixture_is_current():
    """kat_skb.json is what make_golden_skb.py writes (the fixture is regenerated, not edited)."""
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(kat_skb.KAT_SKB_PATH), "make_golden_skb.py")
    spec = importlib.util.spec_from_file_location("make_golden_skb", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert [c["name"] for c in mod.CASES] == [c["name"] for c in CASES]
    assert mod.CASES == CASES


def test_oracle_skb_store_writes_packet_be():
    """A BigEndian u16 store through skb->data lands in the written-back packet memory."""
    c = next(c for c in CASES if c["name"] == "pkt_be_store")
    inp = kat_skb.inputs(c)
    out = run_oracle_skb(kat_skb.scenario(c), inp["buf"], inp["off"], inp["lens"], inp["cpu"])
    o = int(inp["off"][0])
    assert bytes(out["pkt"][o + 32:o + 34]) == b"\xab\xcd"
    assert not out["pkt"][o:o + 32].any()                      # headroom zeroed
    L = int(inp["lens"][0])
    assert not out["pkt"][o + 32 + L:o + 96 + L].any()         # tailroom zeroed


def test_skb_workload_variety_hits_every_walk_branch():
    from mimic_amd import workloads as W

    rng = np.random.Generator(np.random.PCG64(7))
    kinds = set()
    for _ in range(400):
        f = W.skb_variant(rng, int(rng.choice([14, 40, 64, 128, 576])))
        kinds.add(f[12:14] if len(f) >= 14 else b"short")
    assert {b"\x08\x00", b"\x86\xdd", b"\x81\x00", b"\x88\xa8", b"short"} <= kinds
