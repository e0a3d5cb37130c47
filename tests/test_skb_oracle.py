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


def test_oracle_memory_indexes_match_literal_scans(monkeypatch):
    """The oracle's first-fit gap index and object index (oracle/mimic_oracle.c mc_add /
    mc_del_obj) give exactly the addresses of the literal MemoryController loops
    (memory_controller.go:58-112, 202-232): sk_buff batches (leaked entries, freed stack and
    context holes of many sizes) returning skb->data, and the cfg-5 chain, both ways."""
    from harness import Scenario
    from mimic_amd import asm as A
    from mimic_amd import workloads as W

    S = A.SKB
    raw, rel = A.assemble([A.ldx(4, 0, 1, S["data"]), A.ldx(4, 2, 1, S["data_end"]), A.alu64("lsh", 2, 32),
                           A.alu64("or", 0, 2, reg=True), A.exit_()])
    rng = np.random.default_rng(9)
    pk = [bytes(rng.integers(0, 256, int(rng.choice([0, 1, 14, 60, 64, 200, 576, 1500])), dtype=np.uint8))
          for _ in range(1500)]
    from harness import skb_packets_to_buffer
    buf, off, lens = skb_packets_to_buffer(pk)
    cpu = rng.integers(0, 4, len(pk)).astype(np.int32)
    progs, maps, pa = W.skb_programs()
    cases = [(Scenario(vcpus=4, progs=[("addr", raw, rel)]), None),
             (Scenario(vcpus=4, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa),
              [500, 501, 1200])]
    for sc, splits in cases:
        monkeypatch.setenv("MIMIC_ORACLE_LITERAL_MC", "1")
        lit = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=1, splits=splits)
        monkeypatch.setenv("MIMIC_ORACLE_LITERAL_MC", "0")
        fast = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=1, splits=splits)
        for k in ("r0", "status", "steps", "err_pc", "pkt"):
            assert np.array_equal(lit[k], fast[k]), k
        assert lit["maps"] == fast["maps"]
        if splits is None:
            assert len(set(lit["r0"].tolist())) > 1000   # addresses drift over the batch (leaks)
