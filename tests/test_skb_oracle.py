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
    out = run_oracle_skb(kat_skb.scenario(c), inp["buf"], inp["off"], inp["lens"], inp["cpu"], ifindex=inp["ifindex"],
                         custom=inp["custom"])
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


def test_context_json_sock_and_flow_keys():
    """UnmarshalContextJSON (context_sk_buff.go:8-17, :20-29) keeps a user-given "sock" and
    "flowKeys": SK.UnmarshalJSON's address rules (net.ParseIP's 16 bytes, else make(net.IP, 4 / 16);
    emulator_linux_sk_buff.go:721-757), encoding/json's case-insensitive field names, and the
    mimic_skb_custom record the engine and the oracle read."""
    import base64
    import json

    import mimic_amd as M
    from mimic_amd import _lib as L

    pkt = bytes(range(64))
    text = json.dumps({"name": "c1", "type": "sk_buff", "ctx": {
        "packet": base64.b64encode(pkt).decode(), "dev": {"ifIndex": 3},
        "sock": {"family": 10, "SRCIP4": "1.2.3.4", "dstIP6": "2001:db8::7", "dstIP4": "bogus", "srcPort": 9,
                 "rxQueueMapping": -2, "state": 1},
        "flowKeys": {"nhoff": 14, "sport": 80, "flowLabel": 5, "ip": "10.0.0.1"}}})
    ctx = M.UnmarshalContextJSON(text)
    assert isinstance(ctx, M.LinuxContextSKBuff) and ctx.Packet == pkt and ctx.Dev.IFIndex == 3
    sk, fk = ctx.SK, ctx.FlowKeys
    assert sk.Family == 10 and sk.SrcPort == 9 and sk.RXQueueMapping == -2 and sk.State == 1
    src4, dst4, src6, dst6 = sk.ips
    assert src4 == bytes(10) + b"\xff\xff" + bytes([1, 2, 3, 4])        # ParseIP: 16 bytes
    assert dst4 == bytes(4)                                              # unparsable: make(net.IP, 4)
    assert src6 == bytes(16) and dst6 == bytes.fromhex("20010db8000000000000000000000007")
    assert fk.Nhoff == 14 and fk.Sport == 80 and fk.FlowLabel == 5
    r = M.vm.skb_custom_record(ctx)
    assert r.dtype == L.SKB_CUSTOM_DTYPE and r.dtype.itemsize == 136
    assert int(r["flags"]) == L.SKB_CUSTOM_SK | L.SKB_CUSTOM_FLOWKEYS
    assert list(r["sk_ip_len"]) == [16, 4, 16, 16] and int(r["sk_rx_queue_mapping"]) == -2
    assert int(r["fk_nhoff"]) == 14 and int(r["fk_flow_label"]) == 5
    # a context without either: no record flags, no table
    plain = M.UnmarshalContextJSON(json.dumps({"type": "sk_buff", "ctx": {"packet": base64.b64encode(pkt).decode()}}))
    assert plain.SK is None and plain.FlowKeys is None
    assert M.SKBBatch.custom_array([plain, plain]) is None
    # a Go SK literal: nil addresses
    assert int(M.vm.skb_custom_record(M.LinuxContextSKBuff(SK=M.SK(Family=2)))["sk_ip_len"].sum()) == 0
