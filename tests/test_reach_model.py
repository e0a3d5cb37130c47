"""The per-packet read reach bench.py charges as algorithmic bytes (workloads.packet_reach) is sound:
the CPU oracle (the reference restated) gives the same results for every packet -- R0, status,
steps, final map bytes -- after every frame byte at or past the packet's reach is replaced by
random bytes.  So the programs never read past it, and charging the sectors below it is not an
undercount.  Packets are also cut short at random (bounds checks) and, for parse5, given an 802.1Q
tag and IPv4 options."""
import numpy as np
import pytest

from harness import Scenario, run_oracle, run_oracle_skb
from mimic_amd import workloads as W


def _scramble_past_reach(buf, off, lens, reach, base, seed):
    rng = np.random.default_rng(seed)
    out = buf.copy()
    for o, L, r in zip(off.astype(np.int64), lens.astype(np.int64), reach):
        a, b = o + base + int(r), o + base + int(L)
        if b > a:
            out[a:b] = rng.integers(0, 256, b - a, dtype=np.uint8)
    return out


def _same(a, b):
    for k in ("r0", "status", "steps", "err_pc"):
        assert np.array_equal(a[k], b[k]), k
    assert a["maps"].keys() == b["maps"].keys()
    for name in a["maps"]:
        for x, y in zip(a["maps"][name], b["maps"][name]):
            assert bytes(x) == bytes(y), name
    assert a.get("hash") == b.get("hash")


def _xdp_packets(kind, n, seed):
    sizes = dict(sizes=(64,), weights=(1,)) if kind == "classifier" else W.IMIX
    buf, off, lens = W.make_packets(n, **sizes, seed=seed)
    rng = np.random.default_rng(seed + 1)
    lens = lens.copy()
    cut = rng.random(n) < 0.2      # truncated frames exercise every bounds check
    lens[cut] = rng.integers(0, 80, int(cut.sum())).astype(lens.dtype)
    lens = np.minimum(lens, W.make_packets(n, **sizes, seed=seed)[2])
    if kind == "parse5":
        # an 802.1Q tag in front of the IP header, and IPv4 options (IHL 6..15), in some frames
        for i in np.nonzero(rng.random(n) < 0.15)[0]:
            o, L = int(off[i]), int(lens[i])
            if L < 64:
                continue
            if rng.random() < 0.5:
                hdr = buf[o + 12:o + 60].copy()
                buf[o + 12:o + 16] = (0x81, 0x00, 0x00, 0x07)
                buf[o + 16:o + 64] = hdr
            elif buf[o + 12] == 0x08 and buf[o + 13] == 0x00:
                buf[o + 14] = 0x40 | int(rng.integers(6, 16))
    return buf, off, lens


@pytest.mark.parametrize("kind", ["classifier", "parse5", "flowtrack"])
def test_xdp_programs_read_nothing_past_the_reach(kind):
    prog = {"classifier": W.prog_classifier, "parse5": W.prog_parse5,
            "flowtrack": lambda: W.prog_flowtrack(max_entries=4096)}[kind]()
    sc = Scenario(vcpus=16, maps=prog.maps, progs=[(prog.name, prog.raw, prog.relocs)])
    buf, off, lens = _xdp_packets(kind, 3000, 11)
    reach = W.packet_reach(kind, buf, off, lens)
    assert (reach <= lens).all() and (reach >= 0).all()
    assert (reach < lens).mean() > 0.1 if kind != "classifier" else True
    cpu = W.schedule_cpu(len(lens), 16, "chunked")
    want = run_oracle(sc, buf, off, lens, cpu)
    got = run_oracle(sc, _scramble_past_reach(buf, off, lens, reach, 0, 5), off, lens, cpu)
    _same(want, got)
    # and the bytes just below the reach do matter somewhere (the model is not just L)
    if kind != "classifier":
        rng = np.random.default_rng(3)
        b2 = buf.copy()
        for o, r in zip(off.astype(np.int64), reach):
            if r:
                b2[o + r - 1] ^= np.uint8(rng.integers(1, 256))
        other = run_oracle(sc, b2, off, lens, cpu)
        assert not np.array_equal(other["r0"], want["r0"]) or other["maps"] != want["maps"]


def test_skb_chain_reads_nothing_past_the_reach():
    buf, off, lens = W.make_skb_packets(2000, **W.IMIX, variety=0.0, seed=21)
    progs, maps, pa = W.skb_programs()
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(buf, off, lens)]
    sc = Scenario(vcpus=16, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa,
                  map_init=init)
    reach = W.packet_reach("skb", buf, off, lens)
    assert (reach <= lens).all() and (reach < lens).mean() > 0.3
    cpu = W.schedule_cpu(len(lens), 16, "chunked")
    want = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=2)
    got = run_oracle_skb(sc, _scramble_past_reach(buf, off, lens, reach, W.SKB_HEADROOM, 9), off, lens, cpu, ifindex=2)
    for k in ("r0", "status", "steps", "err_pc"):
        assert np.array_equal(want[k], got[k]), k
    assert want["maps"] == got["maps"]


def test_sector_bytes():
    assert W.read_sector_bytes(np.array([0, 1, 32, 33, 64, 65])).tolist() == [0, 32, 32, 64, 64, 96]
