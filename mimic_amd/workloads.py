"""Benchmark workloads of BASELINE.json: programs (hand-assembled eBPF) and synthetic packets.

Packet mix: seed 20261015 (numpy PCG64); Ethernet -> IPv4 90% / IPv6 5% /
ARP 5%; IPv4 protocol TCP 60% / UDP 35% / ICMP 5%; addresses and ports drawn from a 65 536-flow
pool; headroom 0, tailroom 0, ingress ifindex 1, rx queue 0.

Programs are build-authored (the reference ships no XDP programs; there is no BPF compiler in
this image), and use only instruction slots whose reference semantics are unambiguous (SURVEY
Appendix D): no JMP32-X, no atomics, no END, no division.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from . import asm as A

SEED = 20261015
ETH_P_IP, ETH_P_IPV6, ETH_P_ARP = 0x0800, 0x86DD, 0x0806


@dataclass
class Program:
    name: str
    raw: bytes
    relocs: List[Tuple[int, str]]
    maps: List[dict]          # map specs the program references: name/type/key/value/max_entries


# ---------------------------------------------------------------------------------------------
# programs
# ---------------------------------------------------------------------------------------------

def prog_pass8() -> Program:
    """Config 1: 8-instruction XDP_PASS (r0 = 2 after a few ALU ops)."""
    items = [
        A.mov64_imm(0, 0),
        A.mov64_imm(1, 5),
        A.alu64("add", 1, 3),
        A.alu64("mul", 1, 2),
        A.alu64("xor", 1, 18),   # 16 ^ 18 = 2
        A.alu64("and", 1, 0xFF),
        A.mov64_reg(0, 1),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return Program("xdp_pass8", raw, rel, [])


def prog_classifier(map_name: str = "verdicts", max_entries: int = 4) -> Program:
    """Config 2: ~36-slot parse + hash -> DROP/PASS with a per-CPU verdict counter
    (SURVEY.md Appendix D)."""
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),            # data
        A.ldx(4, 3, 6, 4),            # data_end
        A.mov64_imm(7, A.XDP_PASS),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 34),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(2, 5, 2, 12),           # h_proto (little-endian view of the big-endian field)
        A.jmp("jne", 5, 0x0008, "out"),
        A.ldx(1, 5, 2, 23),           # ip->protocol
        A.ldx(4, 8, 2, 26),           # saddr
        A.ldx(4, 9, 2, 30),           # daddr
        A.alu64("xor", 8, 9, reg=True),
        A.mov64_reg(9, 8),
        A.alu64("rsh", 9, 16),
        A.alu64("xor", 8, 9, reg=True),
        A.alu64("mul", 8, 0x9E3779B1 - (1 << 32)),
        A.alu64("xor", 8, 5, reg=True),
        A.mov64_reg(9, 8),
        A.alu64("rsh", 9, 13),
        A.alu64("xor", 8, 9, reg=True),
        A.alu64("and", 8, 3),
        A.jmp("jne", 8, 0, 1),
        A.mov64_imm(7, A.XDP_DROP),
        "out",
        A.stx(4, 10, -4, 7),          # key = verdict
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -4),
        A.ld_map_fd(1, map_name),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, 3),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
        A.mov64_reg(0, 7),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return Program("xdp_classifier", raw, rel,
                   [dict(name=map_name, type=6, key_size=4, value_size=8, max_entries=max_entries)])


def prog_parse5(map_name: str = "flows", max_entries: int = 256) -> Program:
    """Config 3: L2/L3/L4 parse (Ethernet, optional 802.1Q, IPv4 with IHL, IPv6, TCP/UDP ports)
    + 5-tuple hash -> per-CPU counter [hash & (E-1)] of packets and bytes; XDP_PASS, or XDP_DROP
    for non-IP / truncated frames."""
    assert max_entries & (max_entries - 1) == 0
    items = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),            # r2 = data
        A.ldx(4, 3, 6, 4),            # r3 = data_end
        A.mov64_imm(7, A.XDP_DROP),   # verdict
        A.mov64_imm(8, 0),            # hash accumulator
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 14),
        A.jmp("jgt", 4, 3, "count", reg=True),
        A.ldx(2, 5, 2, 12),           # ethertype (LE view)
        A.mov64_imm(9, 14),           # r9 = L3 offset
        A.jmp("jne", 5, 0x0081, "l3"),  # 802.1Q (0x8100 big-endian)
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 18),
        A.jmp("jgt", 4, 3, "count", reg=True),
        A.ldx(2, 5, 2, 16),
        A.mov64_imm(9, 18),
        "l3",
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 9, reg=True),     # r4 = l3 header
        A.jmp("jeq", 5, 0x0008, "ipv4"),
        A.jmp("jeq", 5, 0xDD86, "ipv6"),
        A.ja("count"),
        "ipv4",
        A.mov64_reg(1, 4),
        A.alu64("add", 1, 20),
        A.jmp("jgt", 1, 3, "count", reg=True),
        A.ldx(1, 5, 4, 0),                  # version/ihl
        A.alu64("and", 5, 0x0F),
        A.alu64("lsh", 5, 2),               # ihl * 4
        A.ldx(1, 1, 4, 9),                  # protocol
        A.mov64_reg(8, 1),
        A.ldx(4, 1, 4, 12),                 # saddr
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("mul", 8, 0x01000193),
        A.ldx(4, 1, 4, 16),                 # daddr
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("mul", 8, 0x01000193),
        A.alu64("add", 4, 5, reg=True),     # r4 = L4 header
        A.ja("l4"),
        "ipv6",
        A.mov64_reg(1, 4),
        A.alu64("add", 1, 40),
        A.jmp("jgt", 1, 3, "count", reg=True),
        A.ldx(1, 8, 4, 6),                  # next header
        A.ldx(8, 1, 4, 8),                  # saddr[0:8]
        A.alu64("xor", 8, 1, reg=True),
        A.ldx(8, 1, 4, 16),
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("mul", 8, 0x01000193),
        A.ldx(8, 1, 4, 24),                 # daddr
        A.alu64("xor", 8, 1, reg=True),
        A.ldx(8, 1, 4, 32),
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("mul", 8, 0x01000193),
        A.alu64("add", 4, 40),
        "l4",
        A.mov64_imm(7, A.XDP_PASS),
        A.mov64_reg(1, 4),
        A.alu64("add", 1, 4),
        A.jmp("jgt", 1, 3, "count", reg=True),
        A.ldx(4, 1, 4, 0),                  # src port | dst port
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("mul", 8, 0x01000193),
        "count",
        A.mov64_reg(1, 8),
        A.alu64("rsh", 1, 17),
        A.alu64("xor", 8, 1, reg=True),
        A.alu64("and", 8, max_entries - 1),
        A.stx(4, 10, -4, 8),                # key = hash bucket
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -4),
        A.ld_map_fd(1, map_name),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "done"),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
        "done",
        A.mov64_reg(0, 7),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return Program("xdp_parse5", raw, rel,
                   [dict(name=map_name, type=6, key_size=4, value_size=8, max_entries=max_entries)])


def _flow_key_items():
    """Parse the 5-tuple into a 16-byte key at r10-16: {saddr, daddr, sport|dport, proto, 0, 0, 0}
    (IPv4; IPv6 addresses folded to 32 bits).  r7 = XDP_DROP; non-IP / truncated -> "out"."""
    return [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, 0),            # r2 = data
        A.ldx(4, 3, 6, 4),            # r3 = data_end
        A.mov64_imm(7, A.XDP_DROP),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 14),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(2, 5, 2, 12),           # ethertype (LE view)
        A.jmp("jeq", 5, 0x0008, "ipv4"),
        A.jmp("jeq", 5, 0xDD86, "ipv6"),
        A.ja("out"),
        "ipv4",
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 38),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(4, 1, 2, 26), A.stx(4, 10, -16, 1),     # saddr
        A.ldx(4, 1, 2, 30), A.stx(4, 10, -12, 1),     # daddr
        A.ldx(4, 1, 2, 34), A.stx(4, 10, -8, 1),      # sport | dport
        A.ldx(1, 1, 2, 23), A.stx(4, 10, -4, 1),      # proto + 3 zero bytes
        A.ja("track"),
        "ipv6",
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 58),
        A.jmp("jgt", 4, 3, "out", reg=True),
        A.ldx(8, 1, 2, 22), A.ldx(8, 4, 2, 30), A.alu64("xor", 1, 4, reg=True),
        A.mov64_reg(4, 1), A.alu64("rsh", 4, 32), A.alu64("xor", 1, 4, reg=True), A.stx(4, 10, -16, 1),
        A.ldx(8, 1, 2, 38), A.ldx(8, 4, 2, 46), A.alu64("xor", 1, 4, reg=True),
        A.mov64_reg(4, 1), A.alu64("rsh", 4, 32), A.alu64("xor", 1, 4, reg=True), A.stx(4, 10, -12, 1),
        A.ldx(4, 1, 2, 54), A.stx(4, 10, -8, 1),
        A.ldx(1, 1, 2, 20), A.stx(4, 10, -4, 1),
        "track",
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -16),
    ]


def prog_flowtrack(map_name: str = "flows", max_entries: int = 131072, map_type: int = 1) -> Program:
    """Config 4: insert the packet's 5-tuple key into a shared hash map if absent (BPF_NOEXIST;
    the reference ignores the flags, Q10).  The value is a function of the key only, so the final
    map contents do not depend on the order of the inserts.  XDP_PASS when the flow is (now)
    tracked, XDP_DROP for non-IP / truncated frames or E2BIG (map full)."""
    items = _flow_key_items() + [
        A.ld_map_fd(1, map_name),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jne", 0, 0, "pass"),
        A.ldx(8, 1, 10, -16),                          # value = mix(key)
        A.ldx(8, 4, 10, -8),
        A.alu64("mul", 1, 0x01000193),
        A.alu64("xor", 1, 4, reg=True),
        A.stx(8, 10, -24, 1),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -16),
        A.mov64_reg(3, 10),
        A.alu64("add", 3, -24),
        A.ld_map_fd(1, map_name),
        A.mov64_imm(4, 1),                             # BPF_NOEXIST
        A.call(A.FN_MAP_UPDATE_ELEM),
        A.jmp("jne", 0, 0, "out"),
        "pass",
        A.mov64_imm(7, A.XDP_PASS),
        "out",
        A.mov64_reg(0, 7),
        A.exit_(),
    ]
    raw, rel = A.assemble(items)
    return Program("xdp_flowtrack", raw, rel,
                   [dict(name=map_name, type=map_type, key_size=16, value_size=8, max_entries=max_entries)])


def prog_flowcount(map_name: str = "flowcnt", max_entries: int = 65536, delete_every: int = 0) -> Program:
    """Per-CPU hash: count packets per 5-tuple key (lookup, then increment in place, or insert 1).
    Each vCPU only touches its own values, so the final per-(key, cpu) counters do not depend on
    the interleaving.  delete_every=d > 0: a packet whose key's first word % d == 0 deletes its
    key again after counting (tombstones, freelist reuse)."""
    items = _flow_key_items() + [
        A.ld_map_fd(1, map_name),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, "insert"),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
        A.ja("counted"),
        "insert",
        A.st(8, 10, -24, 1),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -16),
        A.mov64_reg(3, 10),
        A.alu64("add", 3, -24),
        A.ld_map_fd(1, map_name),
        A.mov64_imm(4, 0),
        A.call(A.FN_MAP_UPDATE_ELEM),
        A.jmp("jne", 0, 0, "out"),
        "counted",
        A.mov64_imm(7, A.XDP_PASS),
    ]
    if delete_every:
        items += [
            A.ldx(4, 1, 10, -16),
            A.alu64("mod", 1, delete_every),
            A.jmp("jne", 1, 0, "out"),
            A.mov64_reg(2, 10),
            A.alu64("add", 2, -16),
            A.ld_map_fd(1, map_name),
            A.call(A.FN_MAP_DELETE_ELEM),
            A.mov64_imm(7, A.XDP_TX),
        ]
    items += ["out", A.mov64_reg(0, 7), A.exit_()]
    raw, rel = A.assemble(items)
    return Program("xdp_flowcount", raw, rel,
                   [dict(name=map_name, type=5, key_size=16, value_size=8, max_entries=max_entries)])


# ---------------------------------------------------------------------------------------------
# packets
# ---------------------------------------------------------------------------------------------

def _flow_pool(rng, n_flows: int = 65536):
    return dict(
        src4=rng.integers(0, 2**32, n_flows, dtype=np.uint64).astype(np.uint32),
        dst4=rng.integers(0, 2**32, n_flows, dtype=np.uint64).astype(np.uint32),
        src6=rng.integers(0, 256, (n_flows, 16), dtype=np.uint8),
        dst6=rng.integers(0, 256, (n_flows, 16), dtype=np.uint8),
        sport=rng.integers(1, 65536, n_flows).astype(np.uint16),
        dport=rng.integers(1, 65536, n_flows).astype(np.uint16),
        # a flow keeps one L4 protocol: TCP 60 % / UDP 35 % / ICMP 5 %
        proto=rng.choice(np.array([6, 17, 1]), n_flows, p=[0.60, 0.35, 0.05]).astype(np.uint8),
    )


def make_packets(n: int, sizes=(64,), weights=(1.0,), seed: int = SEED, align: int = 64, headroom: int = 0,
                 tailroom: int = 0, _rows: bool = True):
    """Synthetic frames -> (buf uint8[total], off uint64[n], lens uint32[n]).  Vectorised over
    packet kinds; every packet memory (headroom + L + tailroom bytes, the frame at +headroom)
    starts at a multiple of `align` bytes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pool = _flow_pool(rng)
    return _build_packets(rng, pool, n, sizes, weights, align, headroom, tailroom, _rows)


def _build_packets(rng, pool, n, sizes, weights, align, headroom, tailroom, _rows=True):
    """make_packets' body after the flow pool: every per-packet draw comes from `rng`."""
    w = np.asarray(weights, dtype=np.float64)
    lens = np.asarray(sizes, dtype=np.int64)[rng.choice(len(sizes), n, p=w / w.sum())]
    slot = (headroom + lens + tailroom + align - 1) // align * align
    off = np.zeros(n, dtype=np.int64)
    if n > 1:
        off[1:] = np.cumsum(slot)[:-1]
    total = int(slot.sum())
    buf = _random_fill(total, rng)   # random payload bytes everywhere first (headers overwritten below)
    kind = rng.choice(3, n, p=[0.90, 0.05, 0.05])           # ipv4 / ipv6 / arp
    flow = rng.integers(0, 65536, n)
    proto = pool["proto"][flow]
    # the header bytes (frame offsets 0..57) of every packet are gathered as one row per packet
    # (windows of the buffer at each packet's 64-byte-aligned slot when the slots allow it, else
    # byte gathers), written column by column per packet kind, and scattered back
    W = -(-(headroom + 58) // 64) * 64
    use_rows = _rows and align % 64 == 0 and n > 0 and int(slot.min()) >= W
    win = np.lib.stride_tricks.as_strided(buf, shape=(total // 64 - W // 64 + 1, W), strides=(64, 1)) \
        if use_rows else None

    def part(lo, hi):
        sl = slice(lo, hi)
        if use_rows:
            rix = off[sl] // 64
            rows = np.ascontiguousarray(win[rix])
            _write_headers(rows, headroom, kind[sl], flow[sl], proto[sl], lens[sl], pool)
            win[rix] = rows
        else:
            bidx = (off[sl] + headroom)[:, None] + np.arange(58)
            rows = buf[bidx]
            _write_headers(rows, 0, kind[sl], flow[sl], proto[sl], lens[sl], pool)
            buf[bidx] = rows

    # packet ranges are disjoint byte ranges of the buffer: written in parallel threads
    step = 1 << 20
    cuts = [(lo, min(n, lo + step)) for lo in range(0, n, step)]
    if len(cuts) <= 1:
        for lo, hi in cuts:
            part(lo, hi)
    else:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(min(8, len(cuts))) as ex:
            list(ex.map(lambda c: part(*c), cuts))
    return buf, off.astype(np.uint64), lens.astype(np.uint32)


def _be(v: np.ndarray, nbytes: int) -> np.ndarray:
    """big-endian bytes of unsigned integers: shape (len(v), nbytes) uint8"""
    v = np.asarray(v, dtype=np.uint64)
    return np.stack([((v >> (8 * (nbytes - 1 - k))) & 0xFF).astype(np.uint8) for k in range(nbytes)], axis=1)


def _write_headers(rows: np.ndarray, b: int, kind, flow, proto, lens, pool) -> None:
    """Ethernet / IPv4 / IPv6 / ARP header fields into rows[i, b + frame offset] (frame bytes
    0..57; MACs and the fields not written stay random)."""
    et = np.where(kind == 0, ETH_P_IP, np.where(kind == 1, ETH_P_IPV6, ETH_P_ARP))
    rows[:, b + 12:b + 14] = _be(et, 2)
    s4 = np.nonzero(kind == 0)[0]
    if len(s4):
        h = rows[s4]
        f4 = flow[s4]
        h[:, b + 14] = 0x45
        h[:, b + 15] = 0
        h[:, b + 16:b + 18] = _be((lens[s4] - 14) & 0xFFFF, 2)
        h[:, b + 20] = 0x40
        h[:, b + 21] = 0
        h[:, b + 22] = 64
        h[:, b + 23] = proto[s4]
        h[:, b + 26:b + 30] = _be(pool["src4"][f4], 4)
        h[:, b + 30:b + 34] = _be(pool["dst4"][f4], 4)
        h[:, b + 34:b + 36] = _be(pool["sport"][f4], 2)
        h[:, b + 36:b + 38] = _be(pool["dport"][f4], 2)
        rows[s4] = h
    s6 = np.nonzero(kind == 1)[0]
    if len(s6):
        h = rows[s6]
        f6 = flow[s6]
        h[:, b + 14] = 0x60
        h[:, b + 20] = proto[s6]
        h[:, b + 21] = 64
        h[:, b + 22:b + 38] = pool["src6"][f6]
        h[:, b + 38:b + 54] = pool["dst6"][f6]
        h[:, b + 18:b + 20] = _be(np.maximum(lens[s6] - 54, 0), 2)   # IPv6 payload length
        ok6 = lens[s6] >= 58
        h[ok6, b + 54:b + 56] = _be(pool["sport"][f6[ok6]], 2)
        h[ok6, b + 56:b + 58] = _be(pool["dport"][f6[ok6]], 2)
        rows[s6] = h
    sa = np.nonzero(kind == 2)[0]
    if len(sa):
        rows[sa, b + 14:b + 18] = np.array([0, 1, 8, 0], np.uint8)


def _random_fill(total: int, rng) -> np.ndarray:
    """`total` random bytes: 64-bit PCG64 draws in parallel chunks, each chunk its own stream
    spawned from one seed taken from `rng` (deterministic for a given rng state)."""
    from concurrent.futures import ThreadPoolExecutor

    buf = np.empty(-(-total // 8) * 8, dtype=np.uint8)
    words = buf.view(np.uint64)
    nw = len(words)
    chunk = 1 << 23
    parts = -(-nw // chunk)
    seqs = np.random.SeedSequence(int(rng.integers(0, 2 ** 63))).spawn(max(parts, 1))

    def fill(k):
        a, b = k * chunk, min(nw, (k + 1) * chunk)
        words[a:b] = np.random.PCG64(seqs[k]).random_raw(b - a)

    if parts <= 1:
        for k in range(parts):
            fill(k)
    else:
        with ThreadPoolExecutor(min(8, parts)) as ex:
            list(ex.map(fill, range(parts)))
    return buf[:total]


IMIX = dict(sizes=(64, 576, 1500), weights=(7, 4, 1))

# ---------------------------------------------------------------------------------------------
# one batch, sharded: packets [lo, hi) of a conceptual batch of any size
# ---------------------------------------------------------------------------------------------
RANGE_BLOCK = 1 << 16


def make_packet_range(lo: int, hi: int, sizes=(64,), weights=(1.0,), seed: int = SEED, align: int = 64,
                      block: int = RANGE_BLOCK):
    """Packets [lo, hi) of ONE conceptual batch, as (buf, off, lens) with offsets from 0.

    Every packet is drawn from one flow pool (seed `seed`), and block k of `block` packets from
    its own stream (SeedSequence((seed, k))): packet i has the same bytes whichever range
    contains it, so ranges [r*n, (r+1)*n) for r = 0..N-1 are the N shards of one N*n batch, and
    their flows -- hence the keys a flow-tracking program inserts -- all come from one 65 536-flow
    pool (the bound that keeps cfg 4's shared table within MaxEntries at any N)."""
    assert 0 <= lo <= hi
    pool = _flow_pool(np.random.Generator(np.random.PCG64(seed)))
    ks = list(range(lo // block, -(-hi // block)))

    def one(k):
        rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence((seed, k))))
        b, o, ln = _build_packets(rng, pool, block, sizes, weights, align, 0, 0)
        a, e = max(lo, k * block) - k * block, min(hi, (k + 1) * block) - k * block
        if a == 0 and e == block:
            return b, o, ln
        start = int(o[a])
        end = int(o[e]) if e < block else len(b)
        return b[start:end], o[a:e] - np.uint64(start), ln[a:e]

    if len(ks) <= 1:
        parts = [one(k) for k in ks]
    else:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(min(8, len(ks))) as ex:
            parts = list(ex.map(one, ks))
    if not parts:
        return np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32)
    sizes_b = [len(p[0]) for p in parts]
    base = np.concatenate([[0], np.cumsum(sizes_b)[:-1]]).astype(np.uint64)
    buf = np.concatenate([p[0] for p in parts])
    off = np.concatenate([p[1] + base[j] for j, p in enumerate(parts)])
    lens = np.concatenate([p[2] for p in parts])
    return buf, off, lens


def flowtrack_shard(n: int, rank: int, world: int, batch: int = 0, seed: int = SEED):
    """cfg 4's input on rank `rank` of `world`: packets [(batch*world + rank)*n, +n) of ONE IMIX
    batch (make_packet_range).  bench.py and the shard tests build every cfg-4 shard here, so the
    union of the ranks' replicas is the key set of one batch drawn from one flow pool: at most
    131 072 keys (65 536 flows x {IPv4, IPv6} key forms) = the map's MaxEntries at any N."""
    lo = (batch * world + rank) * n
    return make_packet_range(lo, lo + n, IMIX["sizes"], IMIX["weights"], seed)


def flowtrack_value(keys: np.ndarray) -> np.ndarray:
    """prog_flowtrack's value for each key row (flow_keys_np): u64(key[0:8]) * 0x01000193 ^
    u64(key[8:16]), computed in the program's 64-bit register arithmetic."""
    k = np.ascontiguousarray(keys, np.uint32).view(np.uint64).reshape(-1, 2)
    with np.errstate(over="ignore"):
        return (k[:, 0] * np.uint64(0x01000193)) ^ k[:, 1]


def flow_keys_np(buf, off, lens, with_index: bool = False):
    """The 16-byte keys prog_flowtrack / prog_flowcount build (_flow_key_items), one row per
    packet that reaches the map call (IPv4 frames >= 38 bytes, IPv6 frames >= 58 bytes), as a
    structured view for np.unique.  Host-side workload arithmetic (no engine, no oracle): it
    bounds how many keys a cfg-4 batch inserts.  The key words are little-endian loads of the
    frame bytes, stored as they were loaded, so a key's bytes are the frame's bytes.
    with_index: (keys, the packet index of each row)."""
    off = np.asarray(off, np.int64)
    L = np.asarray(lens, np.int64)
    ok = L >= 14
    et = np.zeros(len(L), np.int64)
    idx = off[ok][:, None] + np.array([12, 13])
    et[ok] = (buf[idx[:, 0]].astype(np.int64) << 8) | buf[idx[:, 1]]
    v4 = np.nonzero((et == 0x0800) & (L >= 38))[0]
    v6 = np.nonzero((et == 0x86DD) & (L >= 58))[0]

    def u32le(rows, at):   # a 4-byte little-endian load at frame offset `at`
        b = buf[off[rows][:, None] + at + np.arange(4)].astype(np.uint32)
        return b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16) | (b[:, 3] << 24)

    def u64le(rows, at):
        b = buf[off[rows][:, None] + at + np.arange(8)].astype(np.uint64)
        return sum(b[:, q] << np.uint64(8 * q) for q in range(8))

    k = np.zeros((len(v4) + len(v6), 4), np.uint32)
    k[:len(v4), 0] = u32le(v4, 26)
    k[:len(v4), 1] = u32le(v4, 30)
    k[:len(v4), 2] = u32le(v4, 34)
    k[:len(v4), 3] = buf[off[v4] + 23]

    def fold(rows, a, b):
        x = u64le(rows, a) ^ u64le(rows, b)
        return ((x ^ (x >> np.uint64(32))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    k[len(v4):, 0] = fold(v6, 22, 30)
    k[len(v4):, 1] = fold(v6, 38, 46)
    k[len(v4):, 2] = u32le(v6, 54)
    k[len(v4):, 3] = buf[off[v6] + 20]
    if with_index:
        return k, np.concatenate([v4, v6])
    return k


def distinct_keys(*key_arrays) -> int:
    """Number of distinct 16-byte keys over flow_keys_np() outputs."""
    ks = [np.ascontiguousarray(k) for k in key_arrays if len(k)]
    if not ks:
        return 0
    allk = np.concatenate(ks).view(np.dtype((np.void, 16)))
    return len(np.unique(allk))


def schedule_cpu(n: int, vcpus: int, mode: str = "chunked") -> np.ndarray:
    """vCPU of each packet: contiguous chunks of ceil(n/V) or i % V."""
    i = np.arange(n, dtype=np.int64)
    if mode == "chunked":
        chunk = -(-n // vcpus)
        return (i // chunk).astype(np.int32)
    return (i % vcpus).astype(np.int32)


# ---------------------------------------------------------------------------------------------
# sk_buff workloads (config 5: context_sk_buff.go path)
# ---------------------------------------------------------------------------------------------
SKB_HEADROOM, SKB_TAILROOM = 32, 64


def make_skb_packets(n: int, sizes=(64,), weights=(1.0,), seed: int = SEED, align: int = 64, variety: float = 0.0):
    """sk_buff batch input: packet memory i = 32 + L + 64 bytes at off[i], the frame at +32.
    variety > 0 replaces that fraction of the frames with header variants (VLAN / QinQ, IPv4
    options and fragments, bad lengths, 802.3 + LLC/SNAP, IPv6 extension headers, UDP tunnels
    and IPIP that give the reference's "multiple layers" Load error, truncated frames)."""
    buf, off, lens = make_packets(n, sizes, weights, seed, align, SKB_HEADROOM, SKB_TAILROOM)
    if variety > 0:
        rng = np.random.Generator(np.random.PCG64(seed ^ 0x5B5B))
        pick = np.nonzero(rng.random(n) < variety)[0]
        for i in pick:
            L = int(lens[i])
            o = int(off[i]) + SKB_HEADROOM
            f = skb_variant(rng, L)               # truncated variants are shorter than L
            buf[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
            lens[i] = len(f)
    return buf, off, lens


def _ipv4(rng, proto, payload_len, ihl=5, frag=0, tl=None, opts=b""):
    total = 4 * ihl + payload_len if tl is None else tl
    h = bytes([0x40 | ihl, 0]) + int(total & 0xFFFF).to_bytes(2, "big") + b"\x12\x34" + int(frag).to_bytes(2, "big")
    h += bytes([64, proto, 0, 0]) + bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    opts = (opts + b"\x00" * 40)[:4 * ihl - 20]
    return h + opts


def _ipv6(rng, nh, plen):
    return (bytes([0x60, 0, 0, 0]) + int(plen & 0xFFFF).to_bytes(2, "big") + bytes([nh, 64]) +
            bytes(rng.integers(0, 256, 32, dtype=np.uint8)))


def _l4(rng, proto, sport=None, dport=None, ulen=None):
    sp = int(rng.integers(1, 65536)) if sport is None else sport
    dp = int(rng.integers(1, 65536)) if dport is None else dport
    if proto == 6:
        return sp.to_bytes(2, "big") + dp.to_bytes(2, "big") + bytes(rng.integers(0, 256, 8, dtype=np.uint8)) + \
            b"\x50\x10" + bytes(6)
    return sp.to_bytes(2, "big") + dp.to_bytes(2, "big") + int(ulen or 0).to_bytes(2, "big") + b"\x00\x00"


def skb_variant(rng, L: int) -> bytes:
    """One frame of length L (truncated variants: at most L) whose headers exercise a corner of
    SKBuffFromBytes' walk."""
    mac = bytes(rng.integers(0, 256, 12, dtype=np.uint8))
    k = int(rng.integers(0, 16))
    proto = int(rng.choice([6, 17, 1]))
    if k == 0:    # 802.1Q VLAN + IPv4
        f = mac + b"\x81\x00" + int(rng.integers(0, 65536)).to_bytes(2, "big") + b"\x08\x00" + \
            _ipv4(rng, proto, max(L - 38, 0)) + _l4(rng, proto, ulen=max(L - 38, 0))
    elif k == 1:  # QinQ (802.1ad + 802.1Q) + IPv6
        f = mac + b"\x88\xa8\x00\x05\x81\x00\x00\x07\x86\xdd" + _ipv6(rng, proto, max(L - 62, 0)) + _l4(rng, proto)
    elif k == 2:  # IPv4 with options (NOP, record-route-ish, bad option)
        ihl = int(rng.integers(6, 16))
        opts = bytes(rng.choice([b"\x01\x01\x01\x01", b"\x07\x07\x04\x00\x00\x00\x00\x00", b"\x44\x01",
                                 b"\x00\x00\x00\x00"]))
        f = mac + b"\x08\x00" + _ipv4(rng, proto, max(L - 14 - 4 * ihl, 0), ihl=ihl, opts=opts) + _l4(rng, proto)
    elif k == 3:  # fragments
        f = mac + b"\x08\x00" + _ipv4(rng, proto, max(L - 34, 0), frag=int(rng.choice([0x2000, 0x0010, 0x4000]))) + \
            _l4(rng, proto)
    elif k == 4:  # total length 0 / < 20 / larger than the frame
        f = mac + b"\x08\x00" + _ipv4(rng, proto, 0, tl=int(rng.choice([0, 12, 19, 20, 4000]))) + _l4(rng, proto)
    elif k == 5:  # VXLAN: a second Ethernet layer -> Load error
        inner = mac + b"\x08\x00" + _ipv4(rng, 17, 8) + _l4(rng, 17)
        f = mac + b"\x08\x00" + _ipv4(rng, 17, 16 + len(inner)) + _l4(rng, 17, dport=4789, ulen=16 + len(inner)) + \
            b"\x08\x00\x00\x00\x00\x00\x01\x00" + inner
    elif k == 6:  # Geneve carrying IPv4: a second network layer -> Load error
        f = mac + b"\x08\x00" + _ipv4(rng, 17, 44) + _l4(rng, 17, dport=6081, ulen=44) + \
            b"\x00\x00\x08\x00\x00\x00\x10\x00" + _ipv4(rng, 6, 20) + _l4(rng, 6)
    elif k == 7:  # GTP-U from a non-tunnel source port towards 2152
        f = mac + b"\x08\x00" + _ipv4(rng, 17, 56) + _l4(rng, 17, dport=2152, ulen=56) + b"\x30\xff\x00\x28" + \
            bytes(4) + _ipv4(rng, 6, 20) + _l4(rng, 6)
    elif k == 8:  # IPIP -> Load error
        f = mac + b"\x08\x00" + _ipv4(rng, 4, 40) + _ipv4(rng, 6, 20) + _l4(rng, 6)
    elif k == 9:  # 802.3 length + LLC/SNAP + IPv4
        f = mac + int(max(min(L - 14, 1500), 0)).to_bytes(2, "big") + b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + \
            _ipv4(rng, proto, max(L - 42, 0)) + _l4(rng, proto)
    elif k == 10:  # IPv6 + routing header + UDP
        f = mac + b"\x86\xdd" + _ipv6(rng, 43, max(L - 54, 0)) + b"\x11\x00\x00\x00\x00\x00\x00\x00" + \
            _l4(rng, 17, ulen=max(L - 62, 0))
    elif k == 11:  # IPv6 fragment / hop-by-hop
        f = mac + b"\x86\xdd" + _ipv6(rng, int(rng.choice([0, 44, 60])), max(L - 54, 0)) + bytes(8) + _l4(rng, 6)
    elif k == 12:  # truncated frames: short Ethernet, short IPv4 / IPv6 headers
        f = (mac + b"\x08\x00" + _ipv4(rng, proto, 20) + _l4(rng, proto))[:int(rng.integers(0, 40))]
        if rng.random() < 0.5:
            f = (mac + b"\x86\xdd" + _ipv6(rng, 6, 20))[:int(rng.integers(14, 54))]
        return f[:L]
    elif k == 13:  # UDP length field variants (0, < 8, larger than the frame)
        f = mac + b"\x08\x00" + _ipv4(rng, 17, max(L - 34, 0)) + _l4(rng, 17, dport=53, ulen=int(rng.choice([0, 5, 8, 9000])))
    elif k == 14:  # ARP / unknown ethertypes
        f = mac + bytes(rng.choice([b"\x08\x06", b"\x88\xcc", b"\x65\x58"])) + bytes(rng.integers(0, 256, 46, dtype=np.uint8))
    else:          # random bytes after a valid IPv4 header
        f = mac + b"\x08\x00" + bytes(rng.integers(0, 256, 40, dtype=np.uint8))
    f = f[:L] + bytes(rng.integers(0, 256, max(L - len(f), 0), dtype=np.uint8))
    return f


def _count(idx: int, stats: str):
    """stats[idx] += 1 through the lookup helper (per-CPU array): 10 slots, r1-r5 / r0 clobbered."""
    return [
        A.st(4, 10, -20, idx),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -20),
        A.ld_map_fd(1, stats),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, 3),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
    ]


def _tail(idx: int, progs: str):
    return [A.mov64_reg(1, 6), A.ld_map_fd(2, progs), A.mov64_imm(3, idx), A.call(A.FN_TAIL_CALL)]


def skb_programs(progs: str = "progs", flows: str = "flows", stats: str = "stats", flow_entries: int = 65536):
    """Config 5: a ~230-slot tc-style classifier over the sk_buff context as a chain of five
    programs joined by tail calls (prog array), with hash-map flow lookups and per-CPU counters.

      skb_entry   __sk_buff field loads / stores, protocol dispatch -> tail call 1 / 2 / 3
      skb_ipv4    LD_ABS / LD_IND header parse -> 5-tuple key, flow lookup -> tail call 4
      skb_ipv6    LD_ABS DW address fold -> key, flow lookup -> tail call 4
      skb_other   counter, verdict
      skb_verdict direct packet access (BigEndian memory), tc_classid / priority / flow_keys,
                  verdict from the fields earlier programs wrote

    Packets of one wavefront take different chains (branch-divergence stress).  Returns
    (list of Program, map specs, prog-array entries [(map, key, program index)])."""
    S = A.SKB
    entry = [
        A.mov64_reg(6, 1),
        A.ldx(4, 7, 6, S["len"]),
        A.ldx(4, 8, 6, S["protocol"]),
        A.ldx(4, 9, 6, S["vlan_present"]),
        A.stx(4, 6, S["mark"], 7),                 # mark = len
        A.ldx(4, 2, 6, S["ifindex"]),
        A.alu64("add", 9, 2, reg=True),
        A.stx(2, 6, S["queue_mapping"], 9),
        A.ldx(4, 2, 6, S["family"]),
        A.ldx(4, 3, 6, S["remote_port"]),
        A.alu64("lsh", 2, 16),
        A.alu64("or", 2, 3, reg=True),
        A.stx(4, 6, S["tc_index"], 2),
        A.ldx(8, 2, 6, S["tstamp"]),
        A.alu64("add", 2, 7, reg=True),
        A.stx(8, 6, S["tstamp"], 2),
        *_count(0, stats),
        A.mov64_imm(3, 3),
        A.jmp("jne", 8, 0x0800, "not4"),
        A.mov64_imm(3, 1),
        A.ja("go"),
        "not4",
        A.jmp("jne", 8, 0x86DD, "go"),
        A.mov64_imm(3, 2),
        "go",
        A.mov64_reg(1, 6),
        A.ld_map_fd(2, progs),
        A.call(A.FN_TAIL_CALL),
        A.mov64_imm(0, A.TC_ACT_OK),               # the tail call failed
        A.exit_(),
    ]
    ipv4 = [
        A.mov64_reg(6, 1),
        A.ld_abs(1, 14),                           # version / IHL
        A.mov64_reg(7, 0),
        A.alu64("and", 7, 0x0F),
        A.alu64("lsh", 7, 2),                      # r7 = IHL * 4
        A.jmp("jlt", 7, 20, "bad"),
        A.ld_abs(1, 23),                           # protocol
        A.stx(4, 10, -4, 0),
        A.ld_abs(4, 26),                           # saddr (host order)
        A.stx(4, 10, -16, 0),
        A.ld_abs(4, 30),                           # daddr
        A.stx(4, 10, -12, 0),
        A.ld_ind(2, 7, 14),                        # sport
        A.mov64_reg(8, 0),
        A.alu64("lsh", 8, 16),
        A.ld_ind(2, 7, 16),                        # dport
        A.alu64("or", 8, 0, reg=True),
        A.stx(4, 10, -8, 8),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -16),
        A.ld_map_fd(1, flows),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.mov64_imm(9, 1),                         # stats index: miss
        A.mov64_imm(8, 0),
        A.jmp("jeq", 0, 0, "miss"),
        A.ldx(8, 8, 0, 0),                         # flow value
        A.mov64_imm(9, 2),                         # hit
        "miss",
        A.stx(4, 10, -20, 9),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -20),
        A.ld_map_fd(1, stats),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.jmp("jeq", 0, 0, 3),
        A.ldx(8, 1, 0, 0),
        A.alu64("add", 1, 1),
        A.stx(8, 0, 0, 1),
        A.mov64_reg(1, 8),
        A.alu64("and", 1, 7),
        A.stx(4, 6, S["priority"], 1),             # priority = flow value & 7
        A.ldx(4, 2, 6, S["local_ip4"]),            # SK's view of the addresses
        A.ldx(4, 3, 6, S["remote_ip4"]),
        A.alu64("xor", 2, 3, reg=True),
        A.ldx(4, 3, 6, S["mark"]),
        A.alu64("xor", 3, 2, reg=True),
        A.stx(4, 6, S["mark"], 3),
        *_tail(4, progs),
        "bad",
        A.mov64_imm(0, A.TC_ACT_SHOT),
        A.exit_(),
    ]
    ipv6 = [
        A.mov64_reg(6, 1),
        A.ld_abs(8, 22),                           # saddr[0:8]
        A.mov64_reg(7, 0),
        A.ld_abs(8, 30),                           # saddr[8:16]
        A.alu64("xor", 7, 0, reg=True),
        A.mov64_reg(8, 7),
        A.alu64("rsh", 8, 32),
        A.alu64("xor", 7, 8, reg=True),
        A.stx(4, 10, -16, 7),
        A.ld_abs(8, 38),                           # daddr
        A.mov64_reg(7, 0),
        A.ld_abs(8, 46),
        A.alu64("xor", 7, 0, reg=True),
        A.mov64_reg(8, 7),
        A.alu64("rsh", 8, 32),
        A.alu64("xor", 7, 8, reg=True),
        A.stx(4, 10, -12, 7),
        A.ld_abs(4, 54),                           # sport | dport
        A.stx(4, 10, -8, 0),
        A.ld_abs(1, 20),                           # next header
        A.stx(4, 10, -4, 0),
        A.mov64_reg(2, 10),
        A.alu64("add", 2, -16),
        A.ld_map_fd(1, flows),
        A.call(A.FN_MAP_LOOKUP_ELEM),
        A.mov64_imm(8, 0),
        A.jmp("jeq", 0, 0, 1),
        A.ldx(8, 8, 0, 0),
        *_count(3, stats),
        A.stx(4, 6, S["priority"], 8),
        *_tail(4, progs),
        A.mov64_imm(0, A.TC_ACT_SHOT),
        A.exit_(),
    ]
    other = [
        A.mov64_reg(6, 1),
        *_count(4, stats),
        A.ldx(4, 0, 6, S["vlan_tci"]),
        A.alu64("and", 0, 1),
        A.exit_(),
    ]
    verdict = [
        A.mov64_reg(6, 1),
        A.ldx(4, 2, 6, S["data"]),
        A.ldx(4, 3, 6, S["data_end"]),
        A.mov64_reg(4, 2),
        A.alu64("add", 4, 14),
        A.mov64_imm(9, 0),
        A.jmp("jgt", 4, 3, "nodata", reg=True),
        A.ldx(2, 9, 2, 12),                        # ethertype, BigEndian packet memory
        A.ldx(1, 4, 2, 0),
        A.alu64("xor", 4, 0xFF),
        A.stx(1, 2, 0, 4),                         # rewrite the first destination-MAC byte
        "nodata",
        A.stx(2, 6, S["tc_classid"], 9),
        A.ldx(4, 7, 6, S["mark"]),
        A.ldx(4, 8, 6, S["priority"]),
        A.ldx(4, 3, 6, S["local_port"]),
        A.ldx(4, 1, 6, S["flow_keys"]),
        A.stx(2, 1, A.FLOW_KEYS["sport"], 3),
        A.ldx(2, 3, 1, A.FLOW_KEYS["sport"]),
        A.alu64("xor", 7, 8, reg=True),
        A.alu64("xor", 7, 3, reg=True),
        A.ldx(4, 3, 6, S["queue_mapping"]),
        A.alu64("add", 7, 3, reg=True),
        *_count(5, stats),
        A.mov64_imm(0, A.TC_ACT_OK),
        A.jmp("jset", 7, 1, 1),                    # Q3: taken when (r7 & 1) == 0
        A.mov64_imm(0, A.TC_ACT_SHOT),
        A.exit_(),
    ]
    out = []
    for name, items in (("skb_entry", entry), ("skb_ipv4", ipv4), ("skb_ipv6", ipv6), ("skb_other", other),
                        ("skb_verdict", verdict)):
        raw, rel = A.assemble(items)
        out.append(Program(name, raw, rel, []))
    maps = [dict(name=progs, type=3, key_size=4, value_size=4, max_entries=8),
            dict(name=flows, type=1, key_size=16, value_size=8, max_entries=flow_entries),
            dict(name=stats, type=6, key_size=4, value_size=8, max_entries=8)]
    prog_array = [(progs, k, k) for k in (1, 2, 3, 4)]
    return out, maps, prog_array


def skb_flow_keys(buf, off, lens, every: int = 3, limit: int = 4096):
    """Keys the cfg-5 programs build for some of the batch's IPv4 / IPv6 frames (plain Ethernet):
    the hash map is pre-populated with every `every`-th distinct key, up to `limit`, value =
    a function of the key.  Returns [(key bytes, value bytes)]."""
    import struct

    keys = {}
    for i in range(len(lens)):
        L = int(lens[i])
        o = int(off[i]) + SKB_HEADROOM
        f = bytes(buf[o:o + L])
        if L < 14:
            continue
        et = int.from_bytes(f[12:14], "big")
        if et == 0x0800 and L >= 38:
            ihl = (f[14] & 0x0F) * 4
            if ihl < 20 or 14 + ihl + 4 > L + SKB_TAILROOM or 14 + ihl + 4 > L:
                continue
            k = struct.pack("<IIII", int.from_bytes(f[26:30], "big"), int.from_bytes(f[30:34], "big"),
                            (int.from_bytes(f[14 + ihl:16 + ihl], "big") << 16) | int.from_bytes(f[16 + ihl:18 + ihl], "big"),
                            f[23])
        elif et == 0x86DD and L >= 58:
            def fold(a, b):
                x = int.from_bytes(f[a:a + 8], "big") ^ int.from_bytes(f[b:b + 8], "big")
                return (x ^ (x >> 32)) & 0xFFFFFFFF
            k = struct.pack("<IIII", fold(22, 30), fold(38, 46), int.from_bytes(f[54:58], "big"), f[20])
        else:
            continue
        keys.setdefault(k, None)
    sel = list(keys)[::every][:limit]
    return [(k, (int.from_bytes(k[:8], "little") * 0x9E3779B1 & (2**64 - 1)).to_bytes(8, "little")) for k in sel]


# ---------------------------------------------------------------------------------------------
# the bytes each workload's programs can read (bench.py's algorithmic-byte model)
# ---------------------------------------------------------------------------------------------
SECTOR = 32   # HBM read granularity: the smallest read request (TCC_EA0_RDREQ_32B, MI355X_MICROARCH.md)


def _header_rows(buf, off, base: int, width: int, lo: int, hi: int) -> np.ndarray:
    idx = off[lo:hi].astype(np.int64)[:, None] + base + np.arange(width, dtype=np.int64)[None, :]
    np.minimum(idx, len(buf) - 1, out=idx)
    return buf[idx]


def _be16(rows, at):
    return (rows[:, at].astype(np.int64) << 8) | rows[:, at + 1]


def packet_reach(kind: str, buf, off, lens, chunk: int = 1 << 20) -> np.ndarray:
    """Per packet: one past the furthest frame byte the workload's programs read, with every bounds
    check they make (0 = no packet byte).  Restates the programs above:

      classifier  L < 34: none; else ethertype [12,14) and, for IPv4, protocol / addresses to 34
      parse5      ethertype, an 802.1Q tag, IPv4 [l3, l3+20) and the ports at l3 + 4*IHL, or IPv6
                  [l3, l3+40) and its ports; each only when its bounds check passes
      flowtrack   ethertype; IPv4 to 38, IPv6 to 58 when the frame is that long
      skb         the header stack SKBuffFromBytes decodes (emulator_linux_sk_buff.go:108-265:
                  Ethernet, IPv4 IHL / IPv6, TCP data offset, UDP / ICMP 8), which covers the
                  chain's LD_ABS / LD_IND reads; other frames (the 5 % variants) min(L, 96)
      pass8       none (reads xdp_md fields only)
    """
    lens = np.asarray(lens)
    n = len(lens)
    out = np.zeros(n, np.int64)
    if kind == "pass8" or n == 0:
        return out
    base = SKB_HEADROOM if kind == "skb" else 0
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        L = lens[lo:hi].astype(np.int64)
        r = _header_rows(buf, off, base, 96, lo, hi)
        et = _be16(r, 12)
        if kind == "classifier":
            reach = np.where(L < 34, 0, np.where(et == 0x0800, 34, 14))
        elif kind == "flowtrack":
            reach = np.where(L < 14, 0, 14)
            reach = np.where((et == 0x0800) & (L >= 38), 38, reach)
            reach = np.where((et == 0x86DD) & (L >= 58), 58, reach)
        elif kind == "parse5":
            reach = np.where(L < 14, 0, 14)
            vlan = (et == 0x8100) & (L >= 18)
            reach = np.where(vlan, 18, reach)
            l3 = np.where(vlan, 18, 14)
            et2 = np.where(vlan, _be16(r, 16), et)
            rows = np.arange(len(L))
            ihl = (r[rows, np.minimum(l3, 95)] & 15).astype(np.int64)
            v4 = (et2 == 0x0800) & (l3 + 20 <= L)
            l4 = l3 + 4 * ihl
            reach = np.where(v4, np.where(l4 + 4 <= L, np.maximum(l3 + 20, l4 + 4), l3 + 20), reach)
            v6 = (et2 == 0x86DD) & (l3 + 40 <= L)
            reach = np.where(v6, np.where(l3 + 44 <= L, l3 + 44, l3 + 40), reach)
        elif kind == "skb":
            rows = np.arange(len(L))
            ihl = (r[:, 14] & 15).astype(np.int64)
            v4 = (et == 0x0800) & ((r[:, 14] >> 4) == 4)
            v6 = (et == 0x86DD)
            l4 = np.where(v4, 14 + 4 * ihl, 54)
            proto = np.where(v4, r[:, 23], r[:, 20]).astype(np.int64)
            doff = (r[rows, np.minimum(l4 + 12, 95)] >> 4).astype(np.int64) * 4
            # TCP: its data offset; UDP, ICMP, ICMPv6: 8; else the ports the chain's LD_IND reads
            l4len = np.where(proto == 6, np.maximum(doff, 20), np.where(np.isin(proto, (17, 1, 58)), 8, 4))
            common = (v4 | v6) & (l4 + l4len <= L) & (l4 + l4len <= 96)
            reach = np.where(common, l4 + l4len, np.minimum(L, 96))
        else:
            raise ValueError(kind)
        out[lo:hi] = np.minimum(reach, L)
    return out


def read_sector_bytes(reach: np.ndarray) -> np.ndarray:
    """Bytes of the 32-byte sectors holding frame bytes [0, reach) (frames start sector-aligned)."""
    return -(-np.asarray(reach, np.int64) // SECTOR) * SECTOR
