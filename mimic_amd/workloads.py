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


def make_packets(n: int, sizes=(64,), weights=(1.0,), seed: int = SEED, align: int = 64):
    """Synthetic frames -> (buf uint8[total], off uint64[n], lens uint32[n]).  Vectorised over
    packet kinds; every packet memory starts at a multiple of `align` bytes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pool = _flow_pool(rng)
    w = np.asarray(weights, dtype=np.float64)
    lens = np.asarray(sizes, dtype=np.int64)[rng.choice(len(sizes), n, p=w / w.sum())]
    slot = (lens + align - 1) // align * align
    off = np.zeros(n, dtype=np.int64)
    if n > 1:
        off[1:] = np.cumsum(slot)[:-1]
    total = int(slot.sum())
    buf = np.zeros(total, dtype=np.uint8)
    # random payload bytes everywhere first (headers overwritten below)
    buf[:] = rng.integers(0, 256, total, dtype=np.uint8)
    kind = rng.choice(3, n, p=[0.90, 0.05, 0.05])           # ipv4 / ipv6 / arp
    flow = rng.integers(0, 65536, n)
    proto = pool["proto"][flow]
    idx = off.astype(np.int64)

    def put(col, vals):
        vals = np.asarray(vals, dtype=np.uint8)
        buf[idx[:, None] + col] = vals

    # Ethernet: dst, src MACs random (already), ethertype
    et = np.where(kind == 0, ETH_P_IP, np.where(kind == 1, ETH_P_IPV6, ETH_P_ARP)).astype(np.uint16)
    buf[idx + 12] = (et >> 8).astype(np.uint8)
    buf[idx + 13] = (et & 0xFF).astype(np.uint8)
    v4 = idx[kind == 0]
    f4 = flow[kind == 0]
    p4 = proto[kind == 0]
    l4 = lens[kind == 0]
    buf[v4 + 14] = 0x45
    buf[v4 + 15] = 0
    tl = (l4 - 14).astype(np.uint16)
    buf[v4 + 16] = (tl >> 8).astype(np.uint8)
    buf[v4 + 17] = (tl & 0xFF).astype(np.uint8)
    buf[v4 + 20] = 0x40
    buf[v4 + 21] = 0
    buf[v4 + 22] = 64
    buf[v4 + 23] = p4.astype(np.uint8)
    for k in range(4):
        buf[v4 + 26 + k] = ((pool["src4"][f4] >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
        buf[v4 + 30 + k] = ((pool["dst4"][f4] >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
    buf[v4 + 34] = (pool["sport"][f4] >> 8).astype(np.uint8)
    buf[v4 + 35] = (pool["sport"][f4] & 0xFF).astype(np.uint8)
    buf[v4 + 36] = (pool["dport"][f4] >> 8).astype(np.uint8)
    buf[v4 + 37] = (pool["dport"][f4] & 0xFF).astype(np.uint8)
    v6 = idx[kind == 1]
    f6 = flow[kind == 1]
    buf[v6 + 14] = 0x60
    buf[v6 + 20] = proto[kind == 1].astype(np.uint8)
    buf[v6 + 21] = 64
    for k in range(16):
        buf[v6 + 22 + k] = pool["src6"][f6, k]
        buf[v6 + 38 + k] = pool["dst6"][f6, k]
    ok6 = lens[kind == 1] >= 58
    buf[v6[ok6] + 54] = (pool["sport"][f6[ok6]] >> 8).astype(np.uint8)
    buf[v6[ok6] + 55] = (pool["sport"][f6[ok6]] & 0xFF).astype(np.uint8)
    buf[v6[ok6] + 56] = (pool["dport"][f6[ok6]] >> 8).astype(np.uint8)
    buf[v6[ok6] + 57] = (pool["dport"][f6[ok6]] & 0xFF).astype(np.uint8)
    va = idx[kind == 2]
    buf[va + 14] = 0
    buf[va + 15] = 1
    buf[va + 16] = 8
    buf[va + 17] = 0
    return buf, off.astype(np.uint64), lens.astype(np.uint32)


IMIX = dict(sizes=(64, 576, 1500), weights=(7, 4, 1))


def schedule_cpu(n: int, vcpus: int, mode: str = "chunked") -> np.ndarray:
    """vCPU of each packet: contiguous chunks of ceil(n/V) or i % V."""
    i = np.arange(n, dtype=np.int64)
    if mode == "chunked":
        chunk = -(-n // vcpus)
        return (i // chunk).astype(np.int32)
    return (i % vcpus).astype(np.int32)
