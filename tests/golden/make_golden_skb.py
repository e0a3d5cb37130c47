#!/usr/bin/env python3
"""Known-answer vectors for the sk_buff context path -> tests/golden/kat_skb.json.

Config 5 of BASELINE.json runs programs over LinuxContextSKBuff (context_sk_buff.go).  No
reference test builds an sk_buff, and the reference cannot be built or run here (Go is absent).
So, as for kat.json, every expected value below is derived BY HAND from the cited Go lines and
the packet bytes written in this file:
  * SKBuffFromBytes (emulator_linux_sk_buff.go:108-265) over gopacket v1.1.19's layers;
  * SKBuff / SK / FlowKeys convertAccess (:295-676, :772-918, :1031-1175);
  * LD_ABS / LD_IND (emulator_linux_.go:198-288);
  * the MemoryController layout of LinuxContextSKBuff.Load / Cleanup (context_sk_buff.go:42-119,
    memory_controller.go:58-112).
This file is independent of the C oracle and of the engine; tests check both against it.

Address layout used below (one program, no maps): the program object is at 0x10000 (8 bytes),
so the stack entry is St = 0x10009 and the sk_buff entry Sk = St + 2049.  The first sk_buff
process's leaked entries follow: sock Ka = Sk + 193, flow keys Fa = Ka + 81, packet
Pa = Fa + 41 (data = Pa + 32, data_end = Pa + L).  Every later successful Load moves the
leaks up by 219 + L (Cleanup frees only the stack and the sk_buff).

Run:  python tests/golden/make_golden_skb.py   (rewrites kat_skb.json)
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mimic_amd import asm as A  # noqa: E402

M64 = (1 << 64) - 1
OK, UNRES, BOUNDS, LDABS, BADREG = 0, 3, 5, 15, 18
CTX_ACCESS, PANIC_SLICE, CTX_LOAD = 26, 27, 28

St = 0x10009
Sk = St + 2049
Ka0 = Sk + 193


def addrs(L, prior=()):
    """(Ka, Fa, Pa) of a process whose earlier successful Loads had lengths `prior`."""
    ka = Ka0 + sum(219 + p for p in prior)
    return ka, ka + 81, ka + 122


S = A.SKB
K = A.SOCK
FK = A.FLOW_KEYS

# ---- packets -------------------------------------------------------------------------------
MAC = bytes.fromhex("001122334455") + bytes.fromhex("66778899aabb")
IP4 = bytes.fromhex("45000032" "00010000" "4006" "0000" "c0a80102" "0a000001")   # tl 50, TCP
TCP = bytes.fromhex("1234" "0050" "00000001" "00000000" "5010" "2000" "0000" "0000")


def pad(b, L):
    return (b + bytes((0x80 + i) & 0xFF for i in range(L)))[:L]


PKT4 = pad(MAC + b"\x08\x00" + IP4 + TCP, 64)            # IPv4 / TCP, 64 bytes
IP6 = (bytes.fromhex("60000000" "0014" "06" "40") + bytes(range(0x10, 0x20)) + bytes(range(0x20, 0x30)))
PKT6 = pad(MAC + b"\x86\xdd" + IP6 + TCP, 80)             # IPv6 / TCP
PKTV = pad(MAC + b"\x81\x00" + b"\x00\x2a" + b"\x08\x00" + IP4 + TCP, 68)   # 802.1Q tci 42 + IPv4
PKT_SHORT4 = MAC + b"\x08\x00" + IP4[:10]               # IPv4 header cut at 10 bytes
PKT_TINY = bytes(range(1, 11))                          # 10 bytes: no Ethernet layer
VXLAN_INNER = MAC + b"\x08\x00" + bytes.fromhex("4500001400000000401100000102030405060708")
UDP_VX = bytes.fromhex("3039" "12b5") + (8 + 8 + len(VXLAN_INNER)).to_bytes(2, "big") + b"\x00\x00"
IP4_UDP = bytes.fromhex("4500") + (20 + 16 + len(VXLAN_INNER)).to_bytes(2, "big") + bytes.fromhex(
    "00010000" "4011" "0000" "c0a80102" "0a000001")
PKT_VXLAN = MAC + b"\x08\x00" + IP4_UDP + UDP_VX + bytes.fromhex("0800000000000100") + VXLAN_INNER
PKT_LLC = pad(MAC + (58).to_bytes(2, "big") + bytes.fromhex("aaaa03000000" "0800") + IP4 + TCP, 72)

CASES = []


def case(name, ref, items, packets, expect, ifindex=0, contexts=None):
    """contexts: per packet, the user-given part of its context JSON ({"sock": ..., "flowKeys": ...},
    context_sk_buff.go:20-29) or None; "nilIPs": true marks an SK built as a Go literal (its net.IP
    fields never set by SK.UnmarshalJSON: nil)."""
    raw, rel = A.assemble(items)
    assert not rel
    d = dict(name=name, ref=ref, raw=raw.hex(), packets=[p.hex() for p in packets], ifindex=ifindex, expect=expect)
    if contexts is not None:
        assert len(contexts) == len(packets)
        d["contexts"] = contexts
    CASES.append(d)


def e(r0=None, status=OK, steps=None, err_pc=-1):
    d = {"status": status, "err_pc": err_pc}
    if r0 is not None:
        d["r0"] = r0 & M64
    if steps is not None:
        d["steps"] = steps
    return d


def ld_field(off, size=4):
    """r0 = *(size *)(r1 + off); exit  (2 steps)"""
    return [A.ldx(size, 0, 1, off), A.exit_()]


# ---- __sk_buff loads (SKBuff.convertAccess, emulator_linux_sk_buff.go:324-676) ----------------
for size in (1, 2, 4, 8):
    case(f"len_u{8 * size}", "emulator_linux_sk_buff.go:324-331", ld_field(S["len"], size), [PKT4], [e(64, steps=2)])
case("len_u8_trunc", "toSize(uint64(sk.len)) with asm.Byte", ld_field(S["len"], 1), [pad(PKT4, 300)],
     [e(300 & 0xFF, steps=2)])
case("protocol_ipv4", "SKBuffFromBytes :187 skb.protocol = EthernetType", ld_field(S["protocol"]), [PKT4],
     [e(0x0800, steps=2)])
case("protocol_vlan", ":187 (outer type)", ld_field(S["protocol"]), [PKTV], [e(0x8100, steps=2)])
case("vlan_present", ":176-179", ld_field(S["vlan_present"]), [PKTV], [e(1, steps=2)])
case("vlan_absent", ":389-395", ld_field(S["vlan_present"]), [PKT4], [e(0, steps=2)])
case("vlan_tci", ":178 BigEndian.Uint16(Contents[:2])", ld_field(S["vlan_tci"]), [PKTV], [e(0x2a, steps=2)])
case("vlan_proto", ":177 uint16(l.Type)", ld_field(S["vlan_proto"]), [PKTV], [e(0x0800, steps=2)])
case("pkt_type", ":333-343 (never set)", ld_field(S["pkt_type"]), [PKT4], [e(0, steps=2)])
case("ingress_ifindex", "skbIIF never set", ld_field(S["ingress_ifindex"]), [PKT4], [e(0, steps=2)])
case("ifindex", "dev.IFIndex", ld_field(S["ifindex"]), [PKT4], [e(7, steps=2)], ifindex=7)
case("hash", "never set", ld_field(S["hash"]), [PKT4], [e(0, steps=2)])
case("napi_id", "never set", ld_field(S["napi_id"]), [PKT4], [e(0, steps=2)])
case("wire_len", "cb[0:4] (zero)", ld_field(S["wire_len"]), [PKT4], [e(0, steps=2)])
case("data_meta", "cb[36:38] (zero)", ld_field(S["data_meta"]), [PKT4], [e(0, steps=2)])
ka, fa, pa = addrs(64)
case("data", "head/data += pktEntry.Addr (context_sk_buff.go:97-100)", ld_field(S["data"]), [PKT4],
     [e(pa + 32, steps=2)])
case("data_end", "cb[32:36] = end = pkt addr + len (skb_reset_tail_pointer before the reserve)",
     ld_field(S["data_end"]), [PKT4], [e(pa + 64, steps=2)])
case("flow_keys_ptr", "flowKeysAddr", ld_field(S["flow_keys"]), [PKT4], [e(fa, steps=2)])
case("flow_keys_ptr_hi", "offset 148 is the same field", ld_field(S["flow_keys"] + 4), [PKT4], [e(fa, steps=2)])
case("sk_ptr", "skAddr", ld_field(S["sk"]), [PKT4], [e(ka, steps=2)])
case("sk_ptr_dw", "no toSize on sk", ld_field(S["sk"], 8), [PKT4], [e(ka, steps=2)])
case("ctx_ptr", "R1 = skBuffentry.Addr", [A.mov64_reg(0, 1), A.exit_()], [PKT4], [e(Sk, steps=2)])
case("family4", "sk.Family = AF_INET", ld_field(S["family"]), [PKT4], [e(2, steps=2)])
case("family6", "AF_INET6", ld_field(S["family"]), [PKT6], [e(10, steps=2)])
case("family_none", "AF_UNSPEC", ld_field(S["family"]), [PKT_TINY], [e(0, steps=2)])
case("remote_port", "sk.DstPort", ld_field(S["remote_port"]), [PKT4], [e(0x50, steps=2)])
case("local_port", "sk.SrcPort", ld_field(S["local_port"]), [PKT4], [e(0x1234, steps=2)])
case("local_port_v6", "TCP after IPv6", ld_field(S["local_port"]), [PKT6], [e(0x1234, steps=2)])
case("local_ip4", "b2i(srcIP4) BigEndian", ld_field(S["local_ip4"]), [PKT4], [e(0xC0A80102, steps=2)])
case("remote_ip4", "dstIP4", ld_field(S["remote_ip4"]), [PKT4], [e(0x0A000001, steps=2)])
case("local_ip4_b1", "ip[1:2]", ld_field(S["local_ip4"] + 1, 1), [PKT4], [e(0xA8, steps=2)])
case("local_ip4_past", "ip[3:7] reads past the 4 address bytes (cap = L - 26)", ld_field(S["local_ip4"] + 3),
     [PKT4], [e(0x020A0000, steps=2)])
case("local_ip4_v6pkt", "srcIP4 = make(net.IP, 4): zeros", ld_field(S["local_ip4"]), [PKT6], [e(0, steps=2)])
case("local_ip6_v4pkt", "make(net.IP, 16)", ld_field(S["local_ip6"] + 12), [PKT4], [e(0, steps=2)])
case("local_ip6_slice_panic", "ip[15:17] of a 16-byte slice", ld_field(S["local_ip6"] + 15, 2), [PKT4],
     [e(0, status=PANIC_SLICE, steps=1, err_pc=0)])
case("local_ip6", "srcIP6[0:4]", ld_field(S["local_ip6"]), [PKT6], [e(0x10111213, steps=2)])
case("remote_ip6_last", "dstIP6[12:16]", ld_field(S["remote_ip6"] + 12), [PKT6], [e(0x2C2D2E2F, steps=2)])
case("remote_ip6_dw", "dstIP6[8:16] as BigEndian.Uint64", ld_field(S["remote_ip6"] + 8, 8), [PKT6],
     [e(0x28292A2B2C2D2E2F, steps=2)])
case("ip4_nil", "IPv4 shorter than 20: SrcIP nil, cap 0", ld_field(S["local_ip4"]), [PKT_SHORT4],
     [e(0, status=PANIC_SLICE, steps=1, err_pc=0)])
case("family_short4", "the IPv4 layer is still added", ld_field(S["family"]), [PKT_SHORT4], [e(2, steps=2)])
case("llc_protocol", "802.3 length: EthernetTypeLLC = 0", ld_field(S["protocol"]), [PKT_LLC], [e(0, steps=2)])
case("llc_family", "LLC/SNAP -> IPv4", ld_field(S["family"]), [PKT_LLC], [e(2, steps=2)])
case("cb_load_panic", "cb[offset:size] with offset > size", ld_field(48), [PKT4],
     [e(0, status=PANIC_SLICE, steps=1, err_pc=0)])
case("gso_segs", "not yet implemented", ld_field(S["gso_segs"]), [PKT4], [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("hwtstamp", "not yet implemented", ld_field(S["hwtstamp"], 8), [PKT4],
     [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("invalid_offset", "offset 9: invalid", ld_field(9, 1), [PKT4], [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("skb_end_offset", "offset 192 resolves (inclusive end), invalid", ld_field(192, 1), [PKT4],
     [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("tstamp_zero", "time.Time{}.Unix()", ld_field(S["tstamp"], 8), [PKT4], [e(-62135596800, steps=2)])


# ---- __sk_buff stores ---------------------------------------------------------------------------
def st_ld(off, val, st_size=4, ld_off=None, ld_size=4):
    return [A.ld_imm64(2, val), A.stx(st_size, 1, off, 2), A.ldx(ld_size, 0, 1, off if ld_off is None else ld_off),
            A.exit_()]


case("mark_rw", "markOrReservedTailroom", st_ld(S["mark"], 0xDEADBEEF), [PKT4], [e(0xDEADBEEF, steps=5)])
case("mark_rw_u8", "uint32(toSize(value)) with asm.Byte", st_ld(S["mark"], 0x1FF, st_size=1), [PKT4],
     [e(0xFF, steps=5)])
case("priority_rw", "priority", st_ld(S["priority"], 0x7), [PKT4], [e(7, steps=5)])
case("queue_mapping_rw", "uint16", st_ld(S["queue_mapping"], 0x12345), [PKT4], [e(0x2345, steps=5)])
case("tc_index_rw", "uint16", st_ld(S["tc_index"], 0xFFFF1), [PKT4], [e(0xFFF1, steps=5)])
case("tc_classid_rw", "cb[6:8] PutUint16 / Uint16, no toSize", st_ld(S["tc_classid"], 0x12345, ld_size=1), [PKT4],
     [e(0x2345, steps=5)])
case("tstamp_rw", "tstamp = time.Unix(int64(value), 0)", st_ld(S["tstamp"], 12345, st_size=8, ld_size=8), [PKT4],
     [e(12345, steps=5)])
case("cb_store_noop", "cb store is a no-op", [A.st(4, 1, 52, 9), A.mov64_imm(0, 1), A.exit_()], [PKT4],
     [e(1, steps=3)])
case("len_store_ro", "errReadOnly", [A.st(4, 1, S["len"], 9), A.exit_()], [PKT4],
     [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("data_store_ro", "errReadOnly", [A.st(4, 1, S["data"], 9), A.exit_()], [PKT4],
     [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])
case("family_store_ro", "errReadOnly", [A.st(4, 1, S["family"], 9), A.exit_()], [PKT4],
     [e(0, status=CTX_ACCESS, steps=1, err_pc=0)])


# ---- bpf_sock through skb->sk (SK.convertAccess :772-918) ----------------------------------------
def via_sk(off, size=4, store=None):
    it = [A.ldx(4, 2, 1, S["sk"])]
    if store is not None:
        it += [A.st(4, 2, off, store)]
    return it + [A.ldx(size, 0, 2, off), A.exit_()]


case("sk_family", "SK.Family", via_sk(K["family"]), [PKT4], [e(2, steps=3)])
case("sk_state", "BPF_TCP_CLOSE", via_sk(K["state"]), [PKT4], [e(7, steps=3)])
case("sk_src_port", "SrcPort", via_sk(K["src_port"]), [PKT4], [e(0x1234, steps=3)])
case("sk_dst_port", "DstPort", via_sk(K["dst_port"]), [PKT4], [e(0x50, steps=3)])
case("sk_src_ip4", "srcIP4", via_sk(K["src_ip4"]), [PKT4], [e(0xC0A80102, steps=3)])
case("sk_dst_ip4", "dstIP4", via_sk(K["dst_ip4"]), [PKT4], [e(0x0A000001, steps=3)])
case("sk_dst_ip6_wrap", "start := offset - 17*4 wraps below 68 -> slice panic", via_sk(K["dst_ip6"]), [PKT6],
     [e(0, status=PANIC_SLICE, steps=2, err_pc=1)])
case("sk_dst_ip6_68", "offset 68: dstIP6[0:4]", via_sk(68), [PKT6], [e(0x20212223, steps=3)])
case("sk_bound_dev_if", "read-write", via_sk(K["bound_dev_if"], store=5), [PKT4], [e(5, steps=4)])
case("sk_mark", "read-write", via_sk(K["mark"], store=0x77), [PKT4], [e(0x77, steps=4)])
case("sk_family_ro", "errReadOnly", [A.ldx(4, 2, 1, S["sk"]), A.st(4, 2, K["family"], 1), A.exit_()], [PKT4],
     [e(0, status=CTX_ACCESS, steps=2, err_pc=1)])
case("sk_invalid", "offset 80 (inclusive end)", via_sk(80, 1), [PKT4], [e(0, status=CTX_ACCESS, steps=2, err_pc=1)])


# ---- bpf_flow_keys through skb->flow_keys (:1031-1175) -------------------------------------------
def via_fk(off, size, store=None, st_size=2, ld_off=None):
    it = [A.ldx(4, 2, 1, S["flow_keys"])]
    if store is not None:
        it += [A.ld_imm64(3, store), A.stx(st_size, 2, off, 3)]
    return it + [A.ldx(size, 0, 2, off if ld_off is None else ld_off), A.exit_()]


case("fk_zero", "new FlowKeys", via_fk(FK["nhoff"], 2), [PKT4], [e(0, steps=3)])
case("fk_sport_rw", "uint16 field", via_fk(FK["sport"], 2, store=0x1234), [PKT4], [e(0x1234, steps=6)])
case("fk_sport_byte13", "offset 13 answers with the whole field, toSize(Byte)",
     via_fk(FK["sport"], 1, store=0x1234, ld_off=13), [PKT4], [e(0x34, steps=6)])
case("fk_flags_rw", "uint32 field", via_fk(FK["flags"], 4, store=0xABCDEF01, st_size=4), [PKT4],
     [e(0xABCDEF01, steps=6)])
case("fk_ip_panic", "ip[offset:...] of a 16-byte slice", via_fk(16, 4), [PKT4],
     [e(0, status=PANIC_SLICE, steps=2, err_pc=1)])
case("fk_end", "offset 40 (inclusive end): invalid", via_fk(40, 1), [PKT4],
     [e(0, status=CTX_ACCESS, steps=2, err_pc=1)])


# ---- packet memory (PlainMemory, ByteOrder BigEndian, :116-124) ------------------------------------
def via_data(off, size, store=None, st_size=None):
    it = [A.ldx(4, 2, 1, S["data"])]
    if store is not None:
        it += [A.st(st_size or size, 2, off, store)]
    return it + [A.ldx(size, 0, 2, off), A.exit_()]


case("pkt_be_u16", "BigEndian.Uint16", via_data(12, 2), [PKT4], [e(0x0800, steps=3)])
case("pkt_be_u32", "BigEndian.Uint32", via_data(26, 4), [PKT4], [e(0xC0A80102, steps=3)])
case("pkt_be_u64", "BigEndian.Uint64", via_data(0, 8), [PKT4], [e(0x0011223344556677, steps=3)])
case("pkt_be_store", "BigEndian.PutUint16", via_data(0, 1, store=0xABCD, st_size=2), [PKT4], [e(0xAB, steps=4)])
case("pkt_headroom", "headroom bytes are zero", via_data(-32, 8), [PKT4], [e(0, steps=3)])
case("pkt_before_head", "data - 33 = the flow keys entry's inclusive end", via_data(-33, 1), [PKT4],
     [e(0, status=CTX_ACCESS, steps=2, err_pc=1)])
case("pkt_tailroom", "tailroom bytes are zero", via_data(64, 8), [PKT4], [e(0, steps=3)])
case("pkt_past_end", "32 + L + 64 bytes: a 2-byte load at offset L+63 is out of bounds", via_data(64 + 63, 2),
     [PKT4], [e(0, status=BOUNDS, steps=2, err_pc=1)])
case("pkt_data_end_short", "data_end = data + L - 32", [A.ldx(4, 2, 1, S["data"]), A.ldx(4, 3, 1, S["data_end"]),
                                                        A.mov64_reg(0, 3), A.alu64("sub", 0, 2, reg=True), A.exit_()],
     [PKT4], [e(32, steps=5)])


# ---- LD_ABS / LD_IND (emulator_linux_.go:198-288) ------------------------------------------------
def r6ctx(items):
    return [A.mov64_reg(6, 1)] + items


case("ldabs_h", "R0 = BigEndian u16 at data + 12", r6ctx([A.ld_abs(2, 12), A.exit_()]), [PKT4], [e(0x0800, steps=3)])
case("ldabs_w", "saddr", r6ctx([A.ld_abs(4, 26), A.exit_()]), [PKT4], [e(0xC0A80102, steps=3)])
case("ldabs_b", "protocol", r6ctx([A.ld_abs(1, 23), A.exit_()]), [PKT4], [e(6, steps=3)])
case("ldabs_dw", "asm.DWord", r6ctx([A.ld_abs(8, 0), A.exit_()]), [PKT4], [e(0x0011223344556677, steps=3)])
case("ldind_b", "data + src + imm", r6ctx([A.mov64_imm(7, 14), A.ld_ind(1, 7, 9), A.exit_()]), [PKT4],
     [e(6, steps=4)])
case("ldind_neg", "uint32(src) wraps into the headroom", r6ctx([A.mov64_imm(7, -4), A.ld_ind(4, 7, 0), A.exit_()]),
     [PKT4], [e(0, steps=4)])
case("ldabs_clobbers", "R1-R5 := 0", r6ctx([A.mov64_imm(1, 1), A.mov64_imm(2, 2), A.mov64_imm(3, 3),
                                           A.mov64_imm(4, 4), A.mov64_imm(5, 5), A.ld_abs(1, 0),
                                           A.mov64_reg(0, 1), A.alu64("or", 0, 2, reg=True),
                                           A.alu64("or", 0, 3, reg=True), A.alu64("or", 0, 4, reg=True),
                                           A.alu64("or", 0, 5, reg=True), A.exit_()]),
     [PKT4], [e(0, steps=13)])
case("ldabs_r6_not_skb", "R6 is not a sk_buff", [A.mov64_reg(6, 10), A.ld_abs(1, 0), A.exit_()], [PKT4],
     [e(0, status=LDABS, steps=2, err_pc=1)])
case("ldabs_r6_inside_skb", "R6 anywhere inside the sk_buff entry", [A.mov64_reg(6, 1), A.alu64("add", 6, 100),
                                                                     A.ld_abs(2, 12), A.exit_()], [PKT4],
     [e(0x0800, steps=4)])
case("ldabs_oob", "packet read out of bounds", r6ctx([A.ld_abs(4, 64 + 62), A.exit_()]), [PKT4],
     [e(0, status=LDABS, steps=2, err_pc=1)])
case("ldabs_unresolved", "no entry past the last leak", r6ctx([A.ld_abs(4, 4096), A.exit_()]), [PKT4],
     [e(0, status=LDABS, steps=2, err_pc=1)])
case("ldabs_into_fk", "data - 33 is the flow keys' offset 40: Load error", r6ctx([A.ld_abs(1, -33), A.exit_()]),
     [PKT4], [e(0, status=LDABS, steps=2, err_pc=1)])
case("ldind_badreg", "Registers.Get(11) panics after the R6 check", r6ctx([A.raw(0x50, 0, 11, 0, 0), A.exit_()]),
     [PKT4], [e(0, status=BADREG, steps=2, err_pc=1)])

# ---- user-given sock / flow keys (context_sk_buff.go:24-26, Load :53-66) --------------------------
# A context's "sock" replaces the SK SKBuffFromBytes made -- every field, the __sk_buff fields read
# through skb.sk included (:522-600) -- and its net.IP fields are what SK.UnmarshalJSON leaves
# (:721-757): make(net.IP, 4 / 16) unless net.ParseIP parses the string, which returns 16 bytes
# (::ffff:a.b.c.d for IPv4), so a user-given IPv4 address reads as zeros through the 4-byte
# ipv4 fields.  "flowKeys" are the flow keys' starting values.
def sock(**kw):
    return {"sock": kw}


def fks(**kw):
    return {"flowKeys": kw}


V4M = bytes(10) + b"\xff\xff"   # net.ParseIP's 16-byte form of an IPv4 address: 10 zeros, ff ff, a.b.c.d
case("sock_family", "SK replaces skb.sk; __sk_buff->family = sk.sk.Family (:522-525)", ld_field(S["family"]),
     [PKT4], [e(10, steps=2)], contexts=[sock(family=10)])
case("sock_sk_family", "bpf_sock->family", via_sk(K["family"]), [PKT4], [e(10, steps=3)], contexts=[sock(family=10)])
case("sock_type", "bpf_sock->type = SockType (:806-811)", via_sk(K["type"]), [PKT4], [e(5, steps=3)],
     contexts=[sock(sockType=5, protocol=17)])
case("sock_protocol", "bpf_sock->protocol (:815-820)", via_sk(K["protocol"]), [PKT4], [e(17, steps=3)],
     contexts=[sock(sockType=5, protocol=17)])
case("sock_state_zero", "a user SK's State is what it gives (0), not BPF_TCP_CLOSE", via_sk(K["state"]), [PKT4],
     [e(0, steps=3)], contexts=[sock(family=2)])
case("sock_state", "bpf_sock->state (:906-911)", via_sk(K["state"]), [PKT4], [e(10, steps=3)],
     contexts=[sock(state=10)])
case("sock_rxq_u32", "toSize(uint64(RXQueueMapping)) of int32 -1, asm.Word", via_sk(K["rx_queue_mapping"]), [PKT4],
     [e(0xFFFFFFFF, steps=3)], contexts=[sock(rxQueueMapping=-1)])
case("sock_rxq_u64", "int32 -1 sign-extends", via_sk(K["rx_queue_mapping"], 8), [PKT4], [e(-1, steps=3)],
     contexts=[sock(rxQueueMapping=-1)])
case("sock_local_port", "__sk_buff->local_port = sk.sk.SrcPort (:593-597)", ld_field(S["local_port"]), [PKT4],
     [e(0xBEEF, steps=2)], contexts=[sock(srcPort=0xBEEF, dstPort=8080)])
case("sock_remote_port", "__sk_buff->remote_port = sk.sk.DstPort (:584-588)", ld_field(S["remote_port"]), [PKT4],
     [e(8080, steps=2)], contexts=[sock(srcPort=0xBEEF, dstPort=8080)])
case("sock_src_port", "bpf_sock->src_port", via_sk(K["src_port"]), [PKT4], [e(0xBEEF, steps=3)],
     contexts=[sock(srcPort=0xBEEF, dstPort=8080)])
case("sock_dst_port", "bpf_sock->dst_port", via_sk(K["dst_port"]), [PKT4], [e(8080, steps=3)],
     contexts=[sock(srcPort=0xBEEF, dstPort=8080)])
case("sock_ip4_reads_zero", "ParseIP's 16-byte form: srcIP4[0:4] are zeros", ld_field(S["local_ip4"]), [PKT4],
     [e(0, steps=2)], contexts=[sock(srcIP4="192.168.1.2")])
case("sock_ip4_16_bytes", "srcIP4[3:11] of ::ffff:192.168.1.2 reaches the ff ff", ld_field(S["local_ip4"] + 3, 8),
     [PKT4], [e(int.from_bytes((V4M + bytes([192, 168, 1, 2]))[3:11], "big"), steps=2)],
     contexts=[sock(srcIP4="192.168.1.2")])
case("sock_sk_ip4_16_bytes", "bpf_sock->src_ip4 at +3, 8 bytes", via_sk(K["src_ip4"] + 3, 8), [PKT4],
     [e(0xFF, steps=3)], contexts=[sock(srcIP4="192.168.1.2")])
case("sock_ip4_default_len4", "dstIP4 = make(net.IP, 4): [3:7] panics", ld_field(S["remote_ip4"] + 3), [PKT4],
     [e(0, status=PANIC_SLICE, steps=1, err_pc=0)], contexts=[sock(family=2)])
case("sock_ip4_unparsable", "ParseIP fails: make(net.IP, 4) stays", ld_field(S["remote_ip4"]), [PKT4],
     [e(0, steps=2)], contexts=[sock(dstIP4="not-an-ip")])
case("sock_ip6", "srcIP6 = ParseIP(...).To16()", ld_field(S["local_ip6"]), [PKT4], [e(0x20010DB8, steps=2)],
     contexts=[sock(srcIP6="2001:db8::1")])
case("sock_ip6_last", "srcIP6[12:16]", ld_field(S["local_ip6"] + 12), [PKT4], [e(1, steps=2)],
     contexts=[sock(srcIP6="2001:db8::1")])
case("sock_ip6_from_v4", "dstIP6 = ParseIP(\"10.0.0.1\").To16(): ::ffff:10.0.0.1", ld_field(S["remote_ip6"] + 8, 8),
     [PKT4], [e(0x0000FFFF0A000001, steps=2)], contexts=[sock(dstIP6="10.0.0.1")])
case("sock_sk_dst_ip6_68", "offset 68: dstIP6[0:4] of the user's address", via_sk(68), [PKT4],
     [e(0x20010DB8, steps=3)], contexts=[sock(dstIP6="2001:db8::2")])
case("sock_mark", "bpf_sock->mark starts at the user's value", via_sk(K["mark"]), [PKT4], [e(5, steps=3)],
     contexts=[sock(mark=5)])
case("sock_mark_rw", "and is writable", via_sk(K["mark"], store=0x77), [PKT4], [e(0x77, steps=4)],
     contexts=[sock(mark=5)])
case("sock_bound_dev_if", "bound_dev_if", via_sk(K["bound_dev_if"]), [PKT4], [e(3, steps=3)],
     contexts=[sock(boundDevIF=3)])
case("sock_priority", "priority", via_sk(K["priority"]), [PKT4], [e(6, steps=3)], contexts=[sock(priority=6)])
case("sock_nil_ips", "an SK literal: its net.IP fields are nil, ip[0:4] panics", ld_field(S["local_ip4"]), [PKT4],
     [e(0, status=PANIC_SLICE, steps=1, err_pc=0)], contexts=[dict(sock(family=2), nilIPs=True)])
case("sock_keeps_skb_fields", "skb.len / protocol still come from the packet", ld_field(S["protocol"]), [PKT4],
     [e(0x0800, steps=2)], contexts=[sock(family=10)])
case("sock_mixed_batch", "per-context: a user SK, none, another user SK", ld_field(S["family"]), [PKT4, PKT4, PKT6],
     [e(10, steps=2), e(2, steps=2), e(99, steps=2)], contexts=[sock(family=10), None, sock(family=99)])
case("fk_user_nhoff", "FlowKeys start from the user's values (:1031-1041)", via_fk(FK["nhoff"], 2), [PKT4],
     [e(14, steps=3)], contexts=[fks(nhoff=14, sport=4660, ipProto=6, flags=7, flowLabel=0x12345)])
case("fk_user_sport", "sport", via_fk(FK["sport"], 2), [PKT4], [e(4660, steps=3)],
     contexts=[fks(nhoff=14, sport=4660, ipProto=6, flags=7, flowLabel=0x12345)])
case("fk_user_ip_proto", "ip_proto", via_fk(FK["ip_proto"], 1), [PKT4], [e(6, steps=3)],
     contexts=[fks(nhoff=14, sport=4660, ipProto=6, flags=7, flowLabel=0x12345)])
case("fk_user_flags", "flags", via_fk(FK["flags"], 4), [PKT4], [e(7, steps=3)],
     contexts=[fks(nhoff=14, sport=4660, ipProto=6, flags=7, flowLabel=0x12345)])
case("fk_user_flow_label", "flow_label", via_fk(FK["flow_label"], 4), [PKT4], [e(0x12345, steps=3)],
     contexts=[fks(nhoff=14, sport=4660, ipProto=6, flags=7, flowLabel=0x12345)])
case("fk_user_store", "a store replaces the user's value", via_fk(FK["sport"], 2, store=0x55), [PKT4],
     [e(0x55, steps=6)], contexts=[fks(sport=4660)])
case("fk_user_ip_panics", "ip[offset:...] panics whatever the user's ip", via_fk(16, 4), [PKT4],
     [e(0, status=PANIC_SLICE, steps=2, err_pc=1)], contexts=[fks(ip="10.0.0.1")])
case("sock_and_fk", "both: flow_keys.nhoff + __sk_buff->family",
     [A.ldx(4, 2, 1, S["flow_keys"]), A.ldx(2, 0, 2, FK["nhoff"]), A.ldx(4, 3, 1, S["family"]),
      A.alu64("add", 0, 3, reg=True), A.exit_()], [PKT4], [e(14 + 10, steps=5)],
     contexts=[dict(sock(family=10), **fks(nhoff=14))])

# ---- context load and the leaked-entry layout (context_sk_buff.go:42-119) -------------------------
case("load_vxlan", "a second Ethernet layer: 'handling of multiple link layers not supported'",
     [A.mov64_imm(0, 1), A.exit_()], [PKT_VXLAN], [e(0, status=CTX_LOAD, steps=0)])
seq = [PKT4, PKT_VXLAN, PKT6, pad(PKT4, 100)]
case("leak_layout", "Cleanup deletes only the sk_buff entry: sock / flow keys / packet leak",
     ld_field(S["sk"]), seq,
     [e(addrs(64)[0], steps=2), e(0, status=CTX_LOAD, steps=0), e(addrs(80, [64])[0], steps=2),
      e(addrs(100, [64, 80])[0], steps=2)])
case("leak_data", "data of later processes", ld_field(S["data"]), [PKT4, PKT4, PKT4],
     [e(addrs(64)[2] + 32, steps=2), e(addrs(64, [64])[2] + 32, steps=2), e(addrs(64, [64, 64])[2] + 32, steps=2)])
case("stack_same", "the stack entry is reused", [A.mov64_reg(0, 10), A.exit_()], [PKT4, PKT6],
     [e(St + 256, steps=2), e(St + 256, steps=2)])

if __name__ == "__main__":
    with open(os.path.join(HERE, "kat_skb.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_skb.py", "cases": CASES}, f, indent=1)
    print(f"{len(CASES)} cases")
