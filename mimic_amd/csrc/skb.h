// skb.h -- the sk_buff context on the device (LinuxContextSKBuff, context_sk_buff.go:42-119,
// and SKBuff / SK / FlowKeys, emulator_linux_sk_buff.go).
//
// One SkbRec per packet holds everything the reference keeps in its SKBuff, SK and FlowKeys
// objects: the fields SKBuffFromBytes derives from the packet headers, the fields a program
// may store into, and a 40-byte copy of the IP-address bytes.  SK's net.IP fields are slices
// of gopacket's private copy of the packet, so reads see the ORIGINAL bytes even after the
// program has rewritten its packet memory.
//
//   mimic_skb_prep_kernel (skb.hip)    : header walk -> SkbRec[i] + address footprint[i]
//   exclusive scan of the footprints   : where packet i's leaked entries sit
//   JIT / interpreter kernels          : context load, then __sk_buff / bpf_sock / flow_keys
//                                        accesses via skb_access(); LD_ABS / LD_IND
//
// Address layout of one sequential reference run (memory_controller.go:58-112 first fit).
// NewProcess adds the stack at St.  Load then adds the sk_buff (192 B) right after it, and
// then the sock (80 B), flow keys (40 B) and packet (32 + L + 64 B).  Cleanup deletes the
// stack and the sk_buff only (context_sk_buff.go:110-119).  So the next process reuses
// [St, St+S+193) exactly, while the sock / flow-keys / packet entries of every earlier
// process stay allocated:
//   Sk = St + S + 1                 sk_buff [Sk, Sk+192]        same for every packet
//   Ka = leak_base + prefix_i       sock    [Ka, Ka+80]
//   Fa = Ka + 81                    flow    [Fa, Fa+40]
//   Pa = Fa + 41                    packet  [Pa, Pa+96+L]       data = Pa+32, data_end = Pa+L
// where prefix_i sums (219 + L_j) over the earlier packets whose Load succeeded.
#pragma once
#include <stdint.h>

#include "../../include/mimic_amd.h"   // mimic_skb_custom (user-given sock / flow keys)

#define SKB_STRUCT_SIZE 192u     // SKBuff.Size(), emulator_linux_sk_buff.go:679-681
#define SKB_SK_SIZE 80u          // SK.Size()
#define SKB_FK_SIZE 40u          // FlowKeys.Size()
#define SKB_HEADROOM 32u         // :113
#define SKB_TAILROOM 64u         // :116
#define SKB_FOOT_FIXED 219u      // (80+1) + (40+1) + (96+1): address span of one packet's leaks
#define SKB_LOAD_FAILED 0x80000000u
// the prep kernel's block (skb.hip): packet i's leak prefix is prefix[i] (within its block) +
// prefix[n + (i >> SKB_PREP_LOG2)] (the block's offset in the batch)
#define SKB_PREP_LOG2 8u
#define SKB_SNAP 40u
#define SKB_REC_BYTES 160u
// flags in packet i's within-block leak prefix word (skb.hip; skb_leak_pre masks them off):
//   EXC   the frame is one skb_fast does not take; with a sparse prep (KParams::skb_rec_built == 2)
//         only such frames have their derived words in skb_drv, every other frame's record is built
//         by whoever loads the process, from the packet's first bytes (skb_fast_rec);
//   DIRTY the packet memory's headroom or tailroom holds a non-zero byte (Load zeroes them)
#define SKB_PFX_EXC (1ull << 63)
#define SKB_PFX_DIRTY (1ull << 62)
#define SKB_PFX_MASK ((1ull << 62) - 1ull)

// net.IP as the reference holds it: kind 0 = make(net.IP, n) (zeros, cap n), 1 = nil,
// 2 = gopacket's packet copy from byte `off` (cap = L - off: Go slices may read past n)
struct SkbIP {
    uint32_t off;
    uint8_t kind, n, pad[2];   // ip[0].pad[0]: the prep kernel's rooms flag (SKB_DIRTY_Q)
};

struct SkbRec {  // 160 bytes
    // ---- derived at load (read-only for the program) ----
    uint32_t len;              // L | SKB_LOAD_FAILED
    uint16_t protocol, vlan_proto, vlan_tci;
    uint8_t vlan_present, family;   // family: SK.Family (AF_UNSPEC 0 / AF_INET 2 / AF_INET6 10)
    uint32_t sport, dport;     // SK.SrcPort / DstPort
    SkbIP ip[4];               // SK srcIP4, dstIP4, srcIP6, dstIP6
    uint32_t snap_base;
    uint8_t snap[SKB_SNAP];    // packet bytes [snap_base, snap_base + 40) (0 beyond L)
    // ---- writable state ----
    uint32_t mark, priority;   // SKBuff.markOrReservedTailroom, priority
    uint16_t queue_mapping, tc_index;
    uint8_t cb6, cb7, pad1[2];   // cb[6:8] (tc_classid)
    int64_t tstamp;            // time.Time as Unix seconds
    uint32_t sk_bound_dev_if, sk_mark, sk_priority;
    // FlowKeys, :1003-1019
    uint16_t fk_nhoff, fk_thoff, fk_addr_proto;
    uint8_t fk_is_frag, fk_is_first_frag, fk_is_encap, fk_ip_proto;
    uint16_t fk_n_proto, fk_sport, fk_dport;
    uint32_t fk_flags, fk_flow_label;
    uint32_t cust;             // 1 + the process's entry in the batch's mimic_skb_custom table (0: none)
};

#define SKB_TSTAMP_ZERO (-62135596800ll)   // time.Time{}.Unix()
// The record's first SKB_DERIVED_Q words are what the header walk derives; the rest is the
// writable state, the same constants for every process at Load (zeros, tstamp = time.Time{}).
// The prep kernel writes only the derived words; whoever loads the process sets the rest
// (skb_load: in HBM; the JIT: in its LDS slot).
#define SKB_DERIVED_Q 12u
static_assert(__builtin_offsetof(SkbRec, mark) == 8 * SKB_DERIVED_Q, "writable state follows the derived words");
// The prep kernel also finds whether the packet memory's headroom or tailroom holds a non-zero byte
// (Load hands the program zeroed rooms, context_sk_buff.go:110-119): a spare byte of the derived
// words, ip[0].pad[0] (word SKB_DIRTY_Q, bit SKB_DIRTY_SHIFT), so whoever loads the process knows
// without reading the rooms itself (a dependent round trip on every process's critical path).
#define SKB_DIRTY_Q 3u
#define SKB_DIRTY_SHIFT 16u
static_assert(__builtin_offsetof(SkbRec, ip) + __builtin_offsetof(SkbIP, pad) == 8 * SKB_DIRTY_Q + SKB_DIRTY_SHIFT / 8,
              "the rooms flag byte");
static_assert(__builtin_offsetof(SkbRec, tstamp) == 8 * (SKB_DERIVED_Q + 2), "tstamp is word 14");
static_assert(sizeof(SkbRec) == 8 * (SKB_DERIVED_Q + 8), "8 writable words");

#ifndef SKB_DEV
#define SKB_DEV static __device__ __forceinline__
#endif
// the field accessors are big switches reached from every generic memory access of a JIT
// kernel: out of line (value arguments and results only, so no scratch) to keep the kernels
// small and their hipRTC compile fast
#ifndef SKB_COLD
#define SKB_COLD static __device__ __noinline__
#endif

SKB_DEV uint64_t skb_writable_word(uint32_t q) {   // word SKB_DERIVED_Q + q of a loaded record
    return q == 2 ? (uint64_t)SKB_TSTAMP_ZERO : 0ull;
}

struct SkbRes {
    uint64_t v;
    int st;   // 0 or a status
};

// packet bytes for the header walk: b[k] is byte k of the packet; here plain memory
struct SkbBytes {
    const uint8_t *p;
    __device__ uint8_t operator[](uint32_t k) const { return p[k]; }
};
// the header walk's bytes from a block's LDS windows: thread t's first SKB_WIN bytes of its
// packet as dwords, dword q at w[q * T + t] (a wave reading the same header offset hits
// consecutive dwords); bytes past the window (deep tunnels only) come from global memory
#define SKB_WIN 96u   // 6 chunks of 16 B: every byte skb_fast reads (up to 67), and a packet's header window stays within two 64-byte sectors of its slot
template <uint32_t T>
struct SkbWinBytes {
    const uint32_t *w;
    const uint8_t *p;    // the packet in global memory
    uint32_t t;
    __device__ uint8_t operator[](uint32_t k) const {
        if (k < SKB_WIN) return (uint8_t)(w[(k >> 2) * T + t] >> (8 * (k & 3)));
        return p[k];
    }
};
// stage the window: 16-byte chunks that start inside the packet (one may run into the tailroom)
template <uint32_t T>
SKB_DEV void skb_stage(uint32_t *w, uint32_t t, const uint8_t *pkt, uint32_t L) {
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
#pragma unroll
    for (uint32_t c = 0; c < SKB_WIN / 16; c++) {
        if (16 * c < L) {
            const u32x4u v = *(const u32x4u *)(pkt + 16 * c);
            w[(4 * c) * T + t] = v.x;
            w[(4 * c + 1) * T + t] = v.y;
            w[(4 * c + 2) * T + t] = v.z;
            w[(4 * c + 3) * T + t] = v.w;
        }
    }
}

template <class B>
SKB_DEV uint16_t skb_rd16(const B &b, uint32_t k) { return (uint16_t)((b[k] << 8) | b[k + 1]); }

// ---------------------------------------------------------------------------------------
// SKBuffFromBytes (emulator_linux_sk_buff.go:108-265) over gopacket v1.1.19's eager decode
// (gopacket.NewPacket(data, LayerTypeEthernet, Default)).  Only the layers that set SKBuff
// fields or lead to another such layer are walked: Ethernet (+802.3 length -> LLC/SNAP),
// Dot1Q / QinQ, IPv4 (+options, fragments stop), IPv6 (+Routing / Destination options),
// TCP, UDP and the UDP tunnels that decode another link / network layer (VXLAN 4789, Geneve
// 6081, GTPv1-U 2152), IPIP / IPv6-in-IP.  A second link, network or transport layer is the
// reference's "handling of multiple ... layers not supported" error.  The walk is iterative
// (a small state machine) rather than recursive.  Returns 0, or 1 for that error.
// ---------------------------------------------------------------------------------------
enum { SW_DONE, SW_ETH, SW_ETYPE, SW_LLC, SW_DOT1Q, SW_IP, SW_PROTO };

template <class B>
SKB_DEV int skb_walk(const B &pkt, uint32_t L, SkbRec &r) {
    uint32_t st = SW_ETH, o = 0, len = L, t = 0;
    uint32_t link = 0, net = 0, trans = 0;
    for (uint32_t guard = 0; guard < L + 64; guard++) {  // each Dot1Q step consumes 4 bytes
        switch (st) {
        case SW_ETH: {
            if (len < 14) return 0;      // "Ethernet packet too small": no layer
            if (link++) return 1;
            t = skb_rd16(pkt, o + 12);
            uint32_t pl = len - 14;
            if (t < 0x0600) {            // 802.3 length field: EthernetTypeLLC, payload trimmed
                if (pl > t) pl = t;
                t = 0;
            }
            r.protocol = (uint16_t)t;    // skb.protocol = EthernetType (:187)
            o += 14;
            len = pl;
            st = SW_ETYPE;
            break;
        }
        case SW_ETYPE:
            if (len == 0) return 0;
            switch (t) {
            case 0x0000: st = SW_LLC; break;
            case 0x0800: case 0x86DD: st = SW_IP; break;
            case 0x8100: case 0x88a8: st = SW_DOT1Q; break;
            case 0x6558: st = SW_ETH; break;   // transparent Ethernet bridging
            default: return 0;
            }
            break;
        case SW_LLC: {   // LLC + SNAP (llc.go)
            if (len < 3) return 0;
            const uint32_t d = o;
            uint32_t hl = 3;
            if (!(pkt[d + 2] & 1) || (pkt[d + 2] & 3) == 1) {   // I- or S-format: 2-byte control
                if (len < 4) return 0;
                hl = 4;
            }
            if ((pkt[d] & 0xfe) != 0xaa || (pkt[d + 1] & 0xfe) != 0xaa) return 0;
            if (len - hl < 5) return 0;
            t = skb_rd16(pkt, d + hl + 3);
            o += hl + 5;
            len -= hl + 5;
            st = SW_ETYPE;
            break;
        }
        case SW_DOT1Q: {
            if (len < 4) return 0;
            r.vlan_proto = skb_rd16(pkt, o + 2);   // Dot1Q.Type (:182)
            r.vlan_tci = skb_rd16(pkt, o);
            r.vlan_present = 1;
            t = skb_rd16(pkt, o + 2);
            o += 4;
            len -= 4;
            st = SW_ETYPE;
            break;
        }
        case SW_IP: {    // decodeIPv4orIPv6
            if (len == 0) return 0;
            const uint32_t v = pkt[o] >> 4;
            const uint32_t d = o;
            if (v == 4) {
                if (net++) return 1;
                r.family = 2;
                if (len < 20) {  // SrcIP / DstIP stay nil
                    r.ip[0].kind = 1;
                    r.ip[1].kind = 1;
                    return 0;
                }
                r.ip[0].kind = 2; r.ip[0].off = o + 12;
                r.ip[1].kind = 2; r.ip[1].off = o + 16;
                const uint32_t ihl = pkt[d] & 0x0f, ff = skb_rd16(pkt, d + 6);
                uint32_t tl = skb_rd16(pkt, d + 2);
                if (tl == 0) tl = len;   // TSO
                if (tl < 20 || ihl < 5 || ihl * 4 > tl) return 0;
                uint32_t dl = len;
                if (len > tl) dl = tl;
                else if (len < tl && ihl * 4 > len) return 0;
                for (uint32_t q = 20; q < ihl * 4;) {   // options: a malformed one ends the decode
                    const uint8_t ot = pkt[d + q];
                    if (ot == 0) break;
                    if (ot == 1) { q++; continue; }
                    if (ihl * 4 - q < 2) return 0;
                    const uint8_t ol = pkt[d + q + 1];
                    if (ihl * 4 - q < ol) return 0;
                    if (ol <= 2) return 0;
                    q += ol;
                }
                if ((ff & 0x2000) || (ff & 0x1fff)) return 0;   // a fragment
                t = pkt[d + 9];
                o += ihl * 4;
                len = dl - ihl * 4;
                st = SW_PROTO;
            } else if (v == 6) {
                if (net++) return 1;
                r.family = 10;
                if (len < 40) {
                    r.ip[2].kind = 1;
                    r.ip[3].kind = 1;
                    return 0;
                }
                r.ip[2].kind = 2; r.ip[2].off = o + 8;
                r.ip[3].kind = 2; r.ip[3].off = o + 24;
                uint32_t next = pkt[d + 6];
                const uint32_t plen = skb_rd16(pkt, d + 4);
                if (next == 0) return 0;   // Hop-by-Hop / jumbograms: not restated
                if (plen == 0) return 0;
                uint32_t po = o + 40, pl = len - 40;
                if (pl > plen) pl = plen;
                for (int k = 0; k < 16; k++) {
                    if (next == 43 || next == 60) {   // Routing / Destination options
                        if (pl < 2) return 0;
                        const uint32_t hl = (pkt[po + 1] + 1u) * 8;
                        if (pl < hl) return 0;
                        next = pkt[po];
                        po += hl;
                        pl -= hl;
                        continue;
                    }
                    if (next == 44) return 0;  // Fragment
                    break;
                }
                t = next;
                o = po;
                len = pl;
                st = SW_PROTO;
            } else {
                return 0;
            }
            break;
        }
        case SW_PROTO:
            if (len == 0) return 0;
            if (t == 6) {            // TCP: the layer is added even when its decode fails
                if (trans++) return 1;
                if (len >= 20) {
                    r.sport = skb_rd16(pkt, o);
                    r.dport = skb_rd16(pkt, o + 2);
                }
                return 0;
            }
            if (t == 4 || t == 41) { st = SW_IP; break; }
            if (t != 17) return 0;
            {                        // UDP (udp.go) and the tunnels behind it
                if (trans++) return 1;
                if (len < 8) return 0;
                r.sport = skb_rd16(pkt, o);
                r.dport = skb_rd16(pkt, o + 2);
                const uint32_t ulen = skb_rd16(pkt, o + 4);
                uint32_t plen;
                if (ulen >= 8) plen = (ulen > len ? len : ulen) - 8;
                else if (ulen == 0) plen = len - 8;
                else return 0;
                if (plen == 0) return 0;
                // NextLayerType: the destination port's type unless it is Payload, else the
                // source port's (gopacket's UDPPortLayerType table)
                uint32_t port = r.sport;
                switch (r.dport) {
                case 53: case 123: case 4789: case 67: case 68: case 546: case 547: case 5060: case 6343:
                case 6081: case 3784: case 2152: case 623: case 1812:
                    port = r.dport;
                    break;
                default:
                    break;
                }
                const uint32_t po = o + 8;
                if (port == 4789) {          // VXLAN, then Ethernet
                    if (plen < 8) return 0;
                    o = po + 8;
                    len = plen - 8;
                    st = SW_ETH;
                } else if (port == 6081) {   // Geneve: 8 + options, then the protocol type
                    if (plen < 8) return 0;
                    const uint32_t hl = 8 + (pkt[po] & 0x3f) * 4u;
                    if (plen < hl) return 0;
                    t = skb_rd16(pkt, po + 2);
                    o = po + hl;
                    len = plen - hl;
                    st = SW_ETYPE;
                } else if (port == 2152) {   // GTPv1-U, then IPv4 / IPv6
                    if (plen < 8) return 0;
                    const uint32_t hl = (pkt[po] & 0x07) ? 12 : 8;
                    if ((pkt[po] & 0x04) || plen <= hl) return 0;
                    o = po + hl;
                    len = plen - hl;
                    st = SW_IP;
                } else {
                    return 0;
                }
            }
            break;
        default:
            return 0;
        }
    }
    return 0;
}

// r.snap[k] = packet byte b + k (0 at or past L), k < SKB_SNAP
template <class B>
SKB_DEV void skb_snap(const B &pkt, uint32_t b, uint32_t L, SkbRec &r) {
#pragma unroll
    for (uint32_t k = 0; k < SKB_SNAP; k++) r.snap[k] = b + k < L ? pkt[b + k] : 0;
}
// from the LDS window: 10 dwords cut out of 11 with funnel shifts instead of 40 byte reads (the
// copy is most of the prep kernel's LDS traffic); bytes at or past L masked to 0
template <uint32_t T>
SKB_DEV void skb_snap(const SkbWinBytes<T> &pkt, uint32_t b, uint32_t L, SkbRec &r) {
    if (b + SKB_SNAP + 4 > SKB_WIN) {
#pragma unroll
        for (uint32_t k = 0; k < SKB_SNAP; k++) r.snap[k] = b + k < L ? pkt[b + k] : 0;
        return;
    }
    const uint32_t q0 = b >> 2, sh = 8 * (b & 3);
    const int32_t valid = (int32_t)L - (int32_t)b;   // bytes of the snap inside the packet
    uint32_t lo = pkt.w[q0 * T + pkt.t];
#pragma unroll
    for (uint32_t k = 0; k < SKB_SNAP / 4; k++) {
        const uint32_t hi = pkt.w[(q0 + k + 1) * T + pkt.t];
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh >> 3);
        const int32_t n = valid - 4 * (int32_t)k;
        v = n >= 4 ? v : n <= 0 ? 0u : (v & ((1u << (8 * n)) - 1u));
        __builtin_memcpy(&r.snap[4 * k], &v, 4);
        lo = hi;
    }
}

// the record before the walk: zero, make(net.IP, 4/16) capacities, time.Time{}
SKB_DEV void skb_rec_reset(SkbRec &r) {
    uint64_t *w = (uint64_t *)&r;
    for (uint32_t q = 0; q < sizeof(SkbRec) / 8; q++) w[q] = 0;
    r.ip[0].n = 4; r.ip[1].n = 4; r.ip[2].n = 16; r.ip[3].n = 16;
    r.tstamp = SKB_TSTAMP_ZERO;
}
// the one IP slice window programs can read (IPv4: src..dst+11, IPv6: src..dst+23)
SKB_DEV uint32_t skb_snap_base(const SkbRec &r) {
    return r.family == 10 && r.ip[2].kind == 2 ? r.ip[2].off : (r.ip[0].kind == 2 ? r.ip[0].off : 0u);
}

// SKBuffFromBytes + the parts of LinuxContextSKBuff.Load that do not depend on addresses
template <class B>
SKB_DEV void skb_init(const B &pkt, uint32_t L, SkbRec &r) {
    skb_rec_reset(r);
    const int err = skb_walk(pkt, L, r);
    r.len = L | (err ? SKB_LOAD_FAILED : 0u);
    const uint32_t b = skb_snap_base(r);
    r.snap_base = b;
    skb_snap(pkt, b, L, r);
}

// ---------------------------------------------------------------------------------------
// The common frames without a walk: Ethernet + IPv4 (no options) / IPv6 (no extension headers)
// + TCP / UDP (no tunnel port), or a non-IP EtherType, decoded straight from the packet's first
// SKB_WIN bytes held in registers (w[q] = bytes 4q..4q+3) at constant offsets -- the same decisions
// skb_walk makes for these frames, in the same order.  Everything else (802.3 / LLC, VLAN tags,
// IPv4 options, IPv6 extension headers, IP-in-IP, UDP tunnels) returns false: the general walk
// decodes it.  No frame taken here fails Load (only a second layer of one kind does).
// ---------------------------------------------------------------------------------------
#define SKW8(k) ((w[(k) >> 2] >> (8 * ((k) & 3))) & 0xffu)
#define SKW16(k) ((SKW8(k) << 8) | SKW8((k) + 1))
template <uint32_t O>   // the transport header's offset: 34 (IPv4) or 54 (IPv6)
SKB_DEV bool skb_fast_l4(const uint32_t *w, uint32_t t, uint32_t len, SkbRec &r) {
    if (len == 0) return true;
    if (t == 6) {            // TCP: ports when the header is complete
        if (len >= 20) {
            r.sport = SKW16(O);
            r.dport = SKW16(O + 2);
        }
        return true;
    }
    if (t == 4 || t == 41) return false;   // IP in IP
    if (t != 17) return true;
    if (len < 8) return true;
    r.sport = SKW16(O);
    r.dport = SKW16(O + 2);
    const uint32_t ulen = SKW16(O + 4);
    uint32_t plen;
    if (ulen >= 8) plen = (ulen > len ? len : ulen) - 8;
    else if (ulen == 0) plen = len - 8;
    else return true;
    if (plen == 0) return true;
    uint32_t port = r.sport;
    switch (r.dport) {
    case 53: case 123: case 4789: case 67: case 68: case 546: case 547: case 5060: case 6343:
    case 6081: case 3784: case 2152: case 623: case 1812:
        port = r.dport;
        break;
    default:
        break;
    }
    return !(port == 4789 || port == 6081 || port == 2152);   // tunnels decode another layer
}
SKB_DEV bool skb_fast(const uint32_t *w, uint32_t L, SkbRec &r) {
    if (L < 14) return true;                       // no Ethernet layer
    const uint32_t t = SKW16(12);
    if (t < 0x0600 || t == 0x8100 || t == 0x88a8 || t == 0x6558) return false;
    r.protocol = (uint16_t)t;
    if (L == 14 || (t != 0x0800 && t != 0x86DD)) return true;
    const uint32_t len = L - 14, v = SKW8(14) >> 4;
    if (v == 4) {
        r.family = 2;
        if (len < 20) {
            r.ip[0].kind = 1;
            r.ip[1].kind = 1;
            return true;
        }
        r.ip[0].kind = 2; r.ip[0].off = 26;
        r.ip[1].kind = 2; r.ip[1].off = 30;
        const uint32_t ihl = SKW8(14) & 0x0f, ff = SKW16(20);
        uint32_t tl = SKW16(16);
        if (tl == 0) tl = len;
        if (tl < 20 || ihl < 5 || ihl * 4 > tl) return true;
        uint32_t dl = len;
        if (len > tl) dl = tl;
        else if (len < tl && ihl * 4 > len) return true;
        if (ihl != 5) return false;                // options
        if ((ff & 0x2000) || (ff & 0x1fff)) return true;
        return skb_fast_l4<34>(w, SKW8(23), dl - 20, r);
    }
    if (v == 6) {
        r.family = 10;
        if (len < 40) {
            r.ip[2].kind = 1;
            r.ip[3].kind = 1;
            return true;
        }
        r.ip[2].kind = 2; r.ip[2].off = 22;
        r.ip[3].kind = 2; r.ip[3].off = 38;
        const uint32_t next = SKW8(20), plen = SKW16(18);
        if (next == 0 || plen == 0) return true;
        uint32_t pl = len - 40;
        if (pl > plen) pl = plen;
        if (next == 43 || next == 60) return false;   // extension headers
        if (next == 44) return true;                  // a fragment
        return skb_fast_l4<54>(w, next, pl, r);
    }
    return true;
}
// r.snap from the registers for a constant base B (0, 22 or 26), bytes at or past L zero
template <uint32_t B>
SKB_DEV void skb_snap_regs(const uint32_t *w, uint32_t L, SkbRec &r) {
    const int32_t valid = (int32_t)L - (int32_t)B;
#pragma unroll
    for (uint32_t k = 0; k < SKB_SNAP / 4; k++) {
        const uint32_t q = (B >> 2) + k;
        uint32_t v = __builtin_amdgcn_alignbyte(w[q + 1], w[q], B & 3);   // v_alignbyte: stays in registers
        const int32_t n = valid - 4 * (int32_t)k;
        v = n >= 4 ? v : n <= 0 ? 0u : (v & ((1u << (8 * n)) - 1u));
        __builtin_memcpy(&r.snap[4 * k], &v, 4);
    }
}
#undef SKW8
#undef SKW16

// the whole record (skb_init) of a frame skb_fast takes, from its first SKB_WIN bytes in registers;
// false (r partly written) for the frames the general walk must decode
SKB_DEV bool skb_fast_rec(const uint32_t *w, uint32_t L, SkbRec &r) {
    skb_rec_reset(r);
    if (!skb_fast(w, L, r)) return false;
    r.len = L;
    const uint32_t b = skb_snap_base(r);
    r.snap_base = b;
    if (b == 26) skb_snap_regs<26>(w, L, r);
    else if (b == 22) skb_snap_regs<22>(w, L, r);
    else skb_snap_regs<0>(w, L, r);
    return true;
}

// skb_init over the packet's first SKB_WIN bytes in registers (w), the general walk through the
// block's LDS window (win, column t) for the frames skb_fast does not take.  Returns whether
// skb_fast took the frame.
template <uint32_t T>
SKB_DEV bool skb_init_regs(const uint32_t *w, uint32_t *win, uint32_t t, const uint8_t *pkt, uint32_t L, SkbRec &r) {
    if (skb_fast_rec(w, L, r)) return true;
#ifdef MIMIC_PREP_FAST_ONLY   // measurement only (tools/prep_probe.py): no general walk
    r.len = L;
    return false;
#endif
#pragma unroll
    for (uint32_t q = 0; q < SKB_WIN / 4; q++) win[q * T + t] = w[q];
    skb_init(SkbWinBytes<T>{win, pkt, t}, L, r);
    return false;
}

// ---------------------------------------------------------------------------------------
// convertAccess (SKBuff :295-676, SK :772-918, FlowKeys :1031-1175).  Status codes are those
// of include/mimic_amd.h; loads return the value in v, stores take it from v.
// ---------------------------------------------------------------------------------------
SKB_DEV uint64_t skb_to_size(uint64_t v, uint32_t n) { return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1)); }

// the process's user-given sock (flag MIMIC_SKB_CUSTOM_SK) or flow keys (_FLOWKEYS), or null
SKB_DEV const mimic_skb_custom *skb_cust(const SkbRec &r, const mimic_skb_custom *cu, uint32_t flag) {
    if (!cu || !r.cust) return nullptr;
    const mimic_skb_custom *c = cu + (r.cust - 1);
    return (c->flags & flag) ? c : nullptr;
}

// LinuxContextSKBuff.Load's user-given SK / FlowKeys (context_sk_buff.go:53-66) for process i,
// after the record's writable state got its defaults: the writable SK words and the flow keys
// start from the user's values; the record remembers the entry for the read-only SK fields
SKB_DEV void skb_apply_custom(SkbRec &r, const mimic_skb_custom *cu, uint32_t i) {
    if (!cu || !cu[i].flags) return;
    const mimic_skb_custom &c = cu[i];
    if (c.flags & MIMIC_SKB_CUSTOM_SK) {
        r.sk_bound_dev_if = c.sk_bound_dev_if;
        r.sk_mark = c.sk_mark;
        r.sk_priority = c.sk_priority;
    }
    if (c.flags & MIMIC_SKB_CUSTOM_FLOWKEYS) {
        r.fk_nhoff = c.fk_nhoff;
        r.fk_thoff = c.fk_thoff;
        r.fk_addr_proto = c.fk_addr_proto;
        r.fk_is_frag = c.fk_is_frag;
        r.fk_is_first_frag = c.fk_is_first_frag;
        r.fk_is_encap = c.fk_is_encap;
        r.fk_ip_proto = c.fk_ip_proto;
        r.fk_n_proto = c.fk_n_proto;
        r.fk_sport = c.fk_sport;
        r.fk_dport = c.fk_dport;
        r.fk_flags = c.fk_flags;
        r.fk_flow_label = c.fk_flow_label;
    }
    r.cust = i + 1;
}

// copy(v, ip[start:start+n]); b2i(v): a slice-bounds panic past the capacity.  A user-given SK's
// addresses are the bytes its UnmarshalJSON parsed (mimic_skb_custom.sk_ip)
SKB_DEV int skb_ip_load(const SkbRec &r, const mimic_skb_custom *cu, uint32_t which, uint64_t start, uint32_t n, uint64_t &v) {
    if (const mimic_skb_custom *c = skb_cust(r, cu, MIMIC_SKB_CUSTOM_SK)) {
        if (start + n > c->sk_ip_len[which]) return 27;   // MIMIC_PANIC_SLICE
        uint64_t x = 0;
        for (uint32_t k = 0; k < n; k++) x = (x << 8) | c->sk_ip[which][(uint32_t)start + k];
        v = x;
        return 0;
    }
    const SkbIP ip = r.ip[which];
    const uint64_t cap = ip.kind == 0 ? ip.n : ip.kind == 1 ? 0 : (uint64_t)(r.len & ~SKB_LOAD_FAILED) - ip.off;
    if (start + n > cap) return 27;   // MIMIC_PANIC_SLICE
    uint64_t x = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t b = ip.kind == 2 ? r.snap[ip.off - r.snap_base + (uint32_t)start + k] : 0u;
        x = (x << 8) | b;
    }
    v = x;
    return 0;
}

#define SKB_RO() do { if (!load) return 26; } while (0)   // errReadOnly -> MIMIC_ERR_CTX_ACCESS

// SKBuff.convertAccess; data = skb.data, end = skb.end, ka/fa = sock / flow-keys addresses; the
// fields read through skb.sk come from a user-given SK when the process has one (cu)
SKB_DEV int skb_convert_(SkbRec &r, const mimic_skb_custom *cu, uint32_t ifindex, uint32_t data, uint32_t end,
                         uint32_t ka, uint32_t fa, uint32_t off, uint32_t n, uint64_t &v, bool load) {
    const uint64_t val = v;
    if (off == 88 || off == 132 || off == 136) {
        if (const mimic_skb_custom *c = skb_cust(r, cu, MIMIC_SKB_CUSTOM_SK)) {
            SKB_RO();
            v = skb_to_size(off == 88 ? c->sk_family : off == 132 ? c->sk_dst_port : c->sk_src_port, n);
            return 0;
        }
    }
    switch (off) {
    case 0: SKB_RO(); v = skb_to_size(r.len & ~SKB_LOAD_FAILED, n); return 0;
    case 4: SKB_RO(); v = 0; return 0;                                   // pkt_type & 7 (never set)
    case 8: if (load) v = skb_to_size(r.mark, n); else r.mark = (uint32_t)skb_to_size(val, n); return 0;
    case 12: if (load) v = skb_to_size(r.queue_mapping, n); else r.queue_mapping = (uint16_t)skb_to_size(val, n); return 0;
    case 16: SKB_RO(); v = skb_to_size(r.protocol, n); return 0;
    case 20: SKB_RO(); v = r.vlan_present ? 1 : 0; return 0;
    case 24: SKB_RO(); v = skb_to_size(r.vlan_tci, n); return 0;
    case 28: SKB_RO(); v = skb_to_size(r.vlan_proto, n); return 0;
    case 32: if (load) v = skb_to_size(r.priority, n); else r.priority = (uint32_t)skb_to_size(val, n); return 0;
    case 36: SKB_RO(); v = 0; return 0;                                  // ingress_ifindex: skbIIF (0)
    case 40: SKB_RO(); v = skb_to_size(ifindex, n); return 0;            // dev.IFIndex
    case 44: if (load) v = skb_to_size(r.tc_index, n); else r.tc_index = (uint16_t)skb_to_size(val, n); return 0;
    case 68: SKB_RO(); v = 0; return 0;                                  // hash (never set)
    case 72:                                                             // tc_classid: native u16 at cb[6:8]
        if (load) v = (uint64_t)(r.cb6 | (r.cb7 << 8));
        else { r.cb6 = (uint8_t)val; r.cb7 = (uint8_t)(val >> 8); }
        return 0;
    case 76: SKB_RO(); v = skb_to_size(data, n); return 0;
    case 80: SKB_RO(); v = end; return 0;                                // data_end: cb[32:36]
    case 84: SKB_RO(); v = 0; return 0;                                  // napi_id
    case 88: SKB_RO(); v = skb_to_size(r.family, n); return 0;           // sk.Family
    case 132: SKB_RO(); v = skb_to_size(r.dport, n); return 0;           // remote_port
    case 136: SKB_RO(); v = skb_to_size(r.sport, n); return 0;           // local_port
    case 140: SKB_RO(); v = 0; return 0;                                 // data_meta: cb[36:38]
    case 144: case 148: SKB_RO(); v = fa; return 0;                      // flow_keys
    case 152: case 156:                                                  // tstamp
        if (load) v = (uint64_t)r.tstamp; else r.tstamp = (int64_t)val;
        return 0;
    case 160: SKB_RO(); v = 0; return 0;                                 // wire_len: cb[0:4]
    case 164: case 176: case 184: case 188: return 26;                   // "not yet implemented"
    case 168: case 172: SKB_RO(); v = ka; return 0;                      // sk
    default: break;
    }
    if (off >= 48 && off < 68) {   // cb[5]: a load slices cb[offset:size] (low > high): panic
        if (load) return 27;
        return 0;
    }
    if (off >= 92 && off < 96) { SKB_RO(); return skb_ip_load(r, cu, 1, off - 92, n, v); }     // remote_ip4
    if (off >= 96 && off < 100) { SKB_RO(); return skb_ip_load(r, cu, 0, off - 96, n, v); }    // local_ip4
    if (off >= 100 && off < 116) { SKB_RO(); return skb_ip_load(r, cu, 3, off - 100, n, v); }  // remote_ip6
    if (off >= 116 && off < 132) { SKB_RO(); return skb_ip_load(r, cu, 2, off - 116, n, v); }  // local_ip6
    return 26;   // "invalid offset"
}

// SK.convertAccess (a user-given SK's read-only fields from its table entry)
SKB_DEV int sk_convert_(SkbRec &r, const mimic_skb_custom *cu, uint32_t off, uint32_t n, uint64_t &v, bool load) {
    const uint64_t val = v;
    if (const mimic_skb_custom *c = skb_cust(r, cu, MIMIC_SKB_CUSTOM_SK)) {
        switch (off) {
        case 4: SKB_RO(); v = skb_to_size(c->sk_family, n); return 0;
        case 8: SKB_RO(); v = skb_to_size(c->sk_type, n); return 0;
        case 12: SKB_RO(); v = skb_to_size(c->sk_protocol, n); return 0;
        case 44: SKB_RO(); v = skb_to_size(c->sk_src_port, n); return 0;
        case 48: SKB_RO(); v = skb_to_size(c->sk_dst_port, n); return 0;
        case 72: SKB_RO(); v = skb_to_size(c->sk_state, n); return 0;
        case 76: SKB_RO(); v = skb_to_size((uint64_t)(int64_t)c->sk_rx_queue_mapping, n); return 0;
        default: break;
        }
    }
    switch (off) {
    case 0: if (load) v = skb_to_size(r.sk_bound_dev_if, n); else r.sk_bound_dev_if = (uint32_t)skb_to_size(val, n); return 0;
    case 4: SKB_RO(); v = skb_to_size(r.family, n); return 0;
    case 8: SKB_RO(); v = 0; return 0;                                   // type
    case 12: SKB_RO(); v = 0; return 0;                                  // protocol
    case 16: if (load) v = skb_to_size(r.sk_mark, n); else r.sk_mark = (uint32_t)skb_to_size(val, n); return 0;
    case 20: if (load) v = skb_to_size(r.sk_priority, n); else r.sk_priority = (uint32_t)skb_to_size(val, n); return 0;
    case 44: SKB_RO(); v = skb_to_size(r.sport, n); return 0;
    case 48: SKB_RO(); v = skb_to_size(r.dport, n); return 0;
    case 72: SKB_RO(); v = skb_to_size(7, n); return 0;                  // state: BPF_TCP_CLOSE
    case 76: SKB_RO(); v = 0; return 0;                                  // rx_queue_mapping
    default: break;
    }
    if (off >= 24 && off < 28) { SKB_RO(); return skb_ip_load(r, cu, 0, off - 24, n, v); }
    if (off >= 28 && off < 44) { SKB_RO(); return skb_ip_load(r, cu, 2, off - 28, n, v); }
    if (off >= 52 && off < 56) { SKB_RO(); return skb_ip_load(r, cu, 1, off - 52, n, v); }
    if (off >= 56 && off < 72) { SKB_RO(); return skb_ip_load(r, cu, 3, (uint64_t)(uint32_t)(off - 68), n, v); }  // start wraps below 68
    return 26;
}

// FlowKeys.convertAccess: each field answers for every offset it covers
#define FK_RW(fld, T) do { if (load) v = skb_to_size(r.fld, n); else r.fld = (T)skb_to_size(val, n); return 0; } while (0)
SKB_DEV int fk_convert_(SkbRec &r, uint32_t off, uint32_t n, uint64_t &v, bool load) {
    const uint64_t val = v;
    switch (off) {
    case 0: case 1: FK_RW(fk_nhoff, uint16_t);
    case 2: case 3: FK_RW(fk_thoff, uint16_t);
    case 4: case 5: FK_RW(fk_addr_proto, uint16_t);
    case 6: FK_RW(fk_is_frag, uint8_t);
    case 7: FK_RW(fk_is_first_frag, uint8_t);
    case 8: FK_RW(fk_is_encap, uint8_t);
    case 9: FK_RW(fk_ip_proto, uint8_t);
    case 10: case 11: FK_RW(fk_n_proto, uint16_t);
    case 12: case 13: FK_RW(fk_sport, uint16_t);
    case 14: case 15: FK_RW(fk_dport, uint16_t);
    case 32: case 33: case 34: case 35: FK_RW(fk_flags, uint32_t);
    case 36: case 37: case 38: case 39: FK_RW(fk_flow_label, uint32_t);
    default: break;
    }
    if (off >= 16 && off < 32) return 27;   // ip[offset:...] of a 16-byte slice
    return 26;
}
#undef FK_RW
#undef SKB_RO

SKB_COLD SkbRes skb_convert(SkbRec *r, const mimic_skb_custom *cu, uint32_t ifindex, uint32_t data, uint32_t end,
                            uint32_t ka, uint32_t fa, uint32_t off, uint32_t n, uint64_t v, bool load) {
    SkbRes o;
    o.st = skb_convert_(*r, cu, ifindex, data, end, ka, fa, off, n, v, load);
    o.v = v;
    return o;
}
SKB_COLD SkbRes sk_convert(SkbRec *r, const mimic_skb_custom *cu, uint32_t off, uint32_t n, uint64_t v, bool load) {
    SkbRes o;
    o.st = sk_convert_(*r, cu, off, n, v, load);
    o.v = v;
    return o;
}
SKB_COLD SkbRes fk_convert(SkbRec *r, uint32_t off, uint32_t n, uint64_t v, bool load) {
    SkbRes o;
    o.st = fk_convert_(*r, off, n, v, load);
    o.v = v;
    return o;
}
