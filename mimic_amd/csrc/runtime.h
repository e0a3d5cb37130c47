// runtime.h -- the device-side model of one reference process, shared by the batch
// interpreter (interp.hip) and the per-program JIT kernels (jit.cpp generates them and
// compiles them with hipRTC at run time; this header is embedded into the library).
//
// A lane of a wavefront is one vCPU of the reference VM; these functions are its memory
// controller (MemoryController.GetEntry over the lane's address space), the stack / xdp_md /
// packet memories, the map helpers and the exact ALU / jump semantics of the effective
// opcode table.
#pragma once
#include <stdint.h>

#include "layout.h"
#include "hashmap.h"
#include "skb.h"
#include "../../include/mimic_amd.h"

typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

#define DEV static __device__ __forceinline__
// pop-only launches insert without stripe locks (hashmap.h h_insert_nolock); MIMIC_JIT_DEFS=
// MIMIC_HASH_NOLOCK=0 builds the locked rounds instead (measurement)
#ifndef MIMIC_HASH_NOLOCK
#define MIMIC_HASH_NOLOCK 1
#endif
// no program of the launch deletes (KParams.hash_pop_only); a JIT kernel knows it at compile time
#ifdef MIMIC_HASH_POPONLY
#define HASH_POPONLY(kp) (MIMIC_HASH_POPONLY != 0)
#else
#define HASH_POPONLY(kp) ((kp).hash_pop_only != 0)
#endif
// hash tables read-only during the launch (KParams.hash_ro); a JIT kernel knows it at compile time
#ifdef MIMIC_HASH_RO
#define HASH_RO(kp) (MIMIC_HASH_RO != 0)
#else
#define HASH_RO(kp) ((kp).hash_ro != 0)
#endif

// Read-only tables are read through the constant address space so that wave-uniform
// indices become scalar (s_load) fetches through the scalar cache.
#define CONST_AS __attribute__((address_space(4)))
template <typename T>
DEV T cget(const T *p, uint32_t i) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized tables only");
    uint32_t w[sizeof(T) / 4];
#if defined(__HIP_DEVICE_COMPILE__)
    const CONST_AS uint32_t *q = (const CONST_AS uint32_t *)(p + i);
#else
    const uint32_t *q = (const uint32_t *)(p + i);  // host pass: never executed
#endif
#pragma unroll
    for (unsigned k = 0; k < sizeof(T) / 4; k++) w[k] = q[k];
    T out;
    __builtin_memcpy(&out, w, sizeof(T));
    return out;
}

enum RegionKind : uint32_t {
    RK_UNRES = 0, RK_STACK = 1, RK_XDP = 2, RK_GLOBAL = 3, RK_NOTVMMEM = 4, RK_NOTDATASEC = 5,
    RK_SKB = 6, RK_SK = 7, RK_FK = 8,   // *SKBuff / *SK / *FlowKeys: VMMem via convertAccess
    RK_BEPKT = 9                         // sk_buff packet: PlainMemory with ByteOrder BigEndian
};

// The context kind of a batch.  A JIT kernel is generated for one kind and defines
// MIMIC_CTX_FIXED, so that the other kind's code folds away; the interpreter reads kp.ctx_kind.
#ifdef MIMIC_CTX_FIXED
#define CTX_SKB_MODE(kp) (MIMIC_CTX_FIXED == CTX_SKB)
#else
#define CTX_SKB_MODE(kp) ((kp).ctx_kind == CTX_SKB)
#endif

struct Ref {
    uint32_t rk, off, limit;
    int32_t map, sub, prog;
    uint8_t *ptr;
};

struct Lane {
    uint32_t lane;        // private-memory lane index
    int32_t cpu;
    uint32_t M;           // packet memory length H+L+T
    uint8_t *pkt;         // packet memory (device)
    uint32_t data, data_end, ingress, rxq, egress;
    uint32_t xdp_dirty;
    uint64_t sm0, sm1;    // stack words / granules already written in this process
    uint32_t nframes, tailcalls;
    // one-entry translation cache of a static plain region (a map value backing, set by the
    // lookup helper): addresses in [t_lo, t_lo + t_n) resolve to t_ptr + (a - t_lo) without
    // the segment scan.  Static entries never move, so an entry stays exact; t_n = 0 = empty.
    uint32_t t_lo, t_n;
    uint8_t *t_ptr;
    // the packet entry's address (xdp: P; sk_buff: Pa) and the sk_buff context
    uint32_t pa;
    uint32_t ka;          // sock entry (flow keys at ka + 81)
    SkbRec *rec;          // this process's SKBuff / SK / FlowKeys state (HBM, per packet)
};

static constexpr int EXIT_SIG = -1;

// the CPU ID of the processes lane g runs (KParams::cpu_lanes)
DEV int32_t lane_cpu(const KParams &kp, uint32_t g) {
    if (g < kp.cpu_lanes) return (int32_t)(kp.vcpu_begin + g);
    return g == kp.cpu_lanes ? -1 : (int32_t)kp.total_vcpus;
}

// ---------------------------------------------------------------------------------------
// raw loads / stores (unaligned accesses are legal on gfx950 global memory).  Every engine
// pointer (packets, arena, private memory, results) is global memory: the accesses are made
// through the global address space so they compile to global_* instructions -- FLAT ones would
// also count against lgkmcnt and make every LDS / scalar-load wait drain them too.
// ---------------------------------------------------------------------------------------
#if defined(__HIP_DEVICE_COMPILE__)
#define GAS __attribute__((address_space(1)))
#else
#define GAS
#endif
template <typename T>
DEV GAS T *gp(T *p) { return (GAS T *)p; }

// Run's `select { case <-ctx.Done(): return ctx.Err() }` before a process's first step (vm.go:
// 344-349): the state of packet i's context word -- 0 (not done), 1 (canceled), 2 (deadline
// exceeded).  The word lives in pinned host memory that the host writes while the launch runs: a
// system-scope load reads it past the caches (one PCIe round trip, made only when the launch was
// given a context, KParams::cancel_any).
DEV uint32_t ctx_done(const KParams &kp, uint32_t i) {
    const uint32_t *w = kp.cancel_pp ? kp.cancel_pp[i] : kp.cancel;
    if (!w) return 0u;
    return __hip_atomic_load((GAS const uint32_t *)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
DEV const GAS T *gp(const T *p) { return (const GAS T *)p; }

// index of the j-th packet lane g runs under the batch's schedule, or NO_PKT
#define NO_PKT 0xffffffffu
DEV uint32_t pkt_index(const KParams &kp, uint32_t g, uint32_t j, uint32_t ex_begin, uint32_t ex_count) {
    if (j >= kp.per_lane) return NO_PKT;
    if (kp.sched == SCHED_CHUNKED) {
        const uint64_t ii = (uint64_t)g * kp.per_lane + j;
        return ii < kp.n ? (uint32_t)ii : NO_PKT;
    }
    if (kp.sched == SCHED_INTERLEAVED) {
        const uint64_t ii = (uint64_t)j * kp.lanes + (g >= kp.sched_shift ? g - kp.sched_shift : g + kp.lanes - kp.sched_shift);
        return ii < kp.n ? (uint32_t)ii : NO_PKT;
    }
    return j < ex_count ? *(const GAS uint32_t *)(kp.sched_pkts + ex_begin + j) : NO_PKT;
}

// spread kernels: the lane (vCPU - vcpu_begin) packet i runs on under a chunked / interleaved
// schedule -- the inverse of pkt_index (interleaved: packet ii runs on lane (ii + shift) mod lanes)
DEV uint32_t spread_lane(const KParams &kp, uint32_t i) {
    if (kp.sched == SCHED_CHUNKED) return i / kp.per_lane;
    uint32_t r = i % kp.cpu_lanes + kp.sched_shift;
    return r >= kp.cpu_lanes ? r - kp.cpu_lanes : r;
}

// the packet after packet i (the j-th of lane g) under the schedule: the chunked and
// interleaved schedules step by 1 and by the lane count
DEV uint32_t pkt_next(const KParams &kp, uint32_t i, uint32_t j, uint32_t ex_begin, uint32_t ex_count) {
    if (j >= kp.per_lane) return NO_PKT;
    if (kp.sched == SCHED_EXPLICIT) return j < ex_count ? *(const GAS uint32_t *)(kp.sched_pkts + ex_begin + j) : NO_PKT;
    const uint64_t ii = (uint64_t)i + (kp.sched == SCHED_CHUNKED ? 1u : kp.lanes);
    return ii < kp.n ? (uint32_t)ii : NO_PKT;
}

DEV uint64_t ld_n(const uint8_t *p, uint32_t n) {
    switch (n) {
    case 1: return *gp(p);
    case 2: return *(const GAS u16u *)p;
    case 4: return *(const GAS u32u *)p;
    case 8: return *(const GAS u64u *)p;
    default: {
        uint64_t v = 0;
        for (uint32_t i = n; i-- > 0;) v = (v << 8) | *gp(p + i);
        return v;
    }
    }
}
DEV void st_n(uint8_t *p, uint32_t n, uint64_t v) {
    switch (n) {
    case 1: *gp(p) = (uint8_t)v; return;
    case 2: *(GAS u16u *)p = (uint16_t)v; return;
    case 4: *(GAS u32u *)p = (uint32_t)v; return;
    case 8: *(GAS u64u *)p = v; return;
    default:
        for (uint32_t i = 0; i < n; i++) *gp(p + i) = (uint8_t)(v >> (8 * i));
    }
}

// Streaming accesses (packet bytes, descriptors, per-packet results) are each touched by one
// process: non-temporal loads / stores keep them from evicting the lane-resident lines (per-CPU
// map values, stack words) that later packets of the same vCPU reuse from L2.
DEV uint64_t ld_n_nt(const uint8_t *p, uint32_t n) {
    switch (n) {
    case 1: return __builtin_nontemporal_load(gp(p));
    case 2: return __builtin_nontemporal_load((const GAS u16u *)p);
    case 4: return __builtin_nontemporal_load((const GAS u32u *)p);
    case 8: return __builtin_nontemporal_load((const GAS u64u *)p);
    default: return ld_n(p, n);
    }
}
template <typename T>
DEV T ld_nt(const T *p) { return __builtin_nontemporal_load(gp(p)); }
template <typename T>
DEV void st_nt(T *p, T v) { __builtin_nontemporal_store(v, gp(p)); }

// Lane value cache (JIT, jit.cpp analyze_vc): a lane's own per-CPU array row (<= 32 bytes) held
// in four 64-bit registers w0..w3, little-endian like the arena.  An access of n (1..8) bytes at
// byte offset o of the row, o + n <= row size, any alignment: selects, no dynamic indexing (which
// would put the row in scratch).
DEV uint64_t vc_sel(uint32_t q, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
    return q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : q == 3 ? w3 : 0ull;
}
DEV uint64_t vc_load(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint32_t o, uint32_t n) {
    const uint32_t q = o >> 3, sh = (o & 7) * 8;
    const uint64_t lo = vc_sel(q, w0, w1, w2, w3);
    uint64_t v = lo;
    if (sh) v = (lo >> sh) | (vc_sel(q + 1, w0, w1, w2, w3) << (64 - sh));
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}
DEV void vc_store(uint64_t &w0, uint64_t &w1, uint64_t &w2, uint64_t &w3, uint32_t o, uint32_t n, uint64_t v) {
    const uint32_t q = o >> 3, sh = (o & 7) * 8;
    const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
    v &= m;
    const uint64_t lm = m << sh, lv = v << sh;
    const uint64_t hm = sh ? m >> (64 - sh) : 0ull, hv = sh ? v >> (64 - sh) : 0ull;
    w0 = q == 0 ? ((w0 & ~lm) | lv) : w0;
    w1 = q == 1 ? ((w1 & ~lm) | lv) : q == 0 ? ((w1 & ~hm) | hv) : w1;
    w2 = q == 2 ? ((w2 & ~lm) | lv) : q == 1 ? ((w2 & ~hm) | hv) : w2;
    w3 = q == 3 ? ((w3 & ~lm) | lv) : q == 2 ? ((w3 & ~hm) | hv) : w3;
}

// private memory: byte offset o of lane l lives at priv + ((o>>3)*priv_lanes + l)*8 + (o&7)
DEV uint8_t *priv_b(const KParams &kp, uint32_t lane, uint32_t o) {
    return kp.priv + (((size_t)(o >> 3) * kp.priv_lanes + lane) << 3) + (o & 7);
}
DEV uint64_t priv_load(const KParams &kp, uint32_t lane, uint32_t o, uint32_t n) {
    if ((o & 7) + n <= 8) return ld_n(priv_b(kp, lane, o), n);
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; i++) v |= (uint64_t)*gp(priv_b(kp, lane, o + i)) << (8 * i);
    return v;
}
DEV void priv_store(const KParams &kp, uint32_t lane, uint32_t o, uint32_t n, uint64_t v) {
    if ((o & 7) + n <= 8) {
        st_n(priv_b(kp, lane, o), n, v);
        return;
    }
    for (uint32_t i = 0; i < n; i++) *gp(priv_b(kp, lane, o + i)) = (uint8_t)(v >> (8 * i));
}

// ---------------------------------------------------------------------------------------
// stack (PlainMemory of StackFrameCount*StackFrameSize zero bytes, vm.go:208-210)
//
// The reference gives every process a fresh zeroed stack.  Instead of zeroing 2 KiB per
// packet, validity is tracked per lane: sm0 has one bit per 8-byte word of the first 512
// bytes (frames 0 and 1, where programs live), sm1 one bit per (1<<chunk_shift)-byte
// granule of the rest.  Reads of never-written bytes return 0 without touching memory; the
// first write to a word stores the whole zero-extended word.
// ---------------------------------------------------------------------------------------
#define STK_FINE 512u
// JIT kernels with deferred slow paths keep the validity masks in LDS (MIMIC_SM_LDS): a deferral
// site would otherwise hold the two 64-bit masks live in VGPRs through the whole program
// (measured on cfg 5's chain: +50 VGPRs)
#ifdef MIMIC_SM_LDS
__shared__ uint64_t mimic_sm_[2 * 256];
#define SM0(L) mimic_sm_[threadIdx.x]
#define SM1(L) mimic_sm_[256 + threadIdx.x]
#else
#define SM0(L) (L).sm0
#define SM1(L) (L).sm1
#endif
// LDS stack window (JIT kernels that define MIMIC_LDS_STACK_Q, jit.cpp): the stack bytes
// [256 - 8Q, 256) -- the top of frame 0, where R10 - k lands in programs without BPF-to-BPF
// calls -- live in LDS instead of the lane's private memory in HBM, word q of thread t at
// mimic_lstk_[q * 256 + t] (a wave's same-word accesses hit consecutive banks).  The validity
// bits work the same for both stores; the window is touched only by its own lane.
#ifdef MIMIC_LDS_STACK_Q
#define STK_LDS_LO (256u - 8u * MIMIC_LDS_STACK_Q)
__shared__ uint64_t mimic_lstk_[MIMIC_LDS_STACK_Q * 256];
DEV bool stk_in_lds(uint32_t o) { return o - STK_LDS_LO < 8u * MIMIC_LDS_STACK_Q; }
DEV uint64_t &stk_lw(uint32_t o) { return mimic_lstk_[((o - STK_LDS_LO) >> 3) * 256u + threadIdx.x]; }
#else
DEV bool stk_in_lds(uint32_t) { return false; }
DEV uint64_t &stk_lw(uint32_t) { __builtin_trap(); }
#endif
DEV bool stk_valid(const KParams &kp, const Lane &L, uint32_t o) {
    return o < STK_FINE ? ((SM0(L) >> (o >> 3)) & 1) : ((SM1(L) >> ((o - STK_FINE) >> kp.chunk_shift)) & 1);
}
// the whole 8-byte word holding stack byte o (o & ~7) := w
DEV void stk_word_set(const KParams &kp, const Lane &L, uint32_t o, uint64_t w) {
    if (stk_in_lds(o)) stk_lw(o) = w;
    else *gp((uint64_t *)priv_b(kp, L.lane, o & ~7u)) = w;
}
// one stack byte (valid or not: the caller checks)
DEV uint32_t stk_byte(const KParams &kp, const Lane &L, uint32_t o) {
    if (stk_in_lds(o)) return (uint32_t)(stk_lw(o) >> (8 * (o & 7))) & 0xffu;
    return *gp(priv_b(kp, L.lane, o));
}
DEV void stk_touch(const KParams &kp, Lane &L, uint32_t o) {
    if (o < STK_FINE) {
        const uint32_t q = o >> 3;
        if (!((SM0(L) >> q) & 1)) {
            stk_word_set(kp, L, q << 3, 0);
            SM0(L) |= 1ull << q;
        }
    } else {
        const uint32_t c = (o - STK_FINE) >> kp.chunk_shift;
        if (!((SM1(L) >> c) & 1)) {
            const uint32_t q0 = (STK_FINE + (c << kp.chunk_shift)) >> 3, nq = (1u << kp.chunk_shift) >> 3;
            for (uint32_t q = 0; q < nq; q++) *gp((uint64_t *)priv_b(kp, L.lane, (q0 + q) << 3)) = 0;
            SM1(L) |= 1ull << c;
        }
    }
}
DEV uint64_t stack_load(const KParams &kp, const Lane &L, uint32_t o, uint32_t n) {
    if ((o & 7) + n <= 8) {
        if (!stk_valid(kp, L, o)) return 0;
        if (stk_in_lds(o)) {
            const uint64_t v = stk_lw(o) >> (8 * (o & 7));
            return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
        }
        return ld_n(priv_b(kp, L.lane, o), n);
    }
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t oo = o + i;
        if (stk_valid(kp, L, oo)) v |= (uint64_t)stk_byte(kp, L, oo) << (8 * i);
    }
    return v;
}
DEV void stack_store(const KParams &kp, Lane &L, uint32_t o, uint32_t n, uint64_t v) {
    if ((o & 7) + n <= 8) {
        const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
        const uint32_t sh = 8 * (o & 7);
        if (o < STK_FINE && !((SM0(L) >> (o >> 3)) & 1)) {
            // first write to this word: store the whole word, zero-extended around the value
            stk_word_set(kp, L, o, (v & m) << sh);
            SM0(L) |= 1ull << (o >> 3);
            return;
        }
        stk_touch(kp, L, o);
        if (stk_in_lds(o)) {
            uint64_t &w = stk_lw(o);
            w = (w & ~(m << sh)) | ((v & m) << sh);
            return;
        }
        st_n(priv_b(kp, L.lane, o), n, v);
        return;
    }
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t oo = o + i;
        stk_touch(kp, L, oo);
        if (stk_in_lds(oo)) {
            uint64_t &w = stk_lw(oo);
            const uint32_t sh = 8 * (oo & 7);
            w = (w & ~(0xffull << sh)) | ((uint64_t)(uint8_t)(v >> (8 * i)) << sh);
        } else {
            *gp(priv_b(kp, L.lane, oo)) = (uint8_t)(v >> (8 * i));
        }
    }
}

// ---------------------------------------------------------------------------------------
// xdp_md (24-byte PlainMemory, context_xdp_md.go:56-105)
// ---------------------------------------------------------------------------------------
DEV uint32_t xdp_word(const Lane &L, uint32_t w) {
    uint32_t v = 0;
    v = w == 0 ? L.data : v;
    v = w == 1 ? L.data_end : v;
    v = w == 2 ? L.data : v;      // data_meta == data
    v = w == 3 ? L.ingress : v;
    v = w == 4 ? L.rxq : v;
    v = w == 5 ? L.egress : v;
    return v;
}
DEV uint64_t xdp_load(const KParams &kp, const Lane &L, uint32_t o, uint32_t n) {
    if (L.xdp_dirty) return priv_load(kp, L.lane, kp.priv_xdp_q * 8 + o, n);
    uint32_t w0 = o >> 2, sh = (o & 3) * 8;
    uint64_t lo = (uint64_t)xdp_word(L, w0) | ((uint64_t)xdp_word(L, w0 + 1) << 32);
    uint64_t hi = xdp_word(L, w0 + 2);
    uint64_t v = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}
DEV void xdp_store(const KParams &kp, Lane &L, uint32_t o, uint32_t n, uint64_t v) {
    if (!L.xdp_dirty) {
        for (uint32_t w = 0; w < 3; w++) {
            uint64_t q = (uint64_t)xdp_word(L, 2 * w) | ((uint64_t)xdp_word(L, 2 * w + 1) << 32);
            *gp((uint64_t *)priv_b(kp, L.lane, (kp.priv_xdp_q + w) * 8)) = q;
        }
        L.xdp_dirty = 1;
    }
    priv_store(kp, L.lane, kp.priv_xdp_q * 8 + o, n, v);
}

// Spread kernels (MIMIC_SPREAD, jit.cpp analyze_spread) run one vCPU's packets on many lanes:
// exact only while per-CPU map memory is touched by fused counter increments alone.  The
// generator proves that for every access (base provenance: a generic load or store whose base it
// cannot place keeps the program set on one lane per vCPU), so this is an internal assertion of
// that analysis: a generic access that still resolved into per-CPU memory marks the launch, which
// the engine reports as an engine error instead of passing silently.
#ifdef MIMIC_SPREAD
#define SPREAD_GUARD(kp) do { if ((kp).spread_bad) *gp((kp).spread_bad) = 1u; } while (0)
#else
#define SPREAD_GUARD(kp) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
// MemoryController.GetEntry (memory_controller.go:117-145) over the lane's address space
// ---------------------------------------------------------------------------------------
// the static entry holding address a, or -1: the entries are disjoint and sorted by address
// (upload_tables), so a binary search for the last one starting at or below a
DEV int32_t seg_find(const KParams &kp, uint32_t a) {
    uint32_t sl = 0, sr = kp.nsegs;
    while (sl < sr) {
        const uint32_t sm = (sl + sr) >> 1;
        if (cget(kp.segs, sm).lo <= a) sl = sm + 1;
        else sr = sm;
    }
    return sl > 0 && a <= cget(kp.segs, sl - 1).hi ? (int32_t)(sl - 1) : -1;
}

DEV Ref resolve(const KParams &kp, const Lane &L, uint32_t a) {
    Ref R;
    R.rk = RK_UNRES;
    R.off = 0;
    R.limit = 0;
    R.map = -1;
    R.sub = -1;
    R.prog = -1;
    R.ptr = nullptr;
    const uint32_t St = kp.static_next;
    if (a >= St) {
        if (a - St <= kp.stack_size) {
            R.rk = RK_STACK;
            R.off = a - St;
            R.limit = kp.stack_size;
        } else if (CTX_SKB_MODE(kp)) {
            // sk_buff right after the stack; this process's sock / flow keys / packet at its
            // leak position.  Earlier processes' leaked entries are not visible.
            const uint32_t Sk = St + kp.stack_size + 1;
            if (a - Sk <= SKB_STRUCT_SIZE) {
                R.rk = RK_SKB;
                R.off = a - Sk;
                R.limit = SKB_STRUCT_SIZE;
            } else if (L.rec && a - L.ka <= SKB_SK_SIZE) {
                R.rk = RK_SK;
                R.off = a - L.ka;
                R.limit = SKB_SK_SIZE;
            } else if (L.rec && a - (L.ka + SKB_SK_SIZE + 1) <= SKB_FK_SIZE) {
                R.rk = RK_FK;
                R.off = a - (L.ka + SKB_SK_SIZE + 1);
                R.limit = SKB_FK_SIZE;
            } else if (L.rec && a - L.pa <= L.M) {
                R.rk = RK_BEPKT;
                R.ptr = L.pkt;
                R.off = a - L.pa;
                R.limit = L.M;
            }
        } else {
            const uint32_t P = St + kp.stack_size + 1;
            if (a - P <= L.M) {
                R.rk = RK_GLOBAL;
                R.ptr = L.pkt;
                R.off = a - P;
                R.limit = L.M;
            } else {
                const uint32_t X = P + L.M + 1;
                if (a - X <= MIMIC_XDP_MD_SIZE) {
                    R.rk = RK_XDP;
                    R.off = a - X;
                    R.limit = MIMIC_XDP_MD_SIZE;
                }
            }
        }
        return R;
    }
    if (a - L.t_lo < L.t_n) {
        SPREAD_GUARD(kp);   // the translation cache holds a lookup's value region
        R.rk = RK_GLOBAL;
        R.ptr = L.t_ptr;
        R.off = a - L.t_lo;
        R.limit = L.t_n - 1;
        return R;
    }
    const int32_t si = seg_find(kp, a);
    if (si >= 0) {
        const Seg g = cget(kp.segs, (uint32_t)si);
        {
            uint32_t off = a - g.lo;
            switch (g.kind) {
            case SEG_PLAIN:
                R.rk = RK_GLOBAL;
                R.ptr = kp.arena + g.dev_off;
                R.off = off;
                R.limit = g.size;
                break;
            case SEG_ARRAY_OBJ:
                R.map = (int32_t)g.id;
                R.rk = g.datasec ? RK_GLOBAL : RK_NOTDATASEC;
                R.ptr = kp.arena + g.dev_off;
                R.off = off;
                R.limit = g.size;
                break;
            case SEG_MAP_OBJ:
                R.map = (int32_t)g.id;
                R.rk = RK_NOTVMMEM;
                break;
            case SEG_PROG:
                R.prog = (int32_t)g.id;
                R.rk = RK_NOTVMMEM;
                break;
            case SEG_PERCPU_ARRAY: {
                SPREAD_GUARD(kp);
                uint32_t c = off / g.period, r = off - c * g.period;
                R.ptr = kp.arena + g.dev_off + (size_t)c * g.dev_stride;
                R.limit = g.size;
                if (r <= 8) { // the sub-array LinuxArrayMap object of cpu c
                    R.map = (int32_t)g.id;
                    R.sub = (int32_t)c;
                    R.rk = g.datasec ? RK_GLOBAL : RK_NOTDATASEC;
                    R.off = r;
                } else {
                    R.rk = RK_GLOBAL;
                    R.off = r - 9;
                }
                break;
            }
            case SEG_PERCPU_VALUES: {
                SPREAD_GUARD(kp);
                uint32_t c = off / g.period, r = off - c * g.period;
                R.rk = RK_GLOBAL;
                R.ptr = kp.arena + g.dev_off + (size_t)c * g.dev_stride;
                R.off = r;
                R.limit = g.size;
                break;
            }
            default: break;
            }
        }
    }
    return R;
}

DEV bool is_vmmem(uint32_t rk) {
    return rk == RK_STACK || rk == RK_XDP || rk == RK_GLOBAL || rk == RK_NOTDATASEC || rk == RK_SKB || rk == RK_SK ||
           rk == RK_FK || rk == RK_BEPKT;
}

// big-endian scalar of n bytes (binary.BigEndian.Uint16/32/64)
DEV uint64_t bswap_n(uint64_t v, uint32_t n) {
    switch (n) {
    case 2: return __builtin_bswap16((uint16_t)v);
    case 4: return __builtin_bswap32((uint32_t)v);
    case 8: return __builtin_bswap64(v);
    default: return v;
    }
}

// SKBuff / SK / FlowKeys .Load / .Store (convertAccess): no PlainMemory bounds check
DEV int skb_access(const KParams &kp, const Lane &L, const Ref &R, uint32_t n, uint64_t &v, bool load) {
    SkbRes o;
    const mimic_skb_custom *cu = (const mimic_skb_custom *)kp.skb_custom;
    if (R.rk == RK_SKB)
        o = skb_convert(L.rec, cu, kp.skb_ifindex, L.pa + SKB_HEADROOM, L.pa + (L.M - SKB_HEADROOM - SKB_TAILROOM), L.ka,
                        L.ka + SKB_SK_SIZE + 1, R.off, n, v, load);
    else if (R.rk == RK_SK) o = sk_convert(L.rec, cu, R.off, n, v, load);
    else o = fk_convert(L.rec, R.off, n, v, load);
    if (load) v = o.v;
    return o.st;
}

// VMMem.Load/Store after GetEntry (inst.go:298-363): returns 0 or a status
DEV int mem_load(const KParams &kp, const Lane &L, const Ref &R, uint32_t n, uint64_t &v) {
    if (R.rk == RK_UNRES) return MIMIC_ERR_MEM_UNRESOLVED;
    if (R.rk == RK_NOTVMMEM) return MIMIC_ERR_MEM_NOT_VMMEM;
    if (R.rk == RK_NOTDATASEC) return MIMIC_ERR_MEM_NOT_DATASEC;
    if (R.rk == RK_SKB || R.rk == RK_SK || R.rk == RK_FK) return skb_access(kp, L, R, n, v, true);
    if ((uint64_t)R.off + n > R.limit) return MIMIC_ERR_MEM_BOUNDS;
    if (R.rk == RK_STACK) v = stack_load(kp, L, R.off, n);
    else if (R.rk == RK_XDP) v = xdp_load(kp, L, R.off, n);
    else if (R.rk == RK_BEPKT) v = bswap_n(ld_n(R.ptr + R.off, n), n);
    else v = ld_n(R.ptr + R.off, n);
    return 0;
}
// a store into an sk_buff's packet memory outside the JIT's frame-only fast store (jit.cpp: those stay
// inside the frame): the batch's rooms-clean word goes back to 0, so the next launch's prep reads the
// rooms again (skb.hip). Every such store marks, not only the head- / tailroom ones: the room test
// here cost the batch interpreter 14 spilled VGPRs (tests/test_interp_regs.py)
DEV void skb_room_mark(const KParams &kp) {
    if (kp.skb_rooms_state) __hip_atomic_store(kp.skb_rooms_state, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV int mem_store(const KParams &kp, Lane &L, const Ref &R, uint32_t n, uint64_t v) {
    if (R.rk == RK_UNRES) return MIMIC_ERR_MEM_UNRESOLVED;
    if (R.rk == RK_NOTVMMEM) return MIMIC_ERR_MEM_NOT_VMMEM;
    if (R.rk == RK_NOTDATASEC) return MIMIC_ERR_MEM_NOT_DATASEC;
    if (R.rk == RK_SKB || R.rk == RK_SK || R.rk == RK_FK) return skb_access(kp, L, R, n, v, false);
    if ((uint64_t)R.off + n > R.limit) return MIMIC_ERR_MEM_BOUNDS;
    if (R.rk == RK_STACK) stack_store(kp, L, R.off, n, v);
    else if (R.rk == RK_XDP) xdp_store(kp, L, R.off, n, v);
    else if (R.rk == RK_BEPKT) {
        st_n(R.ptr + R.off, n, bswap_n(v, n));
        skb_room_mark(kp);
    } else st_n(R.ptr + R.off, n, v);
    return 0;
}
// VMMem.Read bounds check only (the bytes are consumed by the caller chunk-wise)
DEV bool readable(const Ref &R, uint32_t n) {
    // SKBuff / SK / FlowKeys .Read is "not implemented" (an error)
    if (!(R.rk == RK_STACK || R.rk == RK_XDP || R.rk == RK_GLOBAL || R.rk == RK_BEPKT)) return false;
    return (uint64_t)R.off + n <= R.limit;
}
DEV uint64_t region_load(const KParams &kp, const Lane &L, const Ref &R, uint32_t off, uint32_t n) {
    if (R.rk == RK_STACK) return stack_load(kp, L, off, n);
    if (R.rk == RK_XDP) return xdp_load(kp, L, off, n);
    return ld_n(R.ptr + off, n);
}

// ---------------------------------------------------------------------------------------
// helpers (emulator_linux_helpers.go)
// ---------------------------------------------------------------------------------------

// regToMap, emulator_linux_helpers.go:415-447
DEV bool reg_to_map(const KParams &kp, const Lane &L, uint64_t v, int32_t &map, int32_t &sub) {
    Ref R = resolve(kp, L, (uint32_t)v);
    if (R.rk == RK_UNRES) return false;
    if (R.map >= 0) {
        map = R.map;
        sub = R.sub;
        return true;
    }
    if (is_vmmem(R.rk)) {
        uint64_t a = 0;
        if (mem_load(kp, L, R, 4, a)) return false;
        Ref R2 = resolve(kp, L, (uint32_t)a);
        if (R2.map >= 0) {
            map = R2.map;
            sub = R2.sub;
            return true;
        }
    }
    return false;
}

// array-family value address for key k; sub = concrete cpu sub-array (or -1 for a plain array)
DEV uint32_t array_value_addr(const DMap &m, int32_t sub, uint32_t k) {
    if (k >= m.max_entries) return 0;
    uint32_t base = m.backing_addr + (sub > 0 ? (uint32_t)sub * m.addr_period : 0u);
    return base + k * m.value_size;
}
DEV uint8_t *array_value_ptr(const KParams &kp, const DMap &m, int32_t sub, uint32_t k) {
    return kp.arena + m.dev_off + (sub > 0 ? (size_t)sub * m.dev_stride : 0) + (size_t)k * m.value_size;
}

// lane value cache (vc_load / vc_store above): open the lane's row of per-CPU array m when it
// qualifies, and write it back
DEV void vc_open(const KParams &kp, const DMap &m, int32_t cpu, uint8_t *&p, uint32_t &lo, uint32_t &nb, uint32_t &valid,
                 uint64_t &w0, uint64_t &w1, uint64_t &w2, uint64_t &w3) {
    const uint64_t rb = (uint64_t)m.max_entries * m.value_size;
    if (m.family != FAM_PERCPU_ARRAY || cpu < 0 || (uint32_t)cpu >= m.ncpu || rb == 0 || rb > 32 || (rb & 7)) return;
    uint8_t *q = array_value_ptr(kp, m, cpu, 0);
    if ((uintptr_t)q & 7) return;
    p = q;
    lo = m.backing_addr + (cpu > 0 ? (uint32_t)cpu * m.addr_period : 0u);
    nb = (uint32_t)rb;
    const GAS uint64_t *s = (const GAS uint64_t *)q;
    w0 = s[0];
    if (rb > 8) w1 = s[1];
    if (rb > 16) w2 = s[2];
    if (rb > 24) w3 = s[3];
    valid = 1u;
}
DEV void vc_writeback(uint8_t *p, uint32_t nb, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
    GAS uint64_t *d = (GAS uint64_t *)p;
#ifdef MIMIC_VC_NT   // measurement: the row streamed out (non-temporal stores)
    __builtin_nontemporal_store(w0, d);
    if (nb > 8) __builtin_nontemporal_store(w1, d + 1);
    if (nb > 16) __builtin_nontemporal_store(w2, d + 2);
    if (nb > 24) __builtin_nontemporal_store(w3, d + 3);
#else
    d[0] = w0;
    if (nb > 8) d[1] = w1;
    if (nb > 16) d[2] = w2;
    if (nb > 24) d[3] = w3;
#endif
}

// The LDS form of the lane value cache, for rows of 40..MIMIC_VC_MAX_ROW bytes (jit.cpp vc_lds):
// the lane's row in its LDS slot `c` (dword d at c[d * 256], the block's lanes interleaved, so a
// wave's same-offset access hits 64 consecutive banks).  Same semantics as the register form:
// little-endian like the arena, any size / alignment inside the row.
#define LVC_T 256u
DEV void lvc_open(const KParams &kp, const DMap &m, int32_t cpu, uint32_t rb, uint8_t *&p, uint32_t &lo, uint32_t &valid,
                  uint32_t *c) {
    if (m.family != FAM_PERCPU_ARRAY || cpu < 0 || (uint32_t)cpu >= m.ncpu || (uint64_t)m.max_entries * m.value_size != rb) return;
    uint8_t *q = array_value_ptr(kp, m, cpu, 0);
    if ((uintptr_t)q & 7) return;
    p = q;
    lo = m.backing_addr + (cpu > 0 ? (uint32_t)cpu * m.addr_period : 0u);
    const GAS uint64_t *s = (const GAS uint64_t *)q;
    for (uint32_t w = 0; w < rb / 8; w++) {
        const uint64_t v = s[w];
        c[(2 * w) * LVC_T] = (uint32_t)v;
        c[(2 * w + 1) * LVC_T] = (uint32_t)(v >> 32);
    }
    valid = 1u;
}
DEV void lvc_writeback(uint8_t *p, uint32_t nb, const uint32_t *c) {
    GAS uint64_t *d = (GAS uint64_t *)p;
    for (uint32_t w = 0; w < nb / 8; w++) d[w] = (uint64_t)c[(2 * w) * LVC_T] | ((uint64_t)c[(2 * w + 1) * LVC_T] << 32);
}
DEV uint64_t lvc_load(const uint32_t *c, uint32_t o, uint32_t n) {
    const uint32_t d = o >> 2, sh = (o & 3) * 8;
    uint64_t v = ((uint64_t)c[d * LVC_T] | ((uint64_t)c[(d + 1) * LVC_T] << 32)) >> sh;
    if (sh && 8 * n + sh > 64) v |= (uint64_t)c[(d + 2) * LVC_T] << (64 - sh);
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}
DEV void lvc_store(uint32_t *c, uint32_t o, uint32_t n, uint64_t v) {
    if (!(o & 3) && (n == 4 || n == 8)) {
        c[(o >> 2) * LVC_T] = (uint32_t)v;
        if (n == 8) c[((o >> 2) + 1) * LVC_T] = (uint32_t)(v >> 32);
        return;
    }
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t b = o + k, s = (b & 3) * 8;
        uint32_t &w = c[(b >> 2) * LVC_T];
        w = (w & ~(0xffu << s)) | (((uint32_t)(v >> (8 * k)) & 0xffu) << s);
    }
}
// a fused counter increment (4 or 8 bytes at a 4-byte aligned offset o)
DEV void lvc_add(uint32_t *c, uint32_t o, uint32_t n, uint64_t k) {
    uint32_t *w = c + (o >> 2) * LVC_T;
    if (n == 4) {
        w[0] += (uint32_t)k;
        return;
    }
    const uint64_t x = ((uint64_t)w[0] | ((uint64_t)w[LVC_T] << 32)) + k;
    w[0] = (uint32_t)x;
    w[LVC_T] = (uint32_t)(x >> 32);
}

// memmove of n bytes from a VM region into the arena (map update, emulator_linux_map_array.go:112)
DEV void copy_into(const KParams &kp, const Lane &L, const Ref &src, uint8_t *dst, uint32_t n) {
    bool backward = (src.rk == RK_GLOBAL || src.rk == RK_BEPKT) && src.ptr + src.off < dst && dst < src.ptr + src.off + n;
    if (!backward) {
        for (uint32_t o = 0; o < n; o += 8) {
            uint32_t c = n - o < 8 ? n - o : 8;
            st_n(dst + o, c, region_load(kp, L, src, src.off + o, c));
        }
    } else {
        for (uint32_t e = n; e > 0;) {
            uint32_t c = e < 8 ? e : 8;
            e -= c;
            st_n(dst + e, c, region_load(kp, L, src, src.off + e, c));
        }
    }
}

// hash-map key words: derefMapKey (emulator_linux_helpers.go:449-471) copies the key out of VM
// memory once, into the lane's key scratch in private memory (qword-interleaved like the stack)
struct KeyPriv {
    const uint64_t *p;
    uint32_t stride;
    __device__ uint64_t word(uint32_t q) const { return p[(size_t)q * stride]; }
};
DEV KeyPriv key_fetch(const KParams &kp, const Lane &L, const Ref &R, uint32_t K) {
    uint64_t *p = (uint64_t *)kp.priv + (size_t)kp.priv_key_q * kp.priv_lanes + L.lane;
    for (uint32_t q = 0; q * 8 < K; q++) {
        const uint32_t c = K - q * 8 < 8 ? K - q * 8 : 8;
        p[(size_t)q * kp.priv_lanes] = region_load(kp, L, R, R.off + q * 8, c);
    }
    return KeyPriv{p, kp.priv_lanes};
}
// values[cpu] + idx*S (hash: one values backing; per-CPU hash: cpu-major backings)
DEV uint32_t hash_value_addr(const DMap &m, int32_t cpu, uint32_t idx) {
    return m.backing_addr + (m.family == FAM_PERCPU_HASH ? (uint32_t)cpu * m.addr_period : 0u) + idx * m.value_size;
}
DEV uint8_t *hash_value_ptr(const KParams &kp, const DMap &m, int32_t cpu, uint32_t idx) {
    return kp.arena + m.dev_off + (m.family == FAM_PERCPU_HASH ? (size_t)cpu * m.dev_stride : 0) + (size_t)idx * m.value_size;
}

struct HelperOut {
    int st;          // 0 or status
    uint64_t r0;     // new R0 (if set_r0)
    bool set_r0;
    bool tail;       // tail call taken
    uint32_t new_prog;
    uint32_t t_lo, t_n;  // translation-cache entry for the returned value's region (t_n = 0: none)
    uint8_t *t_ptr;
};

// the map descriptor: scalar loads when every active lane names the same map (the usual case)
DEV DMap load_map(const KParams &kp, int32_t mid) {
    const int32_t m0 = __builtin_amdgcn_readfirstlane(mid);
    if (__ballot(mid != m0) == 0) return cget(kp.maps, (uint32_t)m0);
    return kp.maps[mid];
}

// resolve the concrete array (sub-array) a LinuxMap reference names for this process
// returns 0 ok, or MIMIC_ERR_HELPER_MAP_OP for per-CPU cpuid errors
DEV int array_target(const DMap &m, int32_t sub, int32_t cpu, int32_t &which) {
    if (m.family == FAM_PERCPU_ARRAY && sub < 0) {
        if (cpu < 0 || (uint32_t)cpu >= m.ncpu) return MIMIC_ERR_HELPER_MAP_OP;
        which = cpu;
    } else {
        which = sub;
    }
    return 0;
}

DEV HelperOut helper_lookup(const KParams &kp, const Lane &L, uint64_t r1, uint64_t r2) { // :477-504
    HelperOut o = {0, 0, false, false, 0, 0, 0, nullptr};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = load_map(kp, mid);
    Ref K = resolve(kp, L, (uint32_t)r2);
    if (!readable(K, m.key_size)) { o.st = MIMIC_ERR_HELPER_KEY; return o; }
    if (m.family == FAM_ARRAY || m.family == FAM_PERCPU_ARRAY) {
        int32_t which;
        if (array_target(m, sub, L.cpu, which)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        if (m.key_size != 4) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        uint32_t k = (uint32_t)region_load(kp, L, K, K.off, 4);
        o.r0 = array_value_addr(m, which, k);
        o.set_r0 = true;
        if (o.r0) {  // the values backing of that (sub-)array: [base, base + E*S] (inclusive end)
            o.t_lo = m.backing_addr + (which > 0 ? (uint32_t)which * m.addr_period : 0u);
            o.t_n = m.max_entries * m.value_size + 1;
            o.t_ptr = array_value_ptr(kp, m, which, 0);
        }
        return o;
    }
    // LinuxHashMap.Lookup :134-155 / LinuxPerCPUHashMap.Lookup :537-561
    if (m.family == FAM_PERCPU_HASH && (L.cpu < 0 || (uint32_t)L.cpu >= m.ncpu)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
    const KeyPriv ks = key_fetch(kp, L, K, m.key_size);
    const HT t = h_table(kp.arena, m);
    const uint64_t h = h_hash(ks, m.key_size);
    const int32_t idx = HASH_RO(kp) ? h_find_ro(t, ks, h) : h_find(t, ks, h, nullptr, !HASH_POPONLY(kp));
    o.r0 = idx < 0 ? 0 : hash_value_addr(m, L.cpu, (uint32_t)idx);
    o.set_r0 = true;
    if (idx >= 0) {
        o.t_lo = hash_value_addr(m, L.cpu, 0);
        o.t_n = m.max_entries * m.value_size + 1;
        o.t_ptr = hash_value_ptr(kp, m, L.cpu, 0);
    }
    return o;
}

DEV HelperOut helper_update(const KParams &kp, const Lane &L, uint64_t r1, uint64_t r2, uint64_t r3) { // :506-555
    HelperOut o = {0, 0, false, false, 0, 0, 0, nullptr};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = load_map(kp, mid);
    Ref K = resolve(kp, L, (uint32_t)r2);
    if (!readable(K, m.key_size)) { o.st = MIMIC_ERR_HELPER_KEY; return o; }
    Ref V = resolve(kp, L, (uint32_t)r3);
    if (!readable(V, m.value_size)) { o.st = MIMIC_ERR_HELPER_VALUE; return o; }
    if (m.family == FAM_ARRAY || m.family == FAM_PERCPU_ARRAY) {
        int32_t which;
        if (array_target(m, sub, L.cpu, which)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        if (m.key_size != 4) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        uint32_t k = (uint32_t)region_load(kp, L, K, K.off, 4);
        if (k >= m.max_entries) {
            o.r0 = 7; // syscall.E2BIG returned as uint64(errno) (Q9)
            o.set_r0 = true;
            return o;
        }
        copy_into(kp, L, V, array_value_ptr(kp, m, which, k), m.value_size);
        o.r0 = 0;
        o.set_r0 = true;
        return o;
    }
    // LinuxHashMap.Update :158-203 / LinuxPerCPUHashMap.Update :564-612
    if (m.family == FAM_PERCPU_HASH && (L.cpu < 0 || (uint32_t)L.cpu >= m.ncpu)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
    const KeyPriv ks = key_fetch(kp, L, K, m.key_size);
    const uint64_t h = h_hash(ks, m.key_size);
    const HT t = h_table(kp.arena, m);
    // pop-only launches: h_insert_nolock's own walk finds a present key (no separate probe first)
    const bool nolock = HASH_POPONLY(kp) && MIMIC_HASH_NOLOCK;
    int32_t idx = nolock ? -1 : h_find(t, ks, h, nullptr);
    bool inserted = false;
    if (nolock) {
        idx = h_insert_nolock(t, ks, h, &inserted);
    } else if (idx < 0) {
        // a new key: find-or-insert under its stripe lock, the wave's lanes in lock rounds
        // (with MIMIC_HASH_NOLOCK a pop-only launch never gets here: one locked form, not two, is
        // compiled in -- the interpreter's register budget)
#if MIMIC_HASH_NOLOCK
        idx = h_insert_wave(t, ks, h, &inserted, false);
#else
        idx = HASH_POPONLY(kp) ? h_insert_wave(t, ks, h, &inserted, true) : h_insert_wave(t, ks, h, &inserted, false);
#endif
    }
    if (idx < 0) {
        o.r0 = 7; // syscall.E2BIG: the freelist is empty
        o.set_r0 = true;
        return o;
    }
    if (inserted) { // keys.Write(keyOff, key) (the bytes of a found key are already there)
        uint8_t *kd = kp.arena + m.keys_dev_off + (size_t)idx * m.key_size;
        for (uint32_t q = 0; q * 8 < m.key_size; q++) {
            const uint32_t c = m.key_size - q * 8 < 8 ? m.key_size - q * 8 : 8;
            st_n(kd + q * 8, c, ks.word(q));
        }
    }
    // re-resolved here (pure) so that no Ref stays live across the insert
    copy_into(kp, L, resolve(kp, L, (uint32_t)r3), hash_value_ptr(kp, m, L.cpu, (uint32_t)idx), m.value_size);
    o.r0 = 0;
    o.set_r0 = true;
    return o;
}

DEV HelperOut helper_delete(const KParams &kp, const Lane &L, uint64_t r1, uint64_t r2) { // :557-586
    HelperOut o = {0, 0, false, false, 0, 0, 0, nullptr};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = load_map(kp, mid);
    if (m.family == FAM_ARRAY || m.family == FAM_PERCPU_ARRAY) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
    Ref K = resolve(kp, L, (uint32_t)r2);
    if (!readable(K, m.key_size)) { o.st = MIMIC_ERR_HELPER_KEY; return o; }
    // LinuxHashMap.Delete :225-255 / LinuxPerCPUHashMap.Delete :634-664 (absent key: nil)
    const KeyPriv ks = key_fetch(kp, L, K, m.key_size);
    const uint64_t h = h_hash(ks, m.key_size);
    const HT t = h_table(kp.arena, m);
    h_delete_wave(t, ks, h);
    o.r0 = 0;
    o.set_r0 = true;
    return o;
}

DEV HelperOut helper_tailcall(const KParams &kp, const Lane &L, uint64_t r2, uint64_t r3) { // :649-738
    HelperOut o = {0, 0, false, false, 0, 0, 0, nullptr};
    if (L.tailcalls >= kp.max_tail_calls) {
        o.r0 = (uint64_t)(int64_t)-1; // -EPERM
        o.set_r0 = true;
        return o;
    }
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r2, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = load_map(kp, mid);
    if (m.type != MIMIC_MAP_PROG_ARRAY || m.key_size != 4 || m.family != FAM_ARRAY) {
        o.st = MIMIC_ERR_HELPER_TAILCALL;
        return o;
    }
    uint32_t slot = array_value_addr(m, -1, (uint32_t)r3);
    Ref R = resolve(kp, L, slot);
    if (R.rk == RK_UNRES) {
        o.r0 = (uint64_t)(int64_t)-22; // -EINVAL
        o.set_r0 = true;
        return o;
    }
    if (!is_vmmem(R.rk)) { o.st = MIMIC_ERR_HELPER_TAILCALL; return o; }
    uint64_t pa = 0;
    if (mem_load(kp, L, R, 4, pa)) pa = 0; // the load error is ignored (:707-710)
    Ref P = resolve(kp, L, (uint32_t)pa);
    if (P.prog < 0) {
        o.r0 = (uint64_t)(int64_t)-22;
        o.set_r0 = true;
        return o;
    }
    o.tail = true;
    o.new_prog = (uint32_t)P.prog;
    return o;
}

// emulatedLinuxHelpers classification (emulator_linux_helpers.go:28-204)
DEV int helper_class(int32_t n) {
    // 2 = linuxHelperCantEmulate, 1 = emulated by the reference, 0 = nil
    switch (n) {
    case 4: case 14: case 15: case 16: case 17: case 22: case 24: case 27: case 35: case 36: case 42:
    case 45: case 46: case 47: case 55: case 56: case 67: case 69: case 80: case 112: case 113: case 114:
    case 115: case 119: case 120: case 122: case 123: case 128: case 129: case 141: case 148: case 151:
        return 2;
    case 1: case 2: case 3: case 5: case 7: case 8: case 9: case 12: case 25: case 38: case 65: case 87:
    case 88: case 89: case 125: case 160:
        return 1;
    default:
        return 0;
    }
}

// LD_ABS / LD_IND (LinuxEmulator.CustomInstruction, emulator_linux_.go:198-288): R6 must resolve
// to the *SKBuff entry; R0 = Load(size) at skb.data + x (x = imm, or src + imm for LD_IND) in
// whatever entry that address falls in; then R1-R5 = 0 (done by the caller).  A register
// source > 10 panics after the R6 check (the caller passes bad_src).
DEV int ld_abs(const KParams &kp, const Lane &L, uint64_t r6, uint32_t x, uint32_t n, bool bad_src, uint64_t &v) {
    const Ref S = resolve(kp, L, (uint32_t)r6);
    if (S.rk != RK_SKB) return MIMIC_ERR_LDABS;
    if (bad_src) return MIMIC_PANIC_BADREG;
    const Ref P = resolve(kp, L, L.pa + SKB_HEADROOM + x);
    if (!is_vmmem(P.rk)) return MIMIC_ERR_LDABS;
    const int rc = mem_load(kp, L, P, n, v);
    if (rc == MIMIC_PANIC_SLICE) return rc;   // a Go panic stays a panic
    return rc ? MIMIC_ERR_LDABS : 0;
}

// The packet memory's headroom and tailroom are zero at Load (context_sk_buff.go:110-119).  They
// are read first and written only when some byte is not zero already (a program stored there in
// an earlier run of the buffer, or the caller's bytes): the common case writes nothing, and the
// reads share their lines with the packet's first bytes and travel with the header loads.
DEV void skb_rooms_zero(uint8_t *pkt, uint32_t lw) {
    typedef uint64_t u64x2u __attribute__((ext_vector_type(2), aligned(1)));
    const u64x2u z = {0, 0};
    GAS u64x2u *hw = (GAS u64x2u *)pkt, *tw = (GAS u64x2u *)(pkt + SKB_HEADROOM + lw);
    hw[0] = z;
    hw[1] = z;
    for (uint32_t q = 0; q < SKB_TAILROOM / 16; q++) tw[q] = z;
}
// the rooms flag of a record the prep kernel built (skb.h SKB_DIRTY_Q)
DEV bool skb_rec_dirty(const SkbRec &r) { return r.ip[0].pad[0] != 0; }
DEV void skb_rooms_clear(uint8_t *pkt, uint32_t lw) {
#if defined(MIMIC_ROOMS_MODE) && MIMIC_ROOMS_MODE == 2   // measurement only (MIMIC_JIT_ROOMS=2): rooms untouched
    return;
#endif
    typedef uint64_t u64x2u __attribute__((ext_vector_type(2), aligned(1)));
    const GAS u64x2u *h = (const GAS u64x2u *)pkt, *t = (const GAS u64x2u *)(pkt + SKB_HEADROOM + lw);
    const u64x2u h0 = h[0], h1 = h[1], t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
    const u64x2u o = h0 | h1 | t0 | t1 | t2 | t3;
#if defined(MIMIC_ROOMS_MODE) && MIMIC_ROOMS_MODE == 0   // MIMIC_JIT_ROOMS=0: always written (round 2)
    if (true) {
#else
    if (o.x | o.y) {
#endif
        const u64x2u z = {0, 0};
        GAS u64x2u *hw = (GAS u64x2u *)pkt, *tw = (GAS u64x2u *)(pkt + SKB_HEADROOM + lw);
        hw[0] = z;
        hw[1] = z;
        for (uint32_t q = 0; q < SKB_TAILROOM / 16; q++) tw[q] = z;
    }
}
static_assert(SKB_HEADROOM == 32 && SKB_TAILROOM == 64, "skb_rooms_clear covers 2 + 4 16-byte chunks");

// NewProcess + LinuxContextSKBuff.Load (context_sk_buff.go:42-107) for packet i: the entries
// of the skb.h layout, zeroed headroom / tailroom, R1 = the sk_buff address.  Returns 0 or
// MIMIC_ERR_CTX_LOAD (SKBuffFromBytes failed, or AddEntry ran out of 32-bit address space;
// then the packet memory is left untouched, as the reference never writes it).  When the batch's
// records were not built by the prep kernel (KParams::skb_rec_built == 0: its JIT kernel builds
// them in LDS) the record is built here first, unless `attach_only` (a process the resume kernel
// re-attaches: its record, rooms and packet are what the JIT lane left).
// packet i's leak prefix: within its prep block + the block's offset (skb.hip)
// (the word's top bits are the prep kernel's flags, skb.h SKB_PFX_*)
DEV uint64_t skb_leak_pre(const KParams &kp, uint32_t i) {
    return (kp.skb_prefix[i] & SKB_PFX_MASK) + kp.skb_prefix[kp.n + (i >> SKB_PREP_LOG2)];
}
// DECODE = false: a kernel only ever launched after a full prep (skb_rec_built == 1: the batch
// interpreter and the Step kernel, engine.cpp run_xdp_impl) leaves SKBuffFromBytes out -- inlined it
// is the largest register peak of the interpreter body (22 of its spilled VGPRs)
template <bool DECODE = true>
DEV int skb_load(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, bool attach_only = false) {
    SkbRec *rec = kp.skb_rec + i;
    L.pkt = kp.pkt_data + kp.pkt_off[i];
    const uint64_t pf = kp.skb_rec_built ? kp.skb_prefix[i] : 0ull;
    // a sparse prep (skb_rec_built == 2) left derived words for the frames skb_fast rejects only:
    // the others are decoded here from the packet bytes (the same record)
    if ((!kp.skb_rec_built || (kp.skb_rec_built == 2 && !(pf & SKB_PFX_EXC))) && !attach_only) {
        if (!DECODE) return MIMIC_ERR_ENGINE_HELPER;   // not launched so (engine invariant); loud if it were
        skb_init(SkbBytes{L.pkt + SKB_HEADROOM}, kp.pkt_len[i], *rec);
    } else if (kp.skb_drv && !attach_only)   // the prep kernel's derived words into the record
        for (uint32_t q = 0; q < SKB_DERIVED_Q; q++) ((uint64_t *)rec)[q] = kp.skb_drv[(size_t)i * SKB_DERIVED_Q + q];
    const uint32_t lw = rec->len;
    L.rec = nullptr;
    L.ka = 0;
    L.pa = 0;
    L.M = 0;
    if (lw & SKB_LOAD_FAILED) return MIMIC_ERR_CTX_LOAD;
    const uint64_t ka = *kp.skb_base + skb_leak_pre(kp, i);
    if (ka + SKB_FOOT_FIXED - 1 + lw > 0xffffffffull) return MIMIC_ERR_CTX_LOAD;  // "out of memory"
    if (!attach_only) {   // the writable state at Load (the prep kernel writes the derived words only)
        for (uint32_t q = 0; q < 8; q++) ((uint64_t *)rec)[SKB_DERIVED_Q + q] = skb_writable_word(q);
        skb_apply_custom(*rec, (const mimic_skb_custom *)kp.skb_custom, i);
    }
    L.rec = rec;
    L.ka = (uint32_t)ka;
    L.pa = L.ka + SKB_SK_SIZE + 1 + SKB_FK_SIZE + 1;
    L.M = SKB_HEADROOM + lw + SKB_TAILROOM;
    if (!attach_only) {
        if (!kp.skb_rec_built) skb_rooms_clear(L.pkt, lw);
        else if (pf & SKB_PFX_DIRTY) skb_rooms_zero(L.pkt, lw);
    }
    r1 = kp.static_next + kp.stack_size + 1;
    return 0;
}

// skb_load's tail once the record of packet i is in place (LDS slot d): a user-given sock / flow
// keys, entries, rooms, R1
// dirty: the record's rooms flag (1 / 0), or -1 when no prep kernel looked (read the rooms here)
DEV int skb_attach(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d, uint32_t lw, uint64_t pre, uint64_t base,
                   int dirty) {
    skb_apply_custom(*(SkbRec *)d, (const mimic_skb_custom *)kp.skb_custom, i);
    L.rec = nullptr;
    L.ka = 0;
    L.pa = 0;
    L.M = 0;
    if (lw & SKB_LOAD_FAILED) return MIMIC_ERR_CTX_LOAD;
    const uint64_t ka = base + pre;
    if (ka + SKB_FOOT_FIXED - 1 + lw > 0xffffffffull) return MIMIC_ERR_CTX_LOAD;  // "out of memory"
    L.rec = (SkbRec *)d;
    L.ka = (uint32_t)ka;
    L.pa = L.ka + SKB_SK_SIZE + 1 + SKB_FK_SIZE + 1;
    L.M = SKB_HEADROOM + lw + SKB_TAILROOM;
    if (dirty < 0) skb_rooms_clear(L.pkt, lw);
    else if (dirty) skb_rooms_zero(L.pkt, lw);
    r1 = kp.static_next + kp.stack_size + 1;
    return 0;
}

// skb_load for a JIT kernel that keeps the process's SkbRec in an LDS slot `d`: the record's words,
// the packet offset and the leak prefix are loaded together (one memory round trip, not the
// record length first and the rest after it), then the record goes to LDS.
DEV int skb_load_lds_po(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d, uint64_t po);
DEV int skb_load_lds(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d) {
    return skb_load_lds_po(kp, L, i, r1, d, kp.pkt_off[i]);
}
// the same with packet i's offset given (loaded ahead by the caller)
DEV int skb_load_lds_po(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d, uint64_t po) {
    // the packet's derived words: 96 contiguous bytes of the prep kernel's compact array (consecutive
    // lanes, consecutive records), six 16-byte loads
    typedef uint64_t u64x2a __attribute__((ext_vector_type(2)));
    const GAS u64x2a *s = (const GAS u64x2a *)(kp.skb_drv + (size_t)i * SKB_DERIVED_Q);
    uint64_t w[SKB_DERIVED_Q];
#pragma unroll
    for (uint32_t q = 0; q < SKB_DERIVED_Q / 2; q++) {
        const u64x2a v = s[q];
        w[2 * q] = v.x;
        w[2 * q + 1] = v.y;
    }
    const uint64_t pre = skb_leak_pre(kp, i), base = *kp.skb_base;
#pragma unroll
    for (uint32_t q = 0; q < SKB_DERIVED_Q; q++) d[q] = w[q];
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) d[SKB_DERIVED_Q + q] = skb_writable_word(q);
    L.pkt = kp.pkt_data + po;
#ifdef MIMIC_SKB_ROOMS_CHAIN   // measurement: the rooms read here (engine.cpp skb_prepare)
    return skb_attach(kp, L, i, r1, d, (uint32_t)w[0], pre, base, -1);
#else
    return skb_attach(kp, L, i, r1, d, (uint32_t)w[0], pre, base, (int)((w[SKB_DIRTY_Q] >> SKB_DIRTY_SHIFT) & 1u));
#endif
}

// skb_load for a JIT kernel after a sparse prep (skb_rec_built == 2): the record of a common frame is
// derived here, from the packet's first SKB_WIN bytes, straight into the LDS slot `d` (skb_fast_rec);
// only a frame skb_fast does not take has its derived words in skb_drv (SKB_PFX_EXC).  The prep's
// 96-byte record per packet is neither written nor read back: the header bytes this loads are the
// ones the programs' early loads fetch next.  po / len: packet i's descriptor, pw: its prefix word
// (the caller may have loaded them ahead).
DEV int skb_load_fast(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d, uint64_t po, uint32_t len,
                      uint64_t pw) {
    const uint64_t pre = (pw & SKB_PFX_MASK) + kp.skb_prefix[kp.n + (i >> SKB_PREP_LOG2)], base = *kp.skb_base;
    L.pkt = kp.pkt_data + po;
    typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));   // any pkt_off
    const GAS u32x4u *pk = (const GAS u32x4u *)(L.pkt + SKB_HEADROOM);
    uint32_t w[SKB_WIN / 4];
#pragma unroll
    for (uint32_t c = 0; c < SKB_WIN / 16; c++) {   // chunks that start inside the packet
        u32x4u v = {0u, 0u, 0u, 0u};
        if (16 * c < len) v = pk[c];
        w[4 * c] = v.x;
        w[4 * c + 1] = v.y;
        w[4 * c + 2] = v.z;
        w[4 * c + 3] = v.w;
    }
    uint32_t lw;
    if (pw & SKB_PFX_EXC) {
        typedef uint64_t u64x2a __attribute__((ext_vector_type(2)));
        const GAS u64x2a *s = (const GAS u64x2a *)(kp.skb_drv + (size_t)i * SKB_DERIVED_Q);
        lw = (uint32_t)s[0].x;
#pragma unroll
        for (uint32_t q = 0; q < SKB_DERIVED_Q / 2; q++) {
            const u64x2a v = s[q];
            d[2 * q] = v.x;
            d[2 * q + 1] = v.y;
        }
    } else {
        SkbRec r;
        skb_fast_rec(w, len, r);
        const uint64_t *rw = (const uint64_t *)&r;
#pragma unroll
        for (uint32_t q = 0; q < SKB_DERIVED_Q; q++) d[q] = rw[q];
        lw = len;
    }
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) d[SKB_DERIVED_Q + q] = skb_writable_word(q);
    return skb_attach(kp, L, i, r1, d, lw, pre, base, (pw & SKB_PFX_DIRTY) ? 1 : 0);
}

// skb_load for a JIT kernel that builds the record itself (no prep records: a 160-byte write and
// read per packet less): SKBuffFromBytes over the packet's first bytes staged in the block's LDS
// windows (`win`, SkbWinBytes), straight into the LDS slot `d`
DEV int skb_load_walk(const KParams &kp, Lane &L, uint32_t i, uint64_t &r1, uint64_t *d, uint32_t *win) {
    const uint64_t po = kp.pkt_off[i], pre = skb_leak_pre(kp, i), base = *kp.skb_base;
    const uint32_t len = kp.pkt_len[i];
    L.pkt = kp.pkt_data + po;
    const uint8_t *pkt = L.pkt + SKB_HEADROOM;
    skb_stage<256u>(win, threadIdx.x, pkt, len);
    SkbRec &r = *(SkbRec *)d;
    skb_init(SkbWinBytes<256u>{win, pkt, threadIdx.x}, len, r);
    return skb_attach(kp, L, i, r1, d, r.len, pre, base, -1);
}

// ---------------------------------------------------------------------------------------
// Cold paths of the JIT kernels: real (non-inlined) functions, so that a kernel holds one
// copy of the generic memory controller / helpers instead of one per instruction (hipRTC
// time, instruction cache).  A call site spills the whole process state (lane state and
// r0..r10) into the kernel's Spill record, calls, and reloads all of it: nothing of the
// process is live across the call, so the call's ABI (callee-saved VGPR ranges) does not
// widen the hot path's register allocation.  Results come back through the record.
// ---------------------------------------------------------------------------------------
struct Spill {
    Lane L;
    uint64_t r[11];
    uint64_t v;          // loaded value
    int32_t st;          // 0 or a status
    uint32_t po;         // store: 1 + packet-memory offset when it wrote the packet (window mirror)
    uint32_t tail;       // tail call taken
    uint32_t new_prog;
};
// a fused counter increment (jit.cpp fusable_inc): one atomic add without return, at the scope of
// the lane's own plain accesses (its XCD's L2)
DEV void atomic_add_n(uint8_t *p, uint32_t n, uint64_t v) {
    if (n == 8) __hip_atomic_fetch_add((GAS uint64_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_add((GAS uint32_t *)p, (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The lane-state half of a deferred slow path (jit.cpp, defer mode; the site has stored the
// registers, PC, program and steps, and written back the lane value cache): the LDS copies of
// the process (sk_buff record, stack window) go back to HBM where the interpreter keeps them,
// the dynamic lane state goes into the record, and the record is marked for the resume kernel
// (interp.hip).  The lane then stops: its later packets follow this one on the resume side.
DEV void defer_finish(const KParams &kp, const Lane &L, uint32_t g, uint32_t i, uint32_t j, uint64_t lane_steps) {
    DeferRec *d = kp.defer + g;
    if (L.rec && L.rec != kp.skb_rec + i) {   // the sk_buff record's LDS slot
        const uint64_t *s = (const uint64_t *)L.rec;
        GAS uint64_t *o = (GAS uint64_t *)(kp.skb_rec + i);
        for (uint32_t q = 0; q < sizeof(SkbRec) / 8; q++) o[q] = s[q];
    }
#ifdef MIMIC_LDS_STACK_Q
    for (uint32_t q = 0; q < MIMIC_LDS_STACK_Q; q++) {
        const uint32_t o = STK_LDS_LO + 8u * q;
        if (stk_valid(kp, L, o)) *gp((uint64_t *)priv_b(kp, L.lane, o)) = stk_lw(o);
    }
#endif
    d->sm0 = SM0(L);
    d->sm1 = SM1(L);
    d->xdp_dirty = L.xdp_dirty;
    d->nframes = L.nframes;
    d->tailcalls = L.tailcalls;
    d->j = j;
    d->lane_steps = lane_steps;
    d->flag = kp.defer_epoch;
    *gp(kp.defer_any) = kp.defer_epoch;
}

#if defined(MIMIC_COLD_INLINE) && MIMIC_COLD_INLINE
#define COLD DEV
#define COLD_OPAQUE() do { } while (0)
#else
#define COLD static __device__ __attribute__((noinline, cold))
// the callee is opaque to the caller's alias analysis: the record is always re-read
#define COLD_OPAQUE() asm volatile("" ::: "memory")
#endif
// GetEntry + VMMem.Load (inst.go:298-318)
COLD void cold_load(const KParams &kp, Spill &S, uint32_t a, uint32_t n) {
    COLD_OPAQUE();
    S.v = 0;
    S.st = mem_load(kp, S.L, resolve(kp, S.L, a), n, S.v);
}
// GetEntry + VMMem.Store (inst.go:320-363); may set S.L.sm0 / sm1 / xdp_dirty
COLD void cold_store(const KParams &kp, Spill &S, uint32_t a, uint32_t n, uint64_t v) {
    COLD_OPAQUE();
    const Ref R = resolve(kp, S.L, a);
    S.st = mem_store(kp, S.L, R, n, v);
    S.po = (!S.st && R.ptr == S.L.pkt && (R.rk == RK_GLOBAL || R.rk == RK_BEPKT)) ? R.off + 1 : 0;
}
DEV void cold_take(Spill &S, const HelperOut &ho) {
    S.st = ho.st;
    if (!ho.st && ho.set_r0) S.r[0] = ho.r0;
}
COLD void cold_lookup(const KParams &kp, Spill &S) {
    COLD_OPAQUE();
    const HelperOut ho = helper_lookup(kp, S.L, S.r[1], S.r[2]);
    cold_take(S, ho);
    if (!ho.st && ho.t_n) {
        S.L.t_lo = ho.t_lo;
        S.L.t_n = ho.t_n;
        S.L.t_ptr = ho.t_ptr;
    }
}
COLD void cold_update(const KParams &kp, Spill &S) {
    COLD_OPAQUE();
    cold_take(S, helper_update(kp, S.L, S.r[1], S.r[2], S.r[3]));
}
COLD void cold_delete(const KParams &kp, Spill &S) {
    COLD_OPAQUE();
    cold_take(S, helper_delete(kp, S.L, S.r[1], S.r[2]));
}
COLD void cold_tailcall(const KParams &kp, Spill &S) {
    COLD_OPAQUE();
    const HelperOut ho = helper_tailcall(kp, S.L, S.r[2], S.r[3]);
    cold_take(S, ho);
    S.tail = !ho.st && ho.tail;
    S.new_prog = ho.new_prog;
}
// LD_ABS / LD_IND through the generic path (emulator_linux_.go:198-288): R0, then R1-R5 = 0
COLD void cold_ldabs(const KParams &kp, Spill &S, uint32_t x, uint32_t n, bool bad_src) {
    COLD_OPAQUE();
    uint64_t v = 0;
    S.st = ld_abs(kp, S.L, S.r[6], x, n, bad_src, v);
    if (!S.st) {
        S.r[0] = v;
        for (int q = 1; q <= 5; q++) S.r[q] = 0;
    }
}
// bpf_xdp_adjust_tail (emulator_linux_helpers.go:842-864): R0 = -EINVAL, or a status
COLD void cold_adjust_tail(const KParams &kp, Spill &S) {
    COLD_OPAQUE();
    const Ref R = resolve(kp, S.L, (uint32_t)S.r[1]);
    S.st = ((R.rk == RK_GLOBAL || R.rk == RK_STACK) && R.map < 0 && R.limit == 20) ? MIMIC_ERR_ENGINE_HELPER : 0;
    if (!S.st) S.r[0] = (uint64_t)(int64_t)-22;
}

// Inline form of helper 1 (map_lookup_elem, emulator_linux_helpers.go:477-504) for the usual
// case: R1 is exactly the object of array / per-CPU array map `mid` (a hint from the LD_IMM64
// slot that set R1; checked here, so a wrong hint only costs the slow path) and the 4-byte
// key lies on the stack.  Then regToMap, derefMapKey and LinuxArrayMap.Lookup reduce to the
// lines below.  Returns false when the case does not apply (the caller runs cold_lookup).
// fwd_key: the key's 4 bytes when the JIT knows them from a store earlier in the basic block
// (the stack store itself is still made; the lookup just does not wait for it to read it back)
DEV bool lookup_fast_k(const KParams &kp, Lane &L, uint32_t mid, uint64_t r1, uint64_t r2, uint64_t &r0, bool fwd,
                       uint32_t fwd_key) {
    const DMap m = cget(kp.maps, mid);
    if ((uint32_t)r1 != m.obj_addr || m.key_size != 4) return false;
    if (m.family != FAM_ARRAY && m.family != FAM_PERCPU_ARRAY) return false;
    const uint32_t ko = (uint32_t)r2 - kp.static_next;
    if ((uint64_t)ko + 4 > kp.stack_size) return false;
    int32_t which = -1;
    if (m.family == FAM_PERCPU_ARRAY) {
        if (L.cpu < 0 || (uint32_t)L.cpu >= m.ncpu) return false;   // error path: cold
        which = L.cpu;
    }
    const uint32_t k = fwd ? fwd_key : (uint32_t)stack_load(kp, L, ko, 4);
    r0 = array_value_addr(m, which, k);
    if (r0) {
        L.t_lo = m.backing_addr + (which > 0 ? (uint32_t)which * m.addr_period : 0u);
        L.t_n = m.max_entries * m.value_size + 1;
        L.t_ptr = array_value_ptr(kp, m, which, 0);
    }
    return true;
}
DEV bool lookup_fast(const KParams &kp, Lane &L, uint32_t mid, uint64_t r1, uint64_t r2, uint64_t &r0) {
    return lookup_fast_k(kp, L, mid, r1, r2, r0, false, 0);
}

// key words of a hash-map key held in registers (h_hash / h_key_eq read them repeatedly)
struct KeyRegs {
    uint64_t w0, w1, w2, w3;
    __device__ uint64_t word(uint32_t q) const { return q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3; }
};
// Inline form of helper 1 for hash / per-CPU hash maps (LinuxHashMap.Lookup :134-155,
// LinuxPerCPUHashMap.Lookup :537-561): R1 is exactly the map object `mid` hints, the key (at
// most 32 bytes) lies on the stack.  Then regToMap and derefMapKey reduce to reading the key
// words off the stack (unwritten bytes read as zero, as stack_load does), and the lookup is the
// lock-free probe of hashmap.h.  Returns false when the case does not apply (cold_lookup).
DEV bool hash_lookup_fast(const KParams &kp, Lane &L, uint32_t mid, uint64_t r1, uint64_t r2, uint64_t &r0) {
    const DMap m = cget(kp.maps, mid);
    if ((uint32_t)r1 != m.obj_addr || (m.family != FAM_HASH && m.family != FAM_PERCPU_HASH) || m.key_size == 0 ||
        m.key_size > 32)
        return false;
    if (m.family == FAM_PERCPU_HASH && (L.cpu < 0 || (uint32_t)L.cpu >= m.ncpu)) return false;   // error path: cold
    const uint32_t K = m.key_size, ko = (uint32_t)r2 - kp.static_next;
    if ((uint64_t)ko + K > kp.stack_size) return false;
    KeyRegs ks;
    ks.w0 = stack_load(kp, L, ko, K < 8 ? K : 8);
    ks.w1 = K > 8 ? stack_load(kp, L, ko + 8, K - 8 < 8 ? K - 8 : 8) : 0;
    ks.w2 = K > 16 ? stack_load(kp, L, ko + 16, K - 16 < 8 ? K - 16 : 8) : 0;
    ks.w3 = K > 24 ? stack_load(kp, L, ko + 24, K - 24) : 0;
    const HT t = h_table(kp.arena, m);
    const uint64_t h = h_hash(ks, K);
    const int32_t idx = HASH_RO(kp) ? h_find_ro(t, ks, h) : h_find(t, ks, h, nullptr, !HASH_POPONLY(kp));
    r0 = idx < 0 ? 0 : hash_value_addr(m, L.cpu, (uint32_t)idx);
    if (idx >= 0) {
        L.t_lo = hash_value_addr(m, L.cpu, 0);
        L.t_n = m.max_entries * m.value_size + 1;
        L.t_ptr = hash_value_ptr(kp, m, L.cpu, 0);
    }
    return true;
}

// Inline form of helper 12 (tail_call, emulator_linux_helpers.go:649-738) for the usual case: R2
// is exactly the object of prog-array map `mid` (the LD_IMM64 hint, checked here) and R3 indexes
// one of its slots.  Returns the program to continue in; -1 when the call fails (R0 set as the
// helper sets it: the tail-call budget is spent, or the slot holds no program); -2 when the
// generic path has to decide (cold_tailcall).  helper_tailcall's steps reduce to these for
// that case: regToMap finds the map object, the slot's first 4 bytes are the program address,
// and resolving it finds a program entry or not.
DEV int tail_fast(const KParams &kp, const Lane &L, uint32_t mid, uint64_t r2, uint64_t r3, uint64_t &r0) {
    if (L.tailcalls >= kp.max_tail_calls) {
        r0 = (uint64_t)(int64_t)-1;   // -EPERM
        return -1;
    }
    const DMap m = cget(kp.maps, mid);
    if (r2 != (uint64_t)m.obj_addr || m.type != MIMIC_MAP_PROG_ARRAY || m.key_size != 4 || m.family != FAM_ARRAY ||
        m.value_size < 4 || (uint32_t)r3 >= m.max_entries)
        return -2;
    const uint32_t pa = *(const GAS u32u *)array_value_ptr(kp, m, -1, (uint32_t)r3);
    if (kp.nprogs <= 16) {   // program entries [addr, addr + 8]: compare against each (uniform loads)
        for (uint32_t k = 0; k < kp.nprogs; k++)
            if (pa - cget(kp.progs, k).addr <= 8u) return (int)k;
        r0 = (uint64_t)(int64_t)-22;  // -EINVAL
        return -1;
    }
    const int32_t si = seg_find(kp, pa);
    if (si < 0 || cget(kp.segs, (uint32_t)si).kind != SEG_PROG) {
        r0 = (uint64_t)(int64_t)-22;  // -EINVAL
        return -1;
    }
    return (int)cget(kp.segs, (uint32_t)si).id;
}

// ---------------------------------------------------------------------------------------
// wave-wide minimum of a 32-bit key: DPP within each 16-lane row, then 4 readlanes
// ---------------------------------------------------------------------------------------
DEV uint32_t dpp_min(uint32_t v, int ctrl) {
    uint32_t o;
    switch (ctrl) {
    case 0: o = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0xb1, 0xf, 0xf, false); break;
    case 1: o = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x4e, 0xf, 0xf, false); break;
    case 2: o = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x141, 0xf, 0xf, false); break;
    default: o = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x140, 0xf, 0xf, false); break;
    }
    return v < o ? v : o;
}
DEV uint32_t wave_min(uint32_t v) {
    v = dpp_min(v, 0); // quad_perm [1,0,3,2]
    v = dpp_min(v, 1); // quad_perm [2,3,0,1]
    v = dpp_min(v, 2); // row_half_mirror
    v = dpp_min(v, 3); // row_mirror
    uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    a = a < b ? a : b;
    c = c < d ? c : d;
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(a < c ? a : c));  // provably wave-uniform
}

// ---------------------------------------------------------------------------------------
// conditional jumps (inst_gen.go:227-605, inst.go:205-241)
// ---------------------------------------------------------------------------------------
DEV bool jcond(uint32_t jop, uint64_t d, uint64_t s, bool w32) {
    if (w32) {
        uint32_t a = (uint32_t)d, b = (uint32_t)s;
        int32_t sa = (int32_t)a, sb = (int32_t)b;
        switch (jop) {
        case 0x10: return a == b;
        case 0x20: return a > b;
        case 0x30: return a >= b;
        case 0x40: return (a & b) == 0; // Q3 inverted JSET
        case 0x50: return a != b;
        case 0x60: return sa > sb;
        case 0x70: return sa >= sb;
        case 0xa0: return a < b;
        case 0xb0: return a <= b;
        case 0xc0: return sa < sb;
        default: return sa <= sb; // 0xd0
        }
    }
    int64_t sa = (int64_t)d, sb = (int64_t)s;
    switch (jop) {
    case 0x10: return d == s;
    case 0x20: return d > s;
    case 0x30: return d >= s;
    case 0x40: return (d & s) == 0;
    case 0x50: return d != s;
    case 0x60: return sa > sb;
    case 0x70: return sa >= sb;
    case 0xa0: return d < s;
    case 0xb0: return d <= s;
    case 0xc0: return sa < sb;
    default: return sa <= sb;
    }
}

DEV bool is_cond_jop(uint32_t jop) {
    switch (jop) {
    case 0x10: case 0x20: case 0x30: case 0x40: case 0x50: case 0x60: case 0x70:
    case 0xa0: case 0xb0: case 0xc0: case 0xd0:
        return true;
    default:
        return false;
    }
}

DEV uint32_t size_bytes(uint32_t op) {
    switch (op & 0x18) {
    case 0x00: return 4;
    case 0x08: return 2;
    case 0x10: return 1;
    default: return 8;
    }
}

// ---------------------------------------------------------------------------------------
// fast ALU ops (inst_gen.go:7-225, inst.go:86-136); the host only routes valid forms here
// ---------------------------------------------------------------------------------------
DEV uint64_t alu64(uint32_t hi, uint64_t d, uint64_t x) {
    switch (hi) {
    case 0x00: return d + x;
    case 0x10: return d - x;
    case 0x20: return d * x;
    case 0x30: return d / x;   // K form, x != 0 (predecoded)
    case 0x40: return d | x;
    case 0x50: return d & x;
    case 0x60: return x >= 64 ? 0 : d << x;
    case 0x70: return x >= 64 ? 0 : d >> x;
    case 0x80: return (uint64_t)(-(int64_t)d);
    case 0x90: return d % x;
    case 0xa0: return d ^ x;
    case 0xb0: return x;
    default: { // 0xc0 ARSH (x >= 0)
        const int64_t a = (int64_t)d;
        return (uint64_t)(x >= 64 ? (a < 0 ? -1 : 0) : (a >> x));
    }
    }
}
DEV uint64_t alu32(uint32_t hi, uint64_t d, uint64_t x) {
    const uint32_t a = (uint32_t)d, b = (uint32_t)x;
    switch (hi) {
    case 0x00: return (uint32_t)(a + b);
    case 0x10: return (uint32_t)(a - b);
    case 0x20: return (uint32_t)(a * b);
    case 0x30: return a / b;
    case 0x40: return a | b;
    case 0x50: return a & b;
    case 0x60: return b >= 32 ? 0 : (uint32_t)(a << b);
    case 0x70: return b >= 32 ? 0 : a >> b;
    case 0x80: return (uint64_t)(int64_t)(int32_t)(0u - a);          // Q6: sign-extends
    case 0x90: return a % b;
    case 0xa0: return a ^ b;
    case 0xb0: return b;
    default: { // ARSH: the 64-bit shift count is not truncated; result sign-extends (Q5/Q6)
        const int32_t sa = (int32_t)a;
        return (uint64_t)(int64_t)(x >= 32 ? (sa < 0 ? -1 : 0) : (sa >> x));
    }
    }
}


// ---------------------------------------------------------------------------------------
// JIT packet window: the first bytes of each lane's packet memory staged in LDS, qword-
// interleaved across the block's lanes ([q][lane]: uniform offsets are conflict-free).  The
// window is a copy of global packet memory: every packet store updates both.
// ---------------------------------------------------------------------------------------
#define PWIN_Q 8u        // qwords per lane (64 bytes)
#define PWIN_LANES 256u  // block size
typedef uint64_t PWin[PWIN_Q][PWIN_LANES];

// stage pkt[0, W) with W = min(M, 64) rounded down to whole qwords; returns W
DEV uint32_t win_stage(PWin &w, uint32_t tl, const uint8_t *pkt, uint32_t M) {
    const uint32_t W = M >= PWIN_Q * 8 ? PWIN_Q * 8 : (M & ~7u);
#pragma unroll
    for (uint32_t q = 0; q < PWIN_Q; q++)
        if (q * 8 < W) w[q][tl] = *(const GAS u64u *)(pkt + q * 8);
    return W;
}
// n bytes at offset o, o + n <= W
DEV uint64_t win_load(const PWin &w, uint32_t tl, uint32_t o, uint32_t n) {
    const uint32_t q = o >> 3, sh = (o & 7) * 8;
    uint64_t v = w[q][tl] >> sh;
    if (sh + 8 * n > 64) v |= w[q + 1][tl] << (64 - sh);
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}
// mirror a packet store of n bytes at offset o (o < W) into the window
DEV void win_store(PWin &w, uint32_t tl, uint32_t W, uint32_t o, uint32_t n, uint64_t v) {
    const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
    v &= m;
    const uint32_t q = o >> 3, sh = (o & 7) * 8;
    w[q][tl] = (w[q][tl] & ~(m << sh)) | (v << sh);
    if (sh + 8 * n > 64 && (q + 1) * 8 < W) {
        const uint32_t bits = sh + 8 * n - 64;
        const uint64_t m1 = (1ull << bits) - 1;
        w[q + 1][tl] = (w[q + 1][tl] & ~m1) | (v >> (64 - sh));
    }
}
// mirror a packet store of n bytes at packet-memory offset o into a window that covers packet
// memory [wb, wb + W): the part of the store that overlaps the window, if any
DEV void win_store_rel(PWin &w, uint32_t tl, uint32_t W, uint32_t o, uint32_t wb, uint32_t n, uint64_t v) {
    if (o >= wb) {
        if (o - wb < W) win_store(w, tl, W, o - wb, n, v);
    } else if (o + n > wb && W > 0) {
        const uint32_t d = wb - o;
        win_store(w, tl, W, 0, n - d, v >> (8 * d));
    }
}
