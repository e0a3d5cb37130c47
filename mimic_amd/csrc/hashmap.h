// hashmap.h -- device side of LinuxHashMap / LinuxPerCPUHashMap (emulator_linux_map_hash.go).
//
// The reference keeps, per map: a keys backing and a values backing (E slots each, VM
// memory), a Go map sha256(key) -> slot, and a FIFO freelist of slots (a buffered channel
// holding 0..E-1 initially, :56-64).  A new key takes the slot at the head of the freelist
// (:179-186); Delete returns the slot to the tail (:244-250); a full freelist is E2BIG.
//
// Here the Go map becomes an open-addressing table in HBM that every lane of every wave can
// use concurrently:
//   * bucket record = one u64 word (tag<<32 | state) + the key in ceil(K/8) u64 words;
//     state is a slot index, HT_EMPTY, HT_TOMB (deleted) or HT_BUSY (being filled);
//   * lookups are lock-free: probe from the home bucket until EMPTY, compare the tag, then the
//     key words, then re-read the state word (a concurrent delete+reuse shows up there);
//   * inserts and deletes take a stripe lock chosen by the key's home bucket, so two lanes can
//     never insert the same key twice; a wave runs its inserting lanes one at a time;
//   * the freelist is a ring of 2^k >= 2(E+1) entries with agent-scope head/tail/avail
//     counters.  Popped positions are reset to -1, and a push waits for its position to be
//     free again, so FIFO order is the reference's whenever operations are sequential;
//   * everything shared between lanes of different XCDs (state words, key words, ring,
//     counters) is accessed with agent-scope atomics or sc1 loads/stores.  Per-XCD L2s are not
//     coherent, so plain accesses would be wrong here.
// The map values themselves are plain VM memory.  Concurrent vCPUs writing one shared map race
// on them exactly as the reference's processPool workers do.  Host map operations (LinuxMap.Update
// / Lookup / Delete from the API) run the sequential form of the same algorithm on a host image
// of this index (engine.cpp HashMirror), which is uploaded before the device next uses the map.
#pragma once
#include "layout.h"

#define HDEV static __device__ __forceinline__
#define HHD static __host__ __device__ __forceinline__   // also the host mirror's (engine.cpp)

HDEV uint64_t h_ld(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
HDEV void h_st(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
HDEV bool h_cas(uint64_t *p, uint64_t expect, uint64_t want) {
    return __hip_atomic_compare_exchange_strong(p, &expect, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
HDEV void h_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// the index region of one map: [records | rebuild copy | locks | freelist ring | HashCtl]
struct HT {
    uint8_t *base;
    uint32_t cap, rec_q, K, nlocks, fl_cap, E;
    uint32_t tag;   // nonzero per map: which block combiner (below) is this map's
    uint32_t flags; // DMap::hflags (HT_F_CHUNK)
};
HDEV HT h_table(uint8_t *arena, const DMap &m) {
    return HT{arena + m.ht_dev_off, m.ht_cap, m.rec_q, m.key_size, m.nlocks, m.fl_cap, m.max_entries,
              (uint32_t)(m.ht_dev_off >> 3) | 1u, m.hflags};
}

#ifdef MIMIC_HASH_COMBINE
// Block combining of freelist reservations (pop-only launches of JIT kernels that run their
// inserts inline).  Every inserting wave-round of the GPU reserves its positions with one
// agent-scope add to the map's `head`; those same-address atomics serialise at the memory side
// (cfg 4's inserting launch: 0.42 ms, 0.32 ms with the add spread over 16 addresses).  Here the
// waves of a block that reserve at about the same time share one add: the first to arrive opens a
// batch (`word`: generation << 40 | waves joined << 32 | positions requested so far; a slot's
// ready word carries the generation mod 2^23, so a block may run up to 2^23 batches per launch --
// the combiner is zeroed by every launch), waits ~128
// cycles for others to add their counts, closes it, reserves the total with one add and publishes
// base and count in the batch's slot (generation mod 16); the others take their share at the offset
// their add returned.  The batch's positions are contiguous and ordered by arrival -- a valid order
// of pops, as if those waves had popped one after another -- and a lone wave gets exactly what a
// direct add gives (FIFO slots of sequential runs unchanged).
// Slot reuse (round 6): every batch publishes, joiners or not, and its ready word is
// (generation + 1) << 8 | joiners yet to read.  The opener of generation g claims its slot with a
// CAS from exactly "generation g - 16, no reader left" (0 for g < 16) to "g, being written" (low
// byte 0xff), writes base / got and then stores "g, joiners"; each joiner waits for "g" with a
// count below 0xff, reads, and decrements.  So a slot is never overwritten before every joiner of
// its previous batch read it, and a late publication of g - 16 cannot overwrite g's.  Nothing waits
// on a later generation, so the protocol cannot deadlock; a spin still gives up after
// HCOMB_SPIN_LIMIT sleeps, marks HashCtl::comb_fault (the host reports the launch as failed at the
// next sync) and returns no position, rather than hang.
// (Per-wave mailboxes written in a loop by the opener, round 5's first fix, cost the cfg-4 kernel 8
// more spilled VGPRs and its lookup-hit launch 0.126 -> 0.143 ms.)
#define HCOMB_MAPS 4u
#define HCOMB_SLOTS 16u
struct HComb {
    unsigned long long word;
    uint32_t owner;                     // the map (HT::tag) this combiner serves in this block
    uint32_t ready[HCOMB_SLOTS];        // (generation + 1) << 8 | joiners yet to read (0xff: being written)
    uint32_t got[HCOMB_SLOTS];          // positions below tail (bit 31: tail == E, the ring untouched)
    unsigned long long base[HCOMB_SLOTS];
};
static __shared__ HComb h_comb_[HCOMB_MAPS];
// zeroed by every thread of the block before any of them can insert (the JIT prologue)
HDEV void h_comb_init() {
    uint32_t *w = (uint32_t *)h_comb_;
    for (uint32_t q = threadIdx.x; q < sizeof(h_comb_) / 4; q += blockDim.x) w[q] = 0;
    __syncthreads();
}
#ifndef HCOMB_SPIN_LIMIT
#define HCOMB_SPIN_LIMIT (1u << 22)
#endif
HDEV void h_comb_fault(HashCtl *c) { __hip_atomic_store(&c->comb_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// k (>= 1) positions for the calling wave (one lane): *base, *got (positions below tail), *ident
HDEV bool h_comb_reserve(const HT &t, HashCtl *c, uint32_t k, uint64_t *base, uint32_t *got, uint32_t *ident) {
    HComb &cb = h_comb_[(t.tag >> 4) & (HCOMB_MAPS - 1)];
    uint32_t own = __hip_atomic_load(&cb.owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (own == 0) {
        uint32_t z = 0;
        __hip_atomic_compare_exchange_strong(&cb.owner, &z, t.tag, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        own = __hip_atomic_load(&cb.owner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (own != t.tag) return false;   // another map holds this combiner: reserve directly
    const unsigned long long old = __hip_atomic_fetch_add(&cb.word, (1ull << 32) + k, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t gen = (uint32_t)(old >> 40), off = (uint32_t)old, s = gen & (HCOMB_SLOTS - 1);
    const uint32_t mine = ((gen & 0x7fffffu) + 1u) << 8;   // this batch's ready word, reader count 0
    uint64_t b0;
    uint32_t g0;
    uint32_t spins = 0;
    if (((old >> 32) & 0xffu) == 0) {   // the batch's opener
#ifndef MIMIC_HCOMB_SLEEP
#define MIMIC_HCOMB_SLEEP 2
#endif
        __builtin_amdgcn_s_sleep(MIMIC_HCOMB_SLEEP);
        const unsigned long long closed = __hip_atomic_exchange(&cb.word, (unsigned long long)((gen + 1u) & 0xffffffu) << 40,
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t total = (uint32_t)closed, joiners = ((uint32_t)(closed >> 32) & 0xffu) - 1u;
        b0 = __hip_atomic_fetch_add(&c->head, (unsigned long long)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long tl = __hip_atomic_load(&c->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g0 = (b0 >= tl ? 0u : (tl - b0 < total ? (uint32_t)(tl - b0) : total)) | (tl == t.E ? 0x80000000u : 0u);
        // the slot: published by the batch 16 generations earlier and read by all its joiners
        const uint32_t prev = gen < HCOMB_SLOTS ? 0u : (((gen - HCOMB_SLOTS) & 0x7fffffu) + 1u) << 8;
        for (;;) {
            uint32_t e = prev;
            if (__hip_atomic_compare_exchange_strong(&cb.ready[s], &e, mine | 0xffu, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP))
                break;
            if (++spins > HCOMB_SPIN_LIMIT) {
                h_comb_fault(c);
                *base = 0;
                *got = 0;
                *ident = 0;
                return true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        cb.base[s] = b0;
        cb.got[s] = g0;
        __hip_atomic_store(&cb.ready[s], mine | joiners, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        for (;;) {
            const uint32_t r = __hip_atomic_load(&cb.ready[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((r & ~0xffu) == mine && (r & 0xffu) != 0xffu) break;
            if (++spins > HCOMB_SPIN_LIMIT) {
                h_comb_fault(c);
                *base = 0;
                *got = 0;
                *ident = 0;
                return true;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        b0 = cb.base[s];
        g0 = cb.got[s];
        __hip_atomic_fetch_sub(&cb.ready[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    *ident = g0 >> 31;
    g0 &= 0x7fffffffu;
    *base = b0 + off;
    *got = g0 > off ? (g0 - off < k ? g0 - off : k) : 0u;
    return true;
}
#endif
HDEV size_t h_rec_bytes(const HT &t) { return (size_t)t.cap * t.rec_q * 8; }
HDEV uint64_t *h_rec(const HT &t, uint32_t p) { return (uint64_t *)t.base + (size_t)p * t.rec_q; }
HDEV uint64_t *h_tmp(const HT &t) { return (uint64_t *)(t.base + h_rec_bytes(t)); }
HDEV uint32_t *h_locks(const HT &t) { return (uint32_t *)(t.base + 2 * h_rec_bytes(t)); }
HDEV int32_t *h_ring(const HT &t) { return (int32_t *)(h_locks(t) + t.nlocks); }
HDEV HashCtl *h_ctl(const HT &t) {   // 128-byte aligned after the ring (engine.cpp: ctl_off)
    return (HashCtl *)(((uintptr_t)(h_ring(t) + t.fl_cap) + 127) & ~(uintptr_t)127);
}
// after HashCtl (layout.h ht_ext_bytes): a used byte per slot, slot -> bucket, the blocks' handed-back
// remainders
HDEV uint64_t h_e32(const HT &t) { return ((uint64_t)t.E + 1023) & ~1023ull; }
HDEV uint8_t *h_used8(const HT &t) { return (uint8_t *)h_ctl(t) + sizeof(HashCtl); }
HDEV uint32_t *h_s2b(const HT &t) { return (uint32_t *)(h_used8(t) + h_e32(t)); }
HDEV unsigned long long *h_left(const HT &t) { return (unsigned long long *)(h_s2b(t) + h_e32(t)); }
HDEV uint32_t *h_used_shard(HashCtl *c) {   // the calling wave's shard of the `used` count
    const uint32_t w = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (HT_USED_SHARDS - 1);
    return &c->used_sh[32 * w];
}
HDEV uint32_t h_used_total(const HashCtl *c) {
    uint32_t u = c->used0;
    for (uint32_t s = 0; s < HT_USED_SHARDS; s++) u += c->used_sh[32 * s];
    return u;
}

#ifdef MIMIC_HASH_CHUNK
// Chunked reservations (round 6).  The VM's chunk map (HT_F_CHUNK, one per VM)
// in a pop-only JIT launch whose ring is still the identity (tail == E: nothing was ever pushed,
// so ring position p holds slot p): a block takes freelist positions from `head` in chunks of up to
// MIMIC_HCHUNK with one agent-scope add (cfg 4 made ~60 K same-address adds per launch, one per
// inserting wave-round: they serialise at the memory side), and its waves take from the chunk with
// LDS atomics.  A remainder a block leaves is a hole below head; mimic_hash_compact_kernel, launched
// after every such launch, moves the entries above the holes into them, so after the launch the used
// slots are again exactly [0, m) -- ring positions 0..m-1 popped, as m sequential pops leave them.
// (Which key got which slot inside one concurrent launch already depends on arrival order.)
//
// E2BIG stays exact.  An insert is refused only when every position is live: once head has reached
// tail a block ("scarce") takes positions from the remainders finished blocks handed back (left[],
// h_chunk_fini), and refuses only after proving live == E from the live counts (the positions below
// this launch's first reservation, found in the ring, plus what every block gave to inserts: blocks
// add their LDS count to live_sh when they go scarce and when they finish).  Otherwise its lanes
// wait (no bucket held) for running blocks to finish and hand their remainders back.  A block never
// waits while it holds positions (its chunk is empty when it is scarce), and a non-scarce block never
// waits on another block, so the wait ends; it is bounded anyway (HCHUNK_SPIN_LIMIT rounds, then
// comb_fault: the sync reports an engine error).  Chunk sizes shrink as the table fills (the
// remaining positions / (2 * blocks)), so holes stay below half of what is left and a table that
// does not fill never goes scarce.
#ifndef MIMIC_HCHUNK
#define MIMIC_HCHUNK 32u
#endif
#ifndef HCHUNK_SPIN_LIMIT
#define HCHUNK_SPIN_LIMIT (1u << 16)
#endif
struct HBlk {
    unsigned long long cw;   // the block's chunk: end << 32 | next (ring positions = slots)
    uint32_t lock;           // a wave is refilling cw
    uint32_t mode;           // 0 not known yet, 1 chunks (ring identity), 2 the combiner path (hashmap.h above)
    uint32_t scarce;         // head reached tail: positions only from handed-back remainders
    uint32_t rem1;           // 1 + positions left after the last refill (chunk size hint; 0: none yet)
    uint32_t h0;             // 1 + live positions below this launch's reservations (0: not read yet)
    uint32_t live;           // positions this block gave to inserts, not yet added to live_sh
    uint32_t act, exited;    // waves of the block that run / have reached h_chunk_fini
    uint32_t spins;          // scarce rounds that found nothing
    HashCtl *ctl;            // the chunk map's counters and remainders (h_chunk_fini)
    unsigned long long *left;
};
static __shared__ HBlk h_blk_;
#define HB_LD(p) __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define HB_ST(p, v) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
// thread 0, before the prologue's barrier (h_comb_init): waves whose first lane is below lim run
HDEV void h_chunk_init(uint32_t lim) {
    if (threadIdx.x) return;
    HBlk &B = h_blk_;
    B.cw = 0;
    B.lock = B.mode = B.scarce = B.rem1 = B.h0 = B.live = B.exited = B.spins = 0;
    B.ctl = nullptr;
    B.left = nullptr;
    uint32_t a = 0;
    for (uint32_t w = 0; w * 64 < blockDim.x; w++) a += (uint64_t)blockIdx.x * blockDim.x + w * 64 < lim ? 1u : 0u;
    B.act = a;
}
// is the map's ring the identity this launch (tail == E; pop-only launches never push)?
HDEV bool h_chunk_on(const HT &t, HashCtl *c) {
    if (!(t.flags & HT_F_CHUNK)) return false;
    HBlk &B = h_blk_;
    uint32_t md = HB_LD(&B.mode);
    if (!md) {
        md = __hip_atomic_load(&c->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == t.E ? 1u : 2u;
        HB_ST(&B.mode, md);
    }
    return md == 1u;
}
// ring[0, h0) are -1 (popped before this launch, all live: nothing was pushed) and ring[h0, E) hold
// their own index (chunk launches do not write the ring): the first index that is not -1
HDEV uint32_t h_ring_h0(const HT &t) {
    const int32_t *ring = h_ring(t);
    uint32_t lo = 0, hi = t.E;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (__hip_atomic_load(ring + mid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// One lane of a wave whose k lanes need positions, when the block's chunk is empty: refill it (from
// head; when scarce from a handed-back remainder).  1 = every position is live (E2BIG), 0 = the
// chunk has positions now, or none can be had yet (another wave holds the refill lock, or running
// blocks still hold the rest: try again next round).
static __device__ __attribute__((noinline)) uint32_t h_chunk_fill(const HT &t, HashCtl *c, uint32_t k) {
    HBlk &B = h_blk_;
    uint32_t z = 0;
    if (!__hip_atomic_compare_exchange_strong(&B.lock, &z, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        return 0;
    uint32_t full = 0;
    const unsigned long long w = HB_LD(&B.cw);
    if ((uint32_t)w >= (uint32_t)(w >> 32)) {   // still empty
        B.ctl = c;
        B.left = h_left(t);
        bool got = false;
        if (!HB_LD(&B.scarce)) {
            const uint32_t hint = B.rem1 ? B.rem1 - 1u : t.E;
            uint32_t g = blockIdx.x < HT_LEFT_CAP ? hint / (2u * gridDim.x) : 0u;   // no left[] slot: exact
            g = g > MIMIC_HCHUNK ? MIMIC_HCHUNK : g;
            g = g < k ? k : g;
            const unsigned long long p = __hip_atomic_fetch_add(&c->head, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (p < t.E) {
                const uint32_t n = t.E - p < g ? (uint32_t)(t.E - p) : g;
                __hip_atomic_fetch_max(&c->cminv, 0xffffffffu - (uint32_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                B.rem1 = (uint32_t)(t.E - p) - n + 1u;
                HB_ST(&B.cw, ((p + n) << 32) | p);
                got = true;
            } else {
                HB_ST(&B.scarce, 1u);
            }
        }
        if (!got) {   // scarce: the block's count first, then is every position live?
            const uint32_t lv = __hip_atomic_exchange(&B.live, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lv) __hip_atomic_fetch_add(&c->live_sh[32 * (blockIdx.x & (HT_USED_SHARDS - 1))], lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_load(&c->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                full = 1;
            } else {
                if (!B.h0) B.h0 = h_ring_h0(t) + 1u;
                uint64_t live = B.h0 - 1u;
                for (uint32_t s = 0; s < HT_USED_SHARDS; s++)
                    live += __hip_atomic_load(&c->live_sh[32 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (live >= t.E) {
                    full = 1;
                    __hip_atomic_store(&c->full, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {   // a remainder a finished block handed back
                    unsigned long long *L = B.left;
                    uint32_t nl = __hip_atomic_load(&c->nleft, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    nl = nl < HT_LEFT_CAP ? nl : HT_LEFT_CAP;
                    for (uint32_t j0 = 0; j0 < nl && !got; j0 += 16) {   // 16 loads in flight at a time
                      unsigned long long ev[16];
#pragma unroll
                      for (uint32_t q = 0; q < 16; q++)
                          ev[q] = j0 + q < nl ? __hip_atomic_load(L + j0 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                      for (uint32_t q = 0; q < 16 && !got; q++) {
                        const uint32_t j = j0 + q;
                        unsigned long long e = ev[q];
                        while ((uint32_t)e < (uint32_t)(e >> 32)) {
                            const uint32_t nx = (uint32_t)e, en = (uint32_t)(e >> 32), n = en - nx < k ? en - nx : k;
                            if (__hip_atomic_compare_exchange_strong(L + j, &e, ((unsigned long long)en << 32) | (nx + n),
                                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                                HB_ST(&B.cw, ((unsigned long long)(nx + n) << 32) | nx);
                                got = true;
                                break;
                            }
                        }
                      }
                    }
                    if (!got && ++B.spins > HCHUNK_SPIN_LIMIT) {   // a broken protocol: stop loudly, not hang
                        __hip_atomic_store(&c->comb_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        full = 1;
                    }
                }
            }
        }
    }
    __hip_atomic_store(&B.lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return full;
}
// up to k positions from the block's chunk (LDS): *base, returns how many (the lanes given them insert)
HDEV uint32_t h_chunk_grab(uint32_t k, uint64_t *base) {
    HBlk &B = h_blk_;
    unsigned long long w = HB_LD(&B.cw);
    for (;;) {
        const uint32_t nx = (uint32_t)w, en = (uint32_t)(w >> 32);
        if (nx >= en) return 0;
        const uint32_t n = en - nx < k ? en - nx : k;
        if (__hip_atomic_compare_exchange_strong(&B.cw, &w, ((unsigned long long)en << 32) | (nx + n), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            if (HB_LD(&B.scarce))
                __hip_atomic_fetch_add(&B.ctl->live_sh[32 * (blockIdx.x & (HT_USED_SHARDS - 1))], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                __hip_atomic_fetch_add(&B.live, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            *base = nx;
            return n;
        }
    }
}
HDEV bool h_chunk_empty() {
    const unsigned long long w = HB_LD(&h_blk_.cw);
    return (uint32_t)w >= (uint32_t)(w >> 32);
}
// every running wave at the kernel's end (its active lanes): the last of the block adds the block's
// count to live_sh and hands its chunk's remainder back (left[block], then nleft with release)
HDEV void h_chunk_fini() {
    HBlk &B = h_blk_;
    if (__lane_id() != (uint32_t)__builtin_ctzll(__ballot(1))) return;
    const uint32_t o = __hip_atomic_fetch_add(&B.exited, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (o + 1u != B.act || !B.ctl) return;
    HashCtl *c = B.ctl;
    const uint32_t lv = __hip_atomic_exchange(&B.live, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (lv) __hip_atomic_fetch_add(&c->live_sh[32 * (blockIdx.x & (HT_USED_SHARDS - 1))], lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long w = HB_LD(&B.cw);
    if ((uint32_t)w < (uint32_t)(w >> 32) && blockIdx.x < HT_LEFT_CAP) {
        __hip_atomic_store(B.left + blockIdx.x, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(&c->nleft, blockIdx.x + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}
#endif

// key hash over the zero-padded little-endian key words (any good 64-bit mix; the reference's
// sha256 only names Go-map buckets, which no program can observe)
template <class KS>
HHD uint64_t h_hash(const KS &ks, uint32_t K) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ K;
    const uint32_t nq = (K + 7) >> 3;
    for (uint32_t q = 0; q < nq; q++) {
        h = (h ^ ks.word(q)) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
    }
    h ^= h >> 29;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 32;
    return h;
}

// JIT kernels (MIMIC_CTX_FIXED), keys of up to 32 bytes: every word loaded before any is compared
// (one memory round trip; a load-compare-exit loop waited for each word in turn: two round trips per
// probe of a 16-byte key; cfg-4 lookup-hit step 0.136 -> 0.133 ms).  The batch interpreter keeps the
// loop: the four words cost it 46 more spilled VGPRs.
template <class KS>
HDEV bool h_key_eq(const uint64_t *r, const KS &ks, uint32_t K) {
    const uint32_t nq = (K + 7) >> 3;
#ifdef MIMIC_CTX_FIXED
    if (nq <= 4) {
        uint64_t w[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) w[q] = q < nq ? h_ld(r + 1 + q) : 0ull;
        bool eq = true;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++)
            if (q < nq) eq &= w[q] == ks.word(q);
        return eq;
    }
#endif
    for (uint32_t q = 0; q < nq; q++)
        if (h_ld(r + 1 + q) != ks.word(q)) return false;
    return true;
}

// lock-free lookup: slot index or -1; *pos = bucket of the key.  recheck = false in pop-only
// launches (no program of the launch deletes): a bucket then only moves EMPTY / TOMB -> BUSY ->
// live (or BUSY back, on E2BIG) and a live record never changes, so the state word's re-read that
// guards against a concurrent delete + reuse is not needed (one memory round trip per hit less)
template <class KS>
HDEV int32_t h_find(const HT &t, const KS &ks, uint64_t h, uint32_t *pos, bool recheck = true) {
    const uint32_t mask = t.cap - 1, tag = (uint32_t)(h >> 32);
    uint32_t p = (uint32_t)h & mask;
    for (uint32_t n = 0; n < t.cap; n++, p = (p + 1) & mask) {
        const uint64_t *r = h_rec(t, p);
        const uint64_t w = h_ld(r);
        const uint32_t s = (uint32_t)w;
        if (s == HT_EMPTY) return -1;
        if (s < HT_BUSY && (uint32_t)(w >> 32) == tag && h_key_eq(r, ks, t.K) && (!recheck || h_ld(r) == w)) {
            if (pos) *pos = p;
            return (int32_t)s;
        }
    }
    return -1;
}

// lookup while no writer can run (KParams.hash_ro: no program of the launch updates or deletes,
// and host operations are ordered before the launch): the record -- state word and key words --
// is read with plain loads, all at once, and compared without the re-read that guards against a
// concurrent delete + reuse.  Same result as h_find on an unchanging table.
template <class KS>
HDEV int32_t h_find_ro(const HT &t, const KS &ks, uint64_t h) {
    const uint32_t mask = t.cap - 1, tag = (uint32_t)(h >> 32), nq = (t.K + 7) >> 3;
    // keys over 32 bytes (IPv6 5-tuples): the probe that compares every key word (a second
    // compare loop here would cost every kernel that inlines the generic lookup registers)
    if (nq > 4) return h_find(t, ks, h, nullptr);
    uint32_t p = (uint32_t)h & mask;
    for (uint32_t n = 0; n < t.cap; n++, p = (p + 1) & mask) {
        const uint64_t *r = h_rec(t, p);
        uint64_t w[5];
#pragma unroll
        for (uint32_t q = 0; q < 5; q++)
            if (q <= nq) w[q] = r[q];
        const uint32_t s = (uint32_t)w[0];
        if (s == HT_EMPTY) return -1;
        if (s < HT_BUSY && (uint32_t)(w[0] >> 32) == tag) {
            bool eq = true;
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                if (q < nq) eq &= w[1 + q] == ks.word(q);
            if (eq) return (int32_t)s;
        }
    }
    return -1;
}

HDEV uint32_t *h_lock(const HT &t, uint64_t h) {
    return h_locks(t) + ((uint32_t)h & (t.nlocks - 1));
}
HDEV bool h_try_acquire(uint32_t *lk) {
    uint32_t e = 0;
    return __hip_atomic_compare_exchange_strong(lk, &e, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
HDEV void h_release(uint32_t *lk) {
    h_drain();
    __hip_atomic_store(lk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Probe under the key's stripe lock: the key's slot (found) or -1, and the first reusable
// bucket on its probe path (freep: a tombstone or the terminating EMPTY).
template <class KS>
HDEV int32_t h_probe_held(const HT &t, const KS &ks, uint64_t h, uint32_t *freep) {
    const uint32_t mask = t.cap - 1, tag = (uint32_t)(h >> 32);
    uint32_t p = (uint32_t)h & mask;
    *freep = HT_EMPTY;
    for (uint32_t n = 0; n < t.cap; n++, p = (p + 1) & mask) {
        const uint64_t *r = h_rec(t, p);
        const uint64_t w = h_ld(r);
        const uint32_t s = (uint32_t)w;
        if (s == HT_EMPTY) {
            if (*freep == HT_EMPTY) *freep = p;
            return -1;
        }
        if (s == HT_TOMB) {
            if (*freep == HT_EMPTY) *freep = p;
            continue;
        }
        if (s < HT_BUSY && (uint32_t)(w >> 32) == tag && h_key_eq(r, ks, t.K)) return (int32_t)s;
    }
    return -1;
}

// A new key into slot `idx` (popped), lock held: claim a free bucket from freep on (another
// stripe may take it first: then probe on), write the key words, publish tag | slot.  Returns
// whether the bucket was EMPTY (the table's `used` count grows).
template <class KS>
HDEV bool h_place_held(const HT &t, const KS &ks, uint64_t h, uint32_t freep, int32_t idx) {
    const uint32_t mask = t.cap - 1, tag = (uint32_t)(h >> 32);
    uint32_t p = freep == HT_EMPTY ? ((uint32_t)h & mask) : freep;
    uint64_t *r = nullptr;
    bool was_empty = false;
    for (uint32_t n = 0; n < t.cap; n++, p = (p + 1) & mask) {
        uint64_t *q = h_rec(t, p);
        const uint64_t w = h_ld(q);
        const uint32_t s = (uint32_t)w;
        if ((s == HT_EMPTY || s == HT_TOMB) && h_cas(q, w, ((uint64_t)tag << 32) | HT_BUSY)) {
            r = q;
            was_empty = s == HT_EMPTY;
            break;
        }
    }
    // live + busy <= E < ht_cap, so a free bucket always exists
    const uint32_t nq = (t.K + 7) >> 3;
    for (uint32_t q = 0; q < nq; q++) h_st(r + 1 + q, ks.word(q));
    h_drain();
    h_st(r, ((uint64_t)tag << 32) | (uint32_t)idx);
    return was_empty;
}

// Wave-cooperative locking.  A lane may never spin on a lock while a lane of its own wave holds
// one (the holder could not run on: the wave waits for the spinner at the reconvergence point,
// and two such waves deadlock).  So the lanes of a wave that need a stripe lock go in rounds: in
// a round, one lane per distinct lock (the lowest) tries its lock once; winners run their critical
// section and release, the others retry next round.  Two lanes of a wave with one key (one lock)
// thus never overlap, lanes with different locks insert concurrently, and a single lane
// (sequential runs) takes its lock in the first round.
HDEV bool h_round_leader(uint64_t pend, uint32_t lkid) {
    const uint32_t me = __lane_id();
    bool lead = false;
    for (uint64_t rem = pend; rem;) {  // one leader per distinct lock among the pending lanes
        const uint32_t l = (uint32_t)__builtin_ctzll(rem);
        const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)lkid, (int)l);
        rem &= ~__ballot(lkid == v);
        lead |= me == l;
    }
    return lead;
}

HDEV uint64_t h_bcast64(uint64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((uint64_t)hi << 32) | lo;
}

// find-or-insert for the calling lanes of a wave (the helper path).  The lanes holding their
// locks in a round take their freelist slots with ONE pair of atomics for the round (the
// freelist counters are single words every inserting lane of the GPU would otherwise hit: the
// same-address atomics serialise in L2 and set the insert rate); ranks within the round follow
// lane order.  A lone lane pops exactly like h_fl_pop, so sequential runs get the reference's
// FIFO slots.  Returns the slot or -1 (E2BIG); *inserted = a new slot.
//
// pop_only (no program of the launch deletes, so no push runs concurrently): the round takes its
// positions with one add to head and no `avail` semaphore; positions at or past tail are E2BIG.
// head may then pass tail, and avail is stale: mimic_hash_normalize_kernel sets head = min(head,
// tail), avail = tail - head before any operation that pushes (engine.cpp hash_normalize).
template <class KS>
HDEV int32_t h_insert_wave(const HT &t, const KS &ks, uint64_t h, bool *inserted, bool pop_only = false) {
    uint32_t *lk = h_lock(t, h);
    const uint32_t me = __lane_id();
    const uint32_t lkid = (uint32_t)((uintptr_t)lk >> 2);
    HashCtl *c = h_ctl(t);
    bool done = false;
    int32_t idx = -1;
    *inserted = false;
    for (uint32_t round = 0;; round++) {
        // a lane still waiting for its lock looks for its key without the lock first: once another
        // lane has published it, the lock round would only find it (cfg-4 inserting launch 0.456 ->
        // 0.441 ms).  The helper's own h_find before this call is the same lock-free check.
        if (round && !done) {
            const int32_t f = h_find(t, ks, h, nullptr);
            if (f >= 0) {
                idx = f;
                done = true;
            }
        }
        const uint64_t pend = __ballot(!done);
        if (!pend) break;
        const bool lead = h_round_leader(pend, lkid);
        const bool mine = !done && lead && h_try_acquire(lk);
        uint32_t freep = HT_EMPTY;
        const int32_t found = mine ? h_probe_held(t, ks, h, &freep) : -1;
        const bool need = mine && found < 0;
        const uint64_t needm = __ballot(need);
        int32_t slot = -1;
        if (needm) {
            const uint32_t k = (uint32_t)__builtin_popcountll(needm), first = (uint32_t)__builtin_ctzll(needm);
            uint32_t got = 0;
            uint64_t base = 0;
            if (pop_only) {
                if (me == first) {
                    base = __hip_atomic_fetch_add(&c->head, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long tl = __hip_atomic_load(&c->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    got = base >= tl ? 0u : (tl - base < k ? (uint32_t)(tl - base) : k);
                }
            } else if (me == first) {
                const int32_t a = __hip_atomic_fetch_add(&c->avail, -(int32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                got = a <= 0 ? 0u : ((uint32_t)a < k ? (uint32_t)a : k);
                if (got < k)
                    __hip_atomic_fetch_add(&c->avail, (int32_t)(k - got), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (got) base = __hip_atomic_fetch_add(&c->head, (unsigned long long)got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            got = (uint32_t)__builtin_amdgcn_readlane((int)got, (int)first);
            base = h_bcast64(base, first);
            const uint32_t rank = (uint32_t)__builtin_popcountll(needm & ((1ull << me) - 1));
            if (need && rank < got) {
                int32_t *f = h_ring(t) + ((base + rank) & (t.fl_cap - 1));
                if (pop_only) {   // positions below tail were written before this launch
                    slot = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(f, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    // the push that fills this position has already reserved it (avail counted it)
                    while ((slot = __hip_atomic_exchange(f, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 0)
                        __builtin_amdgcn_s_sleep(1);
                }
            }
        }
        bool empty_used = false;
        if (mine) {
            if (found >= 0) {
                idx = found;
            } else if (slot >= 0) {
                empty_used = h_place_held(t, ks, h, freep, slot);
                idx = slot;
                *inserted = true;
            } else {
                idx = -1;   // the freelist is empty: E2BIG
            }
            h_release(lk);
            done = true;
        }
        const uint64_t um = __ballot(empty_used);
        if (um && me == (uint32_t)__builtin_ctzll(um))
            __hip_atomic_fetch_add(h_used_shard(c), (uint32_t)__builtin_popcountll(um), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!done) __builtin_amdgcn_s_sleep(1);
    }
    return idx;
}

// find-or-insert for the calling lanes of a wave in a pop-only launch (no program of the launch
// deletes): no stripe lock.  A bucket then only moves EMPTY / TOMB -> BUSY -> live during the
// launch (the one exception, a claim given back on E2BIG, happens only once the freelist is spent
// for good), so every lane inserting key k targets the same bucket: the first reusable one on k's
// probe path that no other key holds.  Each round a pending lane walks its path from the home
// bucket: its key live -> found; a BUSY bucket before any reusable one -> it may be k being
// written, wait for the next round; else it tries to claim the first reusable bucket with one CAS
// (lanes of one key race for the same bucket, one wins).  Winners take their freelist positions
// with one head reservation for the round (lane order; while tail is still E -- nothing was ever
// pushed since the ring was filled with 0..E-1 -- position p holds slot p and the ring is not
// read), write the key words and publish tag | slot
// in the same round (a lane never waits on a lane of its own wave), or give the bucket back when
// the freelist is spent (E2BIG).  A lone lane pops exactly as h_insert_wave does (FIFO slots).
template <class KS>
HDEV int32_t h_insert_nolock(const HT &t, const KS &ks, uint64_t h, bool *inserted) {
    const uint32_t mask = t.cap - 1, tag = (uint32_t)(h >> 32);
    const uint32_t me = __lane_id();
    HashCtl *c = h_ctl(t);
    bool done = false;
    int32_t idx = -1;
    *inserted = false;
#ifdef MIMIC_HASH_CHUNK
    const bool chunk = h_chunk_on(t, c);   // positions from the block's chunk (h_chunk_fill above)
#else
    const bool chunk = false;
#endif
    for (;;) {
        const uint64_t pend = __ballot(!done);
        if (!pend) break;
        uint32_t cand = HT_EMPTY;
        uint64_t cw = 0;
        bool blocked = false;
        if (!done) {
            uint32_t p = (uint32_t)h & mask;
            for (uint32_t n = 0; n < t.cap; n++, p = (p + 1) & mask) {
                const uint64_t *r = h_rec(t, p);
                const uint64_t w = h_ld(r);
                const uint32_t s = (uint32_t)w;
                if (s == HT_EMPTY || s == HT_TOMB) {
                    if (cand == HT_EMPTY) {
                        cand = p;
                        cw = w;
                    }
                    if (s == HT_EMPTY) break;
                    continue;
                }
                if (s == HT_BUSY) {
                    if (cand == HT_EMPTY) {   // before any reusable bucket: possibly this key
                        blocked = true;
                        break;
                    }
                    continue;
                }
                if ((uint32_t)(w >> 32) == tag && h_key_eq(r, ks, t.K)) {
                    idx = (int32_t)s;
                    done = true;
                    break;
                }
            }
        }
#ifdef MIMIC_HASH_CHUNK
        if (chunk) {   // an empty chunk is refilled before any bucket is claimed (no claim is held while waiting)
            const uint64_t candm = __ballot(!done && !blocked && cand != HT_EMPTY);
            uint32_t v = 0;   // 1: every position is live (E2BIG); 2: none to be had this round
            if (candm) {
                const uint32_t f = (uint32_t)__builtin_ctzll(candm);
                if (me == f && h_chunk_empty()) v = h_chunk_fill(t, c, (uint32_t)__builtin_popcountll(candm)) ? 1u : h_chunk_empty() ? 2u : 0u;
                v = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)f);
            }
            if (v == 1u && !done && !blocked && cand != HT_EMPTY) {
                idx = -1;
                done = true;
            }
            if (v) cand = HT_EMPTY;
        }
#endif
        const bool mine = !done && !blocked && cand != HT_EMPTY &&
                          h_cas(h_rec(t, cand), cw, ((uint64_t)tag << 32) | HT_BUSY);
        if (mine) {   // the key words go out now: their completion overlaps the reservation's round trip
            uint64_t *r = h_rec(t, cand);
            const uint32_t nq = (t.K + 7) >> 3;
            for (uint32_t q = 0; q < nq; q++) h_st(r + 1 + q, ks.word(q));
        }
        const uint64_t needm = __ballot(mine);
        int32_t slot = -1;
        if (needm) {
            const uint32_t k = (uint32_t)__builtin_popcountll(needm), first = (uint32_t)__builtin_ctzll(needm);
            uint32_t got = 0;
            uint64_t base = 0;
            uint32_t ident = 0;
            if (me == first) {
#ifdef MIMIC_HASH_CHUNK
              if (chunk) {
                  got = h_chunk_grab(k, &base);
                  ident = 1;
              } else
#endif
#ifdef MIMIC_HASH_COMBINE
              if (!h_comb_reserve(t, c, k, &base, &got, &ident))
#endif
              {
#if defined(MIMIC_MEAS_NOHEAD) || defined(MIMIC_MEAS_SPREADHEAD)
                // measurement only (slots collide, results wrong): no shared head counter; SPREADHEAD
                // keeps an atomic with return of the same latency on a per-wave address
                base = ((uint64_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64u) % (t.E > 64 ? t.E - 64 : 1);
#ifdef MIMIC_MEAS_SPREADHEAD
                base += __hip_atomic_fetch_add(&c->used_sh[32 * ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (HT_USED_SHARDS - 1))],
                                               0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0u;
#endif
                got = k;
                ident = 1;
#elif defined(MIMIC_MEAS_NOTAIL)   // measurement only: the head atomic without the tail load
                base = __hip_atomic_fetch_add(&c->head, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                got = base >= t.E ? 0u : (t.E - base < k ? (uint32_t)(t.E - base) : k);
                ident = 1;
#else
                base = __hip_atomic_fetch_add(&c->head, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long tl = __hip_atomic_load(&c->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                got = base >= tl ? 0u : (tl - base < k ? (uint32_t)(tl - base) : k);
                ident = tl == t.E;
#endif
              }
            }
            got = (uint32_t)__builtin_amdgcn_readlane((int)got, (int)first);
            ident = (uint32_t)__builtin_amdgcn_readlane((int)ident, (int)first);
            base = h_bcast64(base, first);
            const uint32_t rank = (uint32_t)__builtin_popcountll(needm & ((1ull << me) - 1));
            if (mine && rank < got) {   // positions below tail were written before this launch
                int32_t *f = h_ring(t) + ((base + rank) & (t.fl_cap - 1));
                slot = ident ? (int32_t)(base + rank) : __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!chunk) __hip_atomic_store(f, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (chunks: the compaction)
            }
        }
        bool empty_used = false;
        if (mine) {
            uint64_t *r = h_rec(t, cand);
            if (slot >= 0) {
                h_drain();   // the key words (written above) before the record goes live
                h_st(r, ((uint64_t)tag << 32) | (uint32_t)slot);
                empty_used = (uint32_t)cw == HT_EMPTY;
                idx = slot;
                *inserted = true;
#ifdef MIMIC_HASH_CHUNK
                if (chunk) {   // for mimic_hash_compact_kernel: the slot is used, and which bucket holds it
                    h_used8(t)[slot] = 1;   // (plain stores: one lane per slot; a bit map's atomic ORs cost more)
                    h_s2b(t)[slot] = cand;
                }
#endif
                done = true;
            } else {
                // the freelist is spent: E2BIG, the bucket as it was (the key words it holds now are
                // never compared: only a live record's are).  Chunks: the block's chunk ran dry between
                // the refill and the claim -- the bucket back, the lane tries again next round.
                h_st(r, cw);
                if (!chunk) {
                    idx = -1;
                    done = true;
                }
            }
        }
        const uint64_t um = __ballot(empty_used);
        if (um && me == (uint32_t)__builtin_ctzll(um))
            __hip_atomic_fetch_add(h_used_shard(c), (uint32_t)__builtin_popcountll(um), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!done) __builtin_amdgcn_s_sleep(1);
    }
    return idx;
}

// delete for the calling lanes of a wave: lock rounds as above; the freed slots of a round go to
// the freelist tail with one reservation and one `avail` release for the round (after every
// ring position of the round is written).
template <class KS>
HDEV void h_delete_wave(const HT &t, const KS &ks, uint64_t h) {
    uint32_t *lk = h_lock(t, h);
    const uint32_t me = __lane_id();
    const uint32_t lkid = (uint32_t)((uintptr_t)lk >> 2);
    HashCtl *c = h_ctl(t);
    bool done = false;
    for (;;) {
        const uint64_t pend = __ballot(!done);
        if (!pend) break;
        const bool lead = h_round_leader(pend, lkid);
        const bool mine = !done && lead && h_try_acquire(lk);
        int32_t idx = -1;
        if (mine) {
            uint32_t p = 0;
            idx = h_find(t, ks, h, &p);
            if (idx >= 0) {
                uint64_t *r = h_rec(t, p);
                h_st(r, (h_ld(r) & ~0xffffffffull) | HT_TOMB);
            }
        }
        const uint64_t pm = __ballot(idx >= 0);
        if (pm) {
            const uint32_t k = (uint32_t)__builtin_popcountll(pm), first = (uint32_t)__builtin_ctzll(pm);
            uint64_t base = 0;
            if (me == first) base = __hip_atomic_fetch_add(&c->tail, (unsigned long long)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base = h_bcast64(base, first);
            if (idx >= 0) {
                int32_t *f = h_ring(t) + ((base + (uint32_t)__builtin_popcountll(pm & ((1ull << me) - 1))) & (t.fl_cap - 1));
                for (;;) {
                    int32_t e = -1;
                    if (__hip_atomic_compare_exchange_strong(f, &e, idx, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT))
                        break;
                    __builtin_amdgcn_s_sleep(1);
                }
                h_drain();
            }
            if (me == first) __hip_atomic_fetch_add(&c->avail, (int32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (mine) {
            h_release(lk);
            done = true;
        }
        if (!done) __builtin_amdgcn_s_sleep(1);
    }
}

// key words taken from device bytes (host-side map operations)
struct KeyBytes {
    const uint8_t *p;
    uint32_t K;
    __host__ __device__ uint64_t word(uint32_t q) const {
        uint64_t v = 0;
        const uint32_t o = q * 8, c = K - o < 8 ? K - o : 8;
        for (uint32_t i = 0; i < c; i++) v |= (uint64_t)p[o + i] << (8 * i);
        return v;
    }
};
// key words from a bucket record (rebuild)
struct KeyRec {
    const uint64_t *r;
    __device__ uint64_t word(uint32_t q) const { return r[1 + q]; }
};
