// skb.hip -- context construction for sk_buff batches (LinuxContextSKBuff.Load,
// context_sk_buff.go:42-107, over SKBuffFromBytes, emulator_linux_sk_buff.go:108-265).
//
// Two stream-ordered kernels before the program kernel (JIT or interpreter) runs:
//   1. mimic_skb_prep_kernel: one thread per packet walks the headers once and writes the
//      packet's SkbRec (skb.h) and its leak prefix within its block: packet i's sock / flow-keys
//      / packet entries start at leak_base + the sum of the footprints (219 + L, or 0 when Load
//      fails) of the packets before it, exactly where a sequential reference run's first-fit
//      AddEntry puts them (Cleanup leaks them, so they pile up);
//   2. mimic_skb_blocks_kernel (one workgroup): the blocks' offsets in the batch, the batch's
//      leak base, and the VM's leak cursor moved past the batch (device-side: no host round trip
//      between batches).  skb.h skb_leak_pre adds the two parts.  Round 2 ran a hipCUB scan of
//      per-packet footprints and a cursor kernel here: 24 us per 1 M packets.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "runtime.h"

// The header walk reads single bytes at data-dependent offsets.  As global byte loads each one is
// a memory instruction touching 64 scattered lines per wave; instead each thread first copies the
// first SKB_WIN bytes of its packet into LDS with 16-byte loads (skb_stage), and the walk reads
// bytes from there (skb.h SkbWinBytes).
#define PREP_W SKB_WIN
#define PREP_T 256u

// packet i: packet bytes at pkt_data + pkt_off[i] + 32, pkt_len[i] of them; its derived record words
// at rec + i * rec_q.  rec == nullptr: the
// leak prefixes only (a JIT kernel that walks the headers itself builds the records in LDS).  Only
// the records' derived words are written (skb.h SKB_DERIVED_Q: the writable state is constant at
// Load and set by whoever loads the process).  They leave through LDS: each thread puts its
// words there and the block writes them with consecutive threads on consecutive 8-byte words --
// stored one record per thread, every store instruction of a wave would touch 64 records 160
// bytes apart.  The block's derived words (24 KiB) fit the windows' 32 KiB.
#ifdef MIMIC_PREP_PLAIN   // measurement: cached record stores
#define PREP_ST(p, v) (*(p) = (v))
#else   // records are streamed out: non-temporal stores
#define PREP_ST(p, v) __builtin_nontemporal_store((v), (p))
#endif
static_assert(sizeof(SkbRec) % 8 == 0, "SkbRec is copied as 8-byte words");
static_assert(SKB_DERIVED_Q * PREP_T <= (PREP_W / 8) * PREP_T, "a block's derived words fit the window area");
static_assert(PREP_T == (1u << SKB_PREP_LOG2), "skb_leak_pre's block");

// exclusive scan of v over the block (wave shuffles, then the waves' totals); *total = the sum
static __device__ uint64_t prep_exscan(uint64_t v, uint64_t *wtot, uint64_t *total) {
    const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[wv] = x;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < PREP_T / 64; k++) {
        const uint64_t s = wtot[k];
        off += k < wv ? s : 0ull;
        tot += s;
    }
    __syncthreads();   // wtot free again
    *total = tot;
    return off + x - v;
}

// prefix: n + ceil(n / PREP_T) words (within-block prefixes, then the blocks' sums)
extern "C" __global__ __launch_bounds__(PREP_T) void mimic_skb_prep_kernel(uint8_t *__restrict__ pkt_data,
                                                                          const uint64_t *__restrict__ pkt_off,
                                                                          const uint32_t *__restrict__ pkt_len,
                                                                          uint32_t n, uint64_t *__restrict__ rec,
                                                                          uint32_t rec_q, uint64_t *__restrict__ prefix,
                                                                          uint32_t rooms, uint32_t sparse,
                                                                          const uint32_t *__restrict__ rooms_state) {
    __shared__ uint64_t area[(PREP_W / 8) * PREP_T];   // the windows first, then the records
    __shared__ uint64_t wtot[PREP_T / 64];
    uint32_t *win = (uint32_t *)area;
    const uint32_t t = threadIdx.x, i0 = blockIdx.x * PREP_T, i = i0 + t;
    if (i0 >= n) return;   // whole block past the batch (uniform: the barriers below are safe)
    const bool live = i < n;
    // the batch's rooms-clean word (mimic_skb_batch.rooms_state): 1 = an earlier launch left every
    // room zero and no program store has touched one since -- nothing to read (rooms 3)
    if (rooms == 1 && rooms_state && *rooms_state == 1u) rooms = 3;
    SkbRec r;
    uint64_t f = 0;   // the leak footprint
    uint64_t flags = 0;   // skb.h SKB_PFX_*
    if (live) {
        const uint32_t L = pkt_len[i];
        uint8_t *pkt = pkt_data + pkt_off[i] + SKB_HEADROOM;
        // the first SKB_WIN bytes into registers (16-byte chunks that start inside the packet; one may
        // run into the 64-byte tailroom); common frames decode from there (skb_fast), the rest
        // through this thread's LDS window
        typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        // every chunk is loaded (a chunk past the packet's start reloads chunk 0, which is always
        // inside the packet memory) and zeroed after: no branch between the loads, so they issue
        // back to back and the decode waits once (a conditional load per chunk made the compiler wait
        // for the first two chunks before issuing the rest: two round trips)
        u32x4u v[SKB_WIN / 16];
#pragma unroll
        for (uint32_t c = 0; c < SKB_WIN / 16; c++) v[c] = *(const u32x4u *)(pkt + (16 * c < L ? 16 * c : 0u));
        // the rooms flag (skb.h SKB_DIRTY_Q): any non-zero byte in the 32 bytes before the packet
        // or the 64 after it (rooms = 0: a measurement build whose JIT kernel reads them itself).
        // Loaded with the window, before the decode: one memory round trip per packet, not two
        // (the headroom shares the window's first line; the tailroom is the packet's last line).
        // Issued after the window and OR-ed after the decode: loads complete in order, so the
        // decode waits for the window only and runs while the tail line is still on its way
        // (measured: the rooms read cost 28 of the prep's 93 us when it was consumed first).
#ifdef MIMIC_PREP_NOROOMS   // measurement only (tools/prep_probe.py): the rooms not read (flag always clean)
        rooms = 0;
#endif
        // (rooms 0 / 1: loaded whatever `rooms` says, one straight-line load sequence for the wait
        // counter; rooms 2: not read, zeroed below; rooms 3: known zero, not read)
        const u32x4u *hr = (const u32x4u *)(pkt - SKB_HEADROOM), *tr = (const u32x4u *)(pkt + L);
        u32x4u rh0 = {0, 0, 0, 0}, rh1 = rh0, rt[SKB_TAILROOM / 16];
        if (rooms < 2) {
            rh0 = hr[0];
            rh1 = hr[1];
#pragma unroll
            for (uint32_t c = 0; c < SKB_TAILROOM / 16; c++) rt[c] = tr[c];
        } else {
#pragma unroll
            for (uint32_t c = 0; c < SKB_TAILROOM / 16; c++) rt[c] = rh0;
        }
        uint32_t w[SKB_WIN / 4];
#pragma unroll
        for (uint32_t c = 0; c < SKB_WIN / 16; c++) {
            const bool in = 16 * c < L;
            w[4 * c] = in ? v[c].x : 0u;
            w[4 * c + 1] = in ? v[c].y : 0u;
            w[4 * c + 2] = in ? v[c].z : 0u;
            w[4 * c + 3] = in ? v[c].w : 0u;
        }
#ifdef MIMIC_PREP_NOWALK   // measurement only (tools/prep_probe.py): loads and footprints, no decode
        r.len = w[0] == 0x12345678u ? SKB_LOAD_FAILED : L;
        const bool fast = true;
#else
        const bool fast = skb_init_regs<PREP_T>(w, win, t, pkt, L, r);
#endif
        u32x4u o = rh0 | rh1;
#pragma unroll
        for (uint32_t c = 0; c < SKB_TAILROOM / 16; c++) o |= rt[c];
        const uint32_t dirty = rooms == 1 && (o.x | o.y | o.z | o.w) ? 1u : 0u;
        if (rooms == 2 && !(r.len & SKB_LOAD_FAILED)) {   // Load's zeroed rooms, written without a look
            typedef uint32_t u32x4w __attribute__((ext_vector_type(4), aligned(1)));
            const u32x4w z = {0, 0, 0, 0};
            u32x4w *hw = (u32x4w *)(pkt - SKB_HEADROOM), *tw = (u32x4w *)(pkt + L);
            hw[0] = z;
            hw[1] = z;
#pragma unroll
            for (uint32_t c = 0; c < SKB_TAILROOM / 16; c++) tw[c] = z;
        }
        r.ip[0].pad[0] = dirty;
        f = (r.len & SKB_LOAD_FAILED) ? 0ull : (uint64_t)SKB_FOOT_FIXED + L;
        flags = (dirty ? SKB_PFX_DIRTY : 0ull) | (fast ? 0ull : SKB_PFX_EXC);
    }
    if (rec && sparse) {
        // sparse: only the frames skb_fast does not take leave their derived words (the loader builds
        // every other record itself from the packet's first bytes, skb.h skb_fast_rec): few threads
        // store, each its own 96 bytes
        if (live && (flags & SKB_PFX_EXC)) {
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            const uint64_t *rw = (const uint64_t *)&r;
            u64x2 *o = (u64x2 *)(rec + (size_t)i * rec_q);
#pragma unroll
            for (uint32_t u = 0; u < SKB_DERIVED_Q / 2; u++) {
                const u64x2 v = {rw[2 * u], rw[2 * u + 1]};
                o[u] = v;
            }
        }
    } else if (rec) {
#ifdef MIMIC_PREP_DIRECT   // measurement: each thread writes its own derived words (16-byte stores)
        if (live) {
            typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
            const u64x2 *rv = (const u64x2 *)&r;
            u64x2 *o = (u64x2 *)(rec + (size_t)i * rec_q);
#pragma unroll
            for (uint32_t u = 0; u < SKB_DERIVED_Q / 2; u++) PREP_ST(o + u, rv[u]);
        }
#else
        __syncthreads();   // every window read
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
        u64x2 *area2 = (u64x2 *)area;
        if (live) {   // as 8-byte words: a vector view of the record would keep it in a second register layout (87 -> 161 VGPRs)
            const uint64_t *rw = (const uint64_t *)&r;
#pragma unroll
            for (uint32_t q = 0; q < SKB_DERIVED_Q; q++) area[t * SKB_DERIVED_Q + q] = rw[q];
        }
        __syncthreads();
        // the block's records are contiguous in rec: 16-byte units, consecutive threads on consecutive
        // units.  rec_q = SKB_DERIVED_Q (a batch's compact derived-word array): the block's output is
        // one contiguous 24 KiB run; rec_q = 20 (SkbRec records, a stepped process): the writable
        // words between the records are not written
        const uint32_t cnt = n - i0 < PREP_T ? n - i0 : PREP_T;
        constexpr uint32_t DU = SKB_DERIVED_Q / 2;
        if (rec_q == SKB_DERIVED_Q) {
            u64x2 *dst = (u64x2 *)(rec + (size_t)i0 * SKB_DERIVED_Q);
            for (uint32_t w = t; w < cnt * DU; w += PREP_T) PREP_ST(dst + w, area2[w]);
        } else {
            u64x2 *dst = (u64x2 *)(rec + (size_t)i0 * rec_q);
            const uint32_t RU = rec_q / 2;
            for (uint32_t w = t; w < cnt * DU; w += PREP_T) {
                const uint32_t k = w / DU, u = w - k * DU;
                PREP_ST(dst + (size_t)k * RU + u, area2[w]);
            }
        }
#endif
    }
    // the leak prefix within the block, and the block's sum (mimic_skb_blocks_kernel scans those)
    uint64_t bsum;
    const uint64_t ex = prep_exscan(f, wtot, &bsum);
    if (live) prefix[i] = ex | flags;
    if (t == 0) prefix[n + blockIdx.x] = bsum;
}

// The blocks' offsets in the batch (exclusive scan of the nb block sums at bs, in place; one
// workgroup, thread t scans blocks [t*per, t*per+per)), then the batch's leak base and the cursor
// past it.  state[0] = the VM's next leak address, state[1] = this batch's leak base.
// (Finishing this in the prep kernel's last block instead needs a device-scope counter whose
// ordering wait held every block's tail: 77 -> 94 us per 1 M packets.)
#define BLK_T 1024u
extern "C" __global__ __launch_bounds__(BLK_T) void mimic_skb_blocks_kernel(uint64_t *bs, uint32_t nb, uint64_t *state,
                                                                          uint64_t init_base, uint32_t use_init,
                                                                          uint32_t *rooms_state) {
    __shared__ uint64_t wtot[BLK_T / 64];
    const uint32_t t = threadIdx.x, lane = __lane_id(), wv = t >> 6;
    const uint32_t per = (nb + BLK_T - 1) / BLK_T, lo = t * per;
    // the cursor first: its round trip overlaps the sums'
    const uint64_t base0 = t == 0 && !use_init ? state[0] : 0ull;
    // up to BLK_PER sums per thread (batches of up to 2 M packets) loaded at once, no branch between
    // the loads (indices clamped, values masked): one wait, and the write-back reuses them
    constexpr uint32_t BLK_PER = 8;
    uint64_t v[BLK_PER];
    uint64_t s = 0;
    const bool held = nb > 0 && per <= BLK_PER;   // (nb = 0: an empty batch, nothing to read)
    if (held) {
#pragma unroll
        for (uint32_t k = 0; k < BLK_PER; k++) {
            const uint32_t i = lo + k < nb ? lo + k : nb - 1u;
            v[k] = bs[i];
        }
#pragma unroll
        for (uint32_t k = 0; k < BLK_PER; k++) {
            v[k] = k < per && lo + k < nb ? v[k] : 0ull;
            s += v[k];
        }
    } else {
        for (uint32_t k = 0; k < per && lo + k < nb; k++) s += bs[lo + k];
    }
    uint64_t x = s;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[wv] = x;
    __syncthreads();
    uint64_t o = x - s, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < BLK_T / 64; k++) {
        o += k < wv ? wtot[k] : 0ull;
        all += wtot[k];
    }
    if (held) {
#pragma unroll
        for (uint32_t k = 0; k < BLK_PER; k++)
            if (k < per && lo + k < nb) {
                bs[lo + k] = o;
                o += v[k];
            }
    } else {
        for (uint32_t k = 0; k < per && lo + k < nb; k++) {
            const uint64_t w = bs[lo + k];
            bs[lo + k] = o;
            o += w;
        }
    }
    // every room of the batch is zero once the chain has run (it zeroes the ones prep flagged) unless
    // a program stores into one, which sets the word back to 0; prep read it already (stream order)
    if (t == 0 && rooms_state) *rooms_state = 1u;
    if (t == 0) {
        const uint64_t base = use_init ? init_base : base0;
        state[1] = base;
        state[0] = base + all;
    }
}

// the prep kernel alone (tools/prep_probe.py)
extern "C" int mimic_skb_prep_only(const uint8_t *pkt_data, const uint64_t *pkt_off, const uint32_t *pkt_len, uint32_t n,
                                   uint64_t *rec, uint32_t rec_q, uint64_t *prefix, uint64_t *state, hipStream_t st) {
    hipLaunchKernelGGL(mimic_skb_prep_kernel, dim3((n + PREP_T - 1) / PREP_T), dim3(PREP_T), 0, st, (uint8_t *)pkt_data, pkt_off, pkt_len, n,
                       rec, rec_q, prefix, 1u, 0u, (const uint32_t *)nullptr);
    hipLaunchKernelGGL(mimic_skb_blocks_kernel, dim3(1), dim3(BLK_T), 0, st, prefix + n, (n + PREP_T - 1) / PREP_T, state,
                       0ull, 0u, (uint32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// prefix: n + ceil(n / 256) words; state: 2 words.  sparse: derived words for the frames skb_fast
// does not take only (SKB_PFX_EXC), every packet's flags in its prefix word
extern "C" int mimic_launch_skb_prep(const uint8_t *pkt_data, const uint64_t *pkt_off, const uint32_t *pkt_len,
                                     uint32_t n, uint64_t *rec, uint32_t rec_q, uint64_t *prefix, uint64_t *state,
                                     uint64_t init_base, uint32_t use_init, uint32_t rooms, uint32_t sparse,
                                     uint32_t *rooms_state, hipStream_t st) {
    if (n)
        hipLaunchKernelGGL(mimic_skb_prep_kernel, dim3((n + PREP_T - 1) / PREP_T), dim3(PREP_T), 0, st, (uint8_t *)pkt_data, pkt_off, pkt_len, n,
                           rec, rec_q, prefix, rooms, sparse, (const uint32_t *)rooms_state);
    hipLaunchKernelGGL(mimic_skb_blocks_kernel, dim3(1), dim3(BLK_T), 0, st, prefix + n, (n + PREP_T - 1) / PREP_T, state,
                       init_base, use_init, rooms == 1 ? rooms_state : (uint32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// mimic_process_run_many: processes whose LinuxContextSKBuff.Load ran at NewProcess, each with its
// own device block (engine.cpp mimic_process::d_skbmem: SkbRec | prefix word | block word | base |
// mimic_skb_custom), as one batch: derived words into drv (SKB_DERIVED_Q per process), the absolute
// leak address of process i (base + prefix, the prep flags kept) into prefix[i], zero block offsets
// after them, and the user-given sock / flow keys (has_cust[i]) into cust.  The batch's leak base is
// then 0 and skb_leak_pre gives every process the addresses its own Load reserved.
extern "C" __global__ __launch_bounds__(256) void mimic_skb_gather_kernel(const uint8_t *const *__restrict__ mem, uint32_t n,
                                                                         uint64_t *__restrict__ drv, uint64_t *__restrict__ prefix,
                                                                         mimic_skb_custom *__restrict__ cust,
                                                                         const uint8_t *__restrict__ has_cust) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t nb = (n + PREP_T - 1) / PREP_T;
    if (i < nb) prefix[n + i] = 0;
    if (i >= n) return;
    const uint64_t *r = (const uint64_t *)mem[i];
#pragma unroll
    for (uint32_t q = 0; q < SKB_DERIVED_Q; q++) drv[(size_t)i * SKB_DERIVED_Q + q] = r[q];
    const uint64_t *px = (const uint64_t *)(mem[i] + sizeof(SkbRec));
    const uint64_t p0 = px[0];
    prefix[i] = (px[2] + (p0 & SKB_PFX_MASK) + px[1]) | (p0 & ~SKB_PFX_MASK);
    if (cust) {
        if (has_cust[i]) cust[i] = *(const mimic_skb_custom *)(mem[i] + sizeof(SkbRec) + 24);
        else cust[i].flags = 0;
    }
}

extern "C" int mimic_launch_skb_gather(const uint8_t *const *mem, uint32_t n, uint64_t *drv, uint64_t *prefix,
                                       mimic_skb_custom *cust, const uint8_t *has_cust, hipStream_t st) {
    const uint32_t nb = (n + PREP_T - 1) / PREP_T, m = n > nb ? n : nb;
    if (m) hipLaunchKernelGGL(mimic_skb_gather_kernel, dim3((m + 255) / 256), dim3(256), 0, st, mem, n, drv, prefix, cust, has_cust);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
