// skb.hip -- context construction for sk_buff batches (LinuxContextSKBuff.Load,
// context_sk_buff.go:42-107, over SKBuffFromBytes, emulator_linux_sk_buff.go:108-265).
//
// Three stream-ordered steps before the program kernel (JIT or interpreter) runs:
//   1. mimic_skb_prep_kernel: one thread per packet walks the headers once and writes the
//      packet's SkbRec (skb.h) and its leak footprint (219 + L, or 0 when Load fails);
//   2. an exclusive scan of the footprints (hipCUB): packet i's sock / flow-keys / packet
//      entries start at leak_base + prefix[i], exactly where a sequential reference run's
//      first-fit AddEntry puts them (Cleanup leaks them, so they pile up);
//   3. mimic_skb_advance_kernel: publishes this batch's leak_base and moves the VM's leak
//      cursor past the batch (device-side: no host round trip between batches).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "runtime.h"

// The header walk reads single bytes at data-dependent offsets.  As global byte loads each one is
// a memory instruction touching 64 scattered lines per wave; instead each thread first copies the
// first SKB_WIN bytes of its packet into LDS with 16-byte loads (skb_stage), and the walk reads
// bytes from there (skb.h SkbWinBytes).
#define PREP_W SKB_WIN
#define PREP_T 256u

// packet i: packet bytes at pkt_data + pkt_off[i] + 32, pkt_len[i] of them.  rec == nullptr: the
// footprints only (a JIT kernel that walks the headers itself builds the records in LDS).  The records leave
// through LDS: each thread puts its record there and the block writes its records (contiguous in
// rec) with consecutive threads on consecutive 8-byte words -- stored one record per thread,
// every store instruction of a wave would touch 64 records 160 bytes apart.  Half a block's
// records at a time, in the windows' 32 KiB (5 blocks per CU instead of 4 with 40 KiB).
#define PREP_RQ (sizeof(SkbRec) / 8)
#define PREP_HALF (PREP_T / 2)
static_assert(sizeof(SkbRec) % 8 == 0, "SkbRec is copied as 8-byte words");
static_assert(PREP_RQ * PREP_HALF <= (PREP_W / 8) * PREP_T, "half the records fit the window area");
extern "C" __global__ __launch_bounds__(PREP_T) void mimic_skb_prep_kernel(const uint8_t *__restrict__ pkt_data,
                                                                          const uint64_t *__restrict__ pkt_off,
                                                                          const uint32_t *__restrict__ pkt_len,
                                                                          uint32_t n, SkbRec *__restrict__ rec,
                                                                          uint64_t *__restrict__ foot) {
    __shared__ uint64_t area[(PREP_W / 8) * PREP_T];   // the windows first, then the records
    uint32_t *win = (uint32_t *)area;
    const uint32_t t = threadIdx.x, i0 = blockIdx.x * PREP_T, i = i0 + t;
    if (i0 >= n) return;   // whole block past the batch (uniform: the barriers below are safe)
    const bool live = i < n;
    SkbRec r;
    if (live) {
        const uint32_t L = pkt_len[i];
        const uint8_t *pkt = pkt_data + pkt_off[i] + SKB_HEADROOM;
        // the first 128 bytes into registers (16-byte chunks that start inside the packet; one may
        // run into the 64-byte tailroom); common frames decode from there (skb_fast), the rest
        // through this thread's LDS window
        typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        uint32_t w[SKB_WIN / 4];
#pragma unroll
        for (uint32_t c = 0; c < SKB_WIN / 16; c++) {
            u32x4u v = {0, 0, 0, 0};
            if (16 * c < L) v = *(const u32x4u *)(pkt + 16 * c);
            w[4 * c] = v.x;
            w[4 * c + 1] = v.y;
            w[4 * c + 2] = v.z;
            w[4 * c + 3] = v.w;
        }
        skb_init_regs<PREP_T>(w, win, t, pkt, L, r);
        foot[i] = (r.len & SKB_LOAD_FAILED) ? 0ull : (uint64_t)SKB_FOOT_FIXED + L;
    }
    if (!rec) return;   // footprints only
    __syncthreads();   // every window read
    const uint32_t cnt = n - i0 < PREP_T ? n - i0 : PREP_T;
    for (uint32_t h = 0; h < 2; h++) {
        if (live && t / PREP_HALF == h) {
            const uint64_t *rw = (const uint64_t *)&r;
            for (uint32_t q = 0; q < PREP_RQ; q++) area[(t % PREP_HALF) * PREP_RQ + q] = rw[q];
        }
        __syncthreads();
        const uint32_t first = h * PREP_HALF;
        const uint32_t words = cnt > first ? (cnt - first < PREP_HALF ? cnt - first : PREP_HALF) * PREP_RQ : 0u;
        uint64_t *dst = (uint64_t *)(rec + i0 + first);
        for (uint32_t w = t; w < words; w += PREP_T) dst[w] = area[w];
        __syncthreads();
    }
}

// state[0] = the VM's next leak address, state[1] = this batch's leak base
extern "C" __global__ void mimic_skb_advance_kernel(uint64_t *state, const uint64_t *prefix, const uint64_t *foot,
                                                    uint32_t n, uint64_t init_base, uint32_t use_init) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t base = use_init ? init_base : state[0];
    state[1] = base;
    state[0] = base + (n ? prefix[n - 1] + foot[n - 1] : 0ull);
}

extern "C" size_t mimic_skb_scan_bytes(uint32_t n) {
    size_t bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr, (int)n) !=
        hipSuccess)
        return 0;
    return bytes;
}

extern "C" int mimic_launch_skb_prep(const uint8_t *pkt_data, const uint64_t *pkt_off, const uint32_t *pkt_len,
                                     uint32_t n, SkbRec *rec, uint64_t *foot, uint64_t *prefix, void *scan_tmp,
                                     size_t scan_bytes, uint64_t *state, uint64_t init_base, uint32_t use_init,
                                     hipStream_t st) {
    if (n) {
        hipLaunchKernelGGL(mimic_skb_prep_kernel, dim3((n + PREP_T - 1) / PREP_T), dim3(PREP_T), 0, st, pkt_data, pkt_off, pkt_len, n,
                           rec, foot);
        if (hipGetLastError() != hipSuccess) return -1;
        size_t bytes = scan_bytes;
        if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, bytes, (const uint64_t *)foot, prefix, (int)n, st) != hipSuccess)
            return -1;
    }
    hipLaunchKernelGGL(mimic_skb_advance_kernel, dim3(1), dim3(64), 0, st, state, prefix, foot, n, init_base, use_init);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
