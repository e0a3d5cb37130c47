// interp.hip -- the gfx950 batch interpreter: one wavefront lane = one vCPU of the
// reference VM, running its packets' processes back to back.
//
// Replaces, per packet, the reference's
//   VM.NewProcess (vm.go:198-235) + LinuxContextXDP.Load (context_xdp_md.go:47-115)
//   Process.SetCPUID (vm.go:268-283)
//   Process.Run -> Process.Step -> instructions[op] (vm.go:291-360, inst.go, inst_gen.go)
//   LinuxEmulator.CallHelperFunction (emulator_linux_.go:125-194) for helpers 1/2/3/8/12/65
//   Process.Cleanup (vm.go:363-374)
// with the reference's effective semantics, bit for bit.
//
// Execution model (CDNA4, wave64):
//  * r0..r10 live in VGPRs (a 12-entry array; index 11 is a write sink).  Register
//    numbers come from the instruction, which is wave-uniform, so `r[dst]` lowers to
//    s_set_gpr_idx / v_mov (VGPR-relative indexing), never to scratch.
//  * Every lane runs the same program; the wave picks the minimum (program, PC) key
//    over its running lanes (DPP row reduction + 4 readlanes), fetches that
//    instruction with scalar loads, and executes it under EXEC = lanes at that key.
//    Divergent lanes reconverge at the smallest PC (min-PC scheduling).
//  * Memory: a 32-bit virtual address is resolved in O(1) for the per-process entries
//    (stack/packet/xdp_md sit after the static entries at lane-computable addresses)
//    and by a short scan of the static segment table otherwise.  Stack and xdp_md
//    overlay live in per-lane private memory interleaved by 8-byte words across lanes
//    (coalesced for the usual R10-relative accesses); the stack is zeroed lazily in
//    32-byte granules (a 64-bit mask per lane) because the reference hands every
//    process a fresh zeroed 2 KiB stack; xdp_md is synthesised from lane registers
//    until a program stores into it.  Packets are read and written in place in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "layout.h"
#include "hashmap.h"
#include "../../include/mimic_amd.h"

typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;

#define DEV static __device__ __forceinline__

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

enum RegionKind : uint32_t { RK_UNRES = 0, RK_STACK = 1, RK_XDP = 2, RK_GLOBAL = 3, RK_NOTVMMEM = 4, RK_NOTDATASEC = 5 };

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
};

static constexpr int EXIT_SIG = -1;

// ---------------------------------------------------------------------------------------
// raw loads / stores (unaligned accesses are legal on gfx950 global memory)
// ---------------------------------------------------------------------------------------
DEV uint64_t ld_n(const uint8_t *p, uint32_t n) {
    switch (n) {
    case 1: return *p;
    case 2: return *(const u16u *)p;
    case 4: return *(const u32u *)p;
    case 8: return *(const u64u *)p;
    default: {
        uint64_t v = 0;
        for (uint32_t i = n; i-- > 0;) v = (v << 8) | p[i];
        return v;
    }
    }
}
DEV void st_n(uint8_t *p, uint32_t n, uint64_t v) {
    switch (n) {
    case 1: *p = (uint8_t)v; return;
    case 2: *(u16u *)p = (uint16_t)v; return;
    case 4: *(u32u *)p = (uint32_t)v; return;
    case 8: *(u64u *)p = v; return;
    default:
        for (uint32_t i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i));
    }
}

// private memory: byte offset o of lane l lives at priv + ((o>>3)*priv_lanes + l)*8 + (o&7)
DEV uint8_t *priv_b(const KParams &kp, uint32_t lane, uint32_t o) {
    return kp.priv + (((size_t)(o >> 3) * kp.priv_lanes + lane) << 3) + (o & 7);
}
DEV uint64_t priv_load(const KParams &kp, uint32_t lane, uint32_t o, uint32_t n) {
    if ((o & 7) + n <= 8) return ld_n(priv_b(kp, lane, o), n);
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; i++) v |= (uint64_t)*priv_b(kp, lane, o + i) << (8 * i);
    return v;
}
DEV void priv_store(const KParams &kp, uint32_t lane, uint32_t o, uint32_t n, uint64_t v) {
    if ((o & 7) + n <= 8) {
        st_n(priv_b(kp, lane, o), n, v);
        return;
    }
    for (uint32_t i = 0; i < n; i++) *priv_b(kp, lane, o + i) = (uint8_t)(v >> (8 * i));
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
DEV bool stk_valid(const KParams &kp, const Lane &L, uint32_t o) {
    return o < STK_FINE ? ((L.sm0 >> (o >> 3)) & 1) : ((L.sm1 >> ((o - STK_FINE) >> kp.chunk_shift)) & 1);
}
DEV void stk_touch(const KParams &kp, Lane &L, uint32_t o) {
    if (o < STK_FINE) {
        const uint32_t q = o >> 3;
        if (!((L.sm0 >> q) & 1)) {
            *(uint64_t *)priv_b(kp, L.lane, q << 3) = 0;
            L.sm0 |= 1ull << q;
        }
    } else {
        const uint32_t c = (o - STK_FINE) >> kp.chunk_shift;
        if (!((L.sm1 >> c) & 1)) {
            const uint32_t q0 = (STK_FINE + (c << kp.chunk_shift)) >> 3, nq = (1u << kp.chunk_shift) >> 3;
            for (uint32_t q = 0; q < nq; q++) *(uint64_t *)priv_b(kp, L.lane, (q0 + q) << 3) = 0;
            L.sm1 |= 1ull << c;
        }
    }
}
DEV uint64_t stack_load(const KParams &kp, const Lane &L, uint32_t o, uint32_t n) {
    if ((o & 7) + n <= 8) {
        if (!stk_valid(kp, L, o)) return 0;
        return ld_n(priv_b(kp, L.lane, o), n);
    }
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t oo = o + i;
        if (stk_valid(kp, L, oo)) v |= (uint64_t)*priv_b(kp, L.lane, oo) << (8 * i);
    }
    return v;
}
DEV void stack_store(const KParams &kp, Lane &L, uint32_t o, uint32_t n, uint64_t v) {
    if ((o & 7) + n <= 8) {
        if (o < STK_FINE && !((L.sm0 >> (o >> 3)) & 1)) {
            // first write to this word: store the whole word, zero-extended around the value
            const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
            *(uint64_t *)priv_b(kp, L.lane, o & ~7u) = (v & m) << (8 * (o & 7));
            L.sm0 |= 1ull << (o >> 3);
            return;
        }
        stk_touch(kp, L, o);
        st_n(priv_b(kp, L.lane, o), n, v);
        return;
    }
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t oo = o + i;
        stk_touch(kp, L, oo);
        *priv_b(kp, L.lane, oo) = (uint8_t)(v >> (8 * i));
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
            *(uint64_t *)priv_b(kp, L.lane, (kp.priv_xdp_q + w) * 8) = q;
        }
        L.xdp_dirty = 1;
    }
    priv_store(kp, L.lane, kp.priv_xdp_q * 8 + o, n, v);
}

// ---------------------------------------------------------------------------------------
// MemoryController.GetEntry (memory_controller.go:117-145) over the lane's address space
// ---------------------------------------------------------------------------------------
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
    bool found = false;
    for (uint32_t s = 0; s < kp.nsegs; s++) {
        const Seg g = cget(kp.segs, s);
        if (!found && a >= g.lo && a <= g.hi) {
            found = true;
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

DEV bool is_vmmem(uint32_t rk) { return rk == RK_STACK || rk == RK_XDP || rk == RK_GLOBAL || rk == RK_NOTDATASEC; }

// VMMem.Load/Store after GetEntry (inst.go:298-363): returns 0 or a status
DEV int mem_load(const KParams &kp, const Lane &L, const Ref &R, uint32_t n, uint64_t &v) {
    if (R.rk == RK_UNRES) return MIMIC_ERR_MEM_UNRESOLVED;
    if (R.rk == RK_NOTVMMEM) return MIMIC_ERR_MEM_NOT_VMMEM;
    if (R.rk == RK_NOTDATASEC) return MIMIC_ERR_MEM_NOT_DATASEC;
    if ((uint64_t)R.off + n > R.limit) return MIMIC_ERR_MEM_BOUNDS;
    if (R.rk == RK_STACK) v = stack_load(kp, L, R.off, n);
    else if (R.rk == RK_XDP) v = xdp_load(kp, L, R.off, n);
    else v = ld_n(R.ptr + R.off, n);
    return 0;
}
DEV int mem_store(const KParams &kp, Lane &L, const Ref &R, uint32_t n, uint64_t v) {
    if (R.rk == RK_UNRES) return MIMIC_ERR_MEM_UNRESOLVED;
    if (R.rk == RK_NOTVMMEM) return MIMIC_ERR_MEM_NOT_VMMEM;
    if (R.rk == RK_NOTDATASEC) return MIMIC_ERR_MEM_NOT_DATASEC;
    if ((uint64_t)R.off + n > R.limit) return MIMIC_ERR_MEM_BOUNDS;
    if (R.rk == RK_STACK) stack_store(kp, L, R.off, n, v);
    else if (R.rk == RK_XDP) xdp_store(kp, L, R.off, n, v);
    else st_n(R.ptr + R.off, n, v);
    return 0;
}
// VMMem.Read bounds check only (the bytes are consumed by the caller chunk-wise)
DEV bool readable(const Ref &R, uint32_t n) {
    if (!(R.rk == RK_STACK || R.rk == RK_XDP || R.rk == RK_GLOBAL)) return false;
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
    if (R.rk == RK_STACK || R.rk == RK_XDP || R.rk == RK_GLOBAL) {
        uint64_t a;
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

// memmove of n bytes from a VM region into the arena (map update, emulator_linux_map_array.go:112)
DEV void copy_into(const KParams &kp, const Lane &L, const Ref &src, uint8_t *dst, uint32_t n) {
    bool backward = src.rk == RK_GLOBAL && src.ptr + src.off < dst && dst < src.ptr + src.off + n;
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
};

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
    HelperOut o = {0, 0, false, false, 0};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = kp.maps[mid];
    Ref K = resolve(kp, L, (uint32_t)r2);
    if (!readable(K, m.key_size)) { o.st = MIMIC_ERR_HELPER_KEY; return o; }
    if (m.family == FAM_ARRAY || m.family == FAM_PERCPU_ARRAY) {
        int32_t which;
        if (array_target(m, sub, L.cpu, which)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        if (m.key_size != 4) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
        uint32_t k = (uint32_t)region_load(kp, L, K, K.off, 4);
        o.r0 = array_value_addr(m, which, k);
        o.set_r0 = true;
        return o;
    }
    // LinuxHashMap.Lookup :134-155 / LinuxPerCPUHashMap.Lookup :537-561
    if (m.family == FAM_PERCPU_HASH && (L.cpu < 0 || (uint32_t)L.cpu >= m.ncpu)) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
    const KeyPriv ks = key_fetch(kp, L, K, m.key_size);
    const int32_t idx = h_find(h_table(kp.arena, m), ks, h_hash(ks, m.key_size), nullptr);
    o.r0 = idx < 0 ? 0 : hash_value_addr(m, L.cpu, (uint32_t)idx);
    o.set_r0 = true;
    return o;
}

DEV HelperOut helper_update(const KParams &kp, const Lane &L, uint64_t r1, uint64_t r2, uint64_t r3) { // :506-555
    HelperOut o = {0, 0, false, false, 0};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = kp.maps[mid];
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
    int32_t idx = h_find(t, ks, h, nullptr);
    bool inserted = false;
    if (idx < 0) {
        // a new key: the lanes of this wave that insert take the stripe locks one at a time
        uint64_t need = __ballot(1);
        const uint32_t me = __lane_id();
        while (need) {
            if (me == (uint32_t)__builtin_ctzll(need)) idx = h_insert_locked(t, ks, h, &inserted);
            need &= need - 1;
        }
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
    HelperOut o = {0, 0, false, false, 0};
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r1, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = kp.maps[mid];
    if (m.family == FAM_ARRAY || m.family == FAM_PERCPU_ARRAY) { o.st = MIMIC_ERR_HELPER_MAP_OP; return o; }
    Ref K = resolve(kp, L, (uint32_t)r2);
    if (!readable(K, m.key_size)) { o.st = MIMIC_ERR_HELPER_KEY; return o; }
    // LinuxHashMap.Delete :225-255 / LinuxPerCPUHashMap.Delete :634-664 (absent key: nil)
    const KeyPriv ks = key_fetch(kp, L, K, m.key_size);
    const uint64_t h = h_hash(ks, m.key_size);
    const HT t = h_table(kp.arena, m);
    uint64_t need = __ballot(1);
    const uint32_t me = __lane_id();
    while (need) {
        if (me == (uint32_t)__builtin_ctzll(need)) h_delete_locked(t, ks, h);
        need &= need - 1;
    }
    o.r0 = 0;
    o.set_r0 = true;
    return o;
}

DEV HelperOut helper_tailcall(const KParams &kp, const Lane &L, uint64_t r2, uint64_t r3) { // :649-738
    HelperOut o = {0, 0, false, false, 0};
    if (L.tailcalls >= kp.max_tail_calls) {
        o.r0 = (uint64_t)(int64_t)-1; // -EPERM
        o.set_r0 = true;
        return o;
    }
    int32_t mid, sub;
    if (!reg_to_map(kp, L, r2, mid, sub)) { o.st = MIMIC_ERR_HELPER_MAP_PTR; return o; }
    const DMap m = kp.maps[mid];
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
// the kernel
// ---------------------------------------------------------------------------------------
#define WAVES_PER_BLOCK 4
#define NREGS 11
#define KEY_DONE 0xffffffffu

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void mimic_xdp_kernel(KParams kp) {
    // eBPF registers r0..r10 of every lane live in LDS, [wave][reg][lane] (8-byte words): a
    // wave-uniform register number addresses 64 consecutive words (conflict-free ds_read_b64),
    // and multi-register updates (exit, helpers) need no register-array copies.
    __shared__ uint64_t sreg[WAVES_PER_BLOCK][NREGS][64];
    uint64_t *const RB = &sreg[threadIdx.x >> 6][0][threadIdx.x & 63];
#define REG(r) RB[(r) * 64]

    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool lane_valid = g < kp.lanes;
    Lane L;
    L.lane = g;
    L.cpu = (int32_t)(kp.vcpu_begin + g);

    uint32_t ex_begin = 0, ex_count = 0;
    if (lane_valid && kp.sched == SCHED_EXPLICIT) {
        ex_begin = kp.sched_start[g];
        ex_count = kp.sched_start[g + 1] - ex_begin;
    }
    uint64_t lane_steps = 0;
    const DProg entry = cget(kp.progs, kp.entry_prog);
    const uint32_t P = kp.static_next + kp.stack_size + 1;

    for (uint32_t j = 0; j < kp.per_lane; j++) {
        // ---- which packet does this lane run in iteration j -----------------------------
        uint32_t i = 0xffffffffu;
        if (lane_valid) {
            if (kp.sched == SCHED_CHUNKED) {
                uint64_t ii = (uint64_t)g * kp.per_lane + j;
                if (ii < kp.n) i = (uint32_t)ii;
            } else if (kp.sched == SCHED_INTERLEAVED) {
                uint64_t ii = (uint64_t)j * kp.lanes + g;
                if (ii < kp.n) i = (uint32_t)ii;
            } else if (j < ex_count) {
                i = kp.sched_pkts[ex_begin + j];
            }
        }

        // ---- NewProcess + LinuxContextXDP.Load --------------------------------------------
#pragma unroll
        for (int q = 0; q < NREGS; q++) REG(q) = 0;
        uint32_t pn = entry.n, pbase = entry.base;
        uint32_t key = KEY_DONE;   // global instruction index = pbase + PC; KEY_DONE = not running
        uint32_t steps = 0;
        L.sm0 = 0;
        L.sm1 = 0;
        L.xdp_dirty = 0;
        L.nframes = 0;
        L.tailcalls = 0;
        L.M = 0;
        L.pkt = nullptr;
        // a process ends here: results straight to HBM (Run's return + p.Registers.R0)
#define TERM(st_, epc_)                                                \
        do {                                                           \
            if (kp.r0) kp.r0[i] = REG(0);                              \
            if (kp.status) kp.status[i] = (uint8_t)(st_);              \
            if (kp.steps) kp.steps[i] = steps;                         \
            if (kp.err_pc) kp.err_pc[i] = (int32_t)(epc_);             \
            lane_steps += steps;                                       \
            key = KEY_DONE;                                            \
        } while (0)
        if (i != 0xffffffffu) {
            const uint32_t H = kp.headroom_arr ? kp.headroom_arr[i] : kp.headroom;
            const uint32_t T = kp.tailroom_arr ? kp.tailroom_arr[i] : kp.tailroom;
            const uint32_t len = kp.pkt_len[i];
            L.pkt = kp.pkt_data + kp.pkt_off[i];
            L.M = H + len + T;
            for (uint32_t b = 0; b < H; b++) L.pkt[b] = 0;
            for (uint32_t b = 0; b < T; b++) L.pkt[H + len + b] = 0;
            L.data = P + H;
            L.data_end = P + H + len;
            L.ingress = (uint32_t)(kp.ingress_arr ? kp.ingress_arr[i] : kp.ingress);
            L.rxq = (uint32_t)(kp.rxq_arr ? kp.rxq_arr[i] : kp.rxq);
            L.egress = (uint32_t)(kp.egress_arr ? kp.egress_arr[i] : kp.egress);
            REG(1) = P + L.M + 1;                        // R1 = xdp_md address
            REG(10) = kp.static_next + kp.frame_size;    // R10 = stack + StackFrameSize (vm.go:224)
            key = pbase;
            if (pn == 0) {                               // Step on an empty program (vm.go:297-299)
                steps = 1;
                TERM(MIMIC_ERR_PC_OOB, 0);
            }
        }

        // ---- Process.Run ------------------------------------------------------------------
        uint64_t wsteps = 0;          // wave-steps since the packets started: bounds every lane's steps
        uint32_t cand = KEY_DONE;     // speculated next key (where the first executing lane went)
        for (;;) {
            const uint64_t live = __ballot(key != KEY_DONE);
            if (live == 0) break;
            uint32_t kw;
            if (cand != KEY_DONE && (__ballot(key != cand) & live) == 0) kw = cand;  // converged
            else kw = wave_min(key);                                                 // min-PC
            kw = (uint32_t)__builtin_amdgcn_readfirstlane((int)kw);
            const DInsn in = cget(kp.insns, kw);    // scalar loads
            const uint64_t act = __ballot(key == kw);
            const uint64_t wbefore = wsteps++;
            if (key == kw) {
                const uint32_t pc = kw - pbase;     // PC of this instruction
                if (wbefore >= kp.budget && (uint64_t)steps == kp.budget) {   // Run's deadline
                    TERM(MIMIC_ERR_STEP_LIMIT, pc);
                } else {
                    steps++;
                    const uint32_t aux = in.aux;
                    const uint32_t op = in.w & 0xff;
                    const uint32_t dst = (in.w >> 8) & 0xf, src = (in.w >> 12) & 0xf;
                    const int32_t off = (int16_t)(in.w >> 16);
                    const uint64_t k = in.k;
                    int st = 0;          // fatal status of this step (EXIT_SIG = clean exit)
                    int jmp = 0;         // 0 fall through, 1 taken (pc+off+1 / call target), 2 explicit nk
                    uint32_t nk = 0;
                    switch (AUX_H(aux)) {
                    case H_NOP:
                        break;
                    case H_ALU64: {
                        const uint64_t d = REG(dst);
                        const uint64_t x = (aux & AUX_X) ? REG(src) : k;
                        REG(dst) = alu64(op & 0xf0, d, x);
                        break;
                    }
                    case H_ALU32: {
                        const uint64_t d = REG(dst);
                        const uint64_t x = (aux & AUX_X) ? REG(src) : k;
                        REG(dst) = alu32(op & 0xf0, d, x);
                        break;
                    }
                    case H_LDIMM:
                        REG(dst) = k;
                        break;
                    case H_JA:
                        jmp = 1;
                        break;
                    case H_JCC: {
                        const uint64_t d = REG(dst);
                        const uint64_t x = (aux & AUX_X) ? REG(src) : k;
                        jmp = jcond(AUX_ARG(aux), d, x, (aux & AUX_W32) != 0) ? 1 : 0;
                        break;
                    }
                    case H_LDX: {
                        const Ref R = resolve(kp, L, (uint32_t)(REG(src) + (uint64_t)(int64_t)off));
                        uint64_t v = 0;
                        st = mem_load(kp, L, R, AUX_SZ(aux), v);
                        if (!st) REG(dst) = v;
                        break;
                    }
                    case H_ST:
                    case H_STX: {
                        const uint64_t v = AUX_H(aux) == H_STX ? REG(src) : k;
                        const Ref R = resolve(kp, L, (uint32_t)(REG(dst) + (uint64_t)(int64_t)off));
                        st = mem_store(kp, L, R, AUX_SZ(aux), v);
                        break;
                    }
                    case H_EXIT:  // inst.go:277-296
                        if (L.nframes > 0) {
                            L.nframes--;
                            const uint32_t fq = kp.priv_frame_q + L.nframes * MIMIC_FRAME_QWORDS;
                            const uint32_t spc = (uint32_t)priv_load(kp, L.lane, fq * 8, 8);
                            REG(6) = priv_load(kp, L.lane, (fq + 1) * 8, 8);
                            REG(7) = priv_load(kp, L.lane, (fq + 2) * 8, 8);
                            REG(8) = priv_load(kp, L.lane, (fq + 3) * 8, 8);
                            REG(9) = priv_load(kp, L.lane, (fq + 4) * 8, 8);
                            REG(10) = REG(10) - kp.frame_size;
                            if (pn <= spc + 1) st = MIMIC_ERR_PC_OOB;   // vm.go:328-334
                            else { jmp = 2; nk = pbase + spc + 1; }
                        } else {
                            st = EXIT_SIG;
                        }
                        break;
                    case H_CALL_LOCAL:  // BPF-to-BPF, inst.go:244-258
                        if (L.nframes >= MIMIC_MAX_FRAMES) {
                            st = MIMIC_ERR_CALL_DEPTH;
                        } else {
                            const uint32_t fq = kp.priv_frame_q + L.nframes * MIMIC_FRAME_QWORDS;
                            priv_store(kp, L.lane, fq * 8, 8, (uint64_t)pc);
                            priv_store(kp, L.lane, (fq + 1) * 8, 8, REG(6));
                            priv_store(kp, L.lane, (fq + 2) * 8, 8, REG(7));
                            priv_store(kp, L.lane, (fq + 3) * 8, 8, REG(8));
                            priv_store(kp, L.lane, (fq + 4) * 8, 8, REG(9));
                            L.nframes++;
                            REG(10) = REG(10) + kp.frame_size;
                            jmp = 1;
                        }
                        break;
                    case H_CALL: {  // helpers, emulator_linux_.go:125-194
                        const int32_t hn = (int32_t)(uint32_t)k;
                        HelperOut ho = {0, 0, false, false, 0};
                        if (hn == 1) ho = helper_lookup(kp, L, REG(1), REG(2));
                        else if (hn == 2) ho = helper_update(kp, L, REG(1), REG(2), REG(3));
                        else if (hn == 3) ho = helper_delete(kp, L, REG(1), REG(2));
                        else if (hn == 8) { ho.r0 = (uint64_t)(int64_t)L.cpu; ho.set_r0 = true; }
                        else if (hn == 12) ho = helper_tailcall(kp, L, REG(2), REG(3));
                        else {  // 65: bpf_xdp_adjust_tail, emulator_linux_helpers.go:842-864
                            const Ref R = resolve(kp, L, (uint32_t)REG(1));
                            const bool plain20 = (R.rk == RK_GLOBAL || R.rk == RK_STACK) && R.map < 0 && R.limit == 20;
                            if (plain20) ho.st = MIMIC_ERR_ENGINE_HELPER;
                            else { ho.r0 = (uint64_t)(int64_t)-22; ho.set_r0 = true; }
                        }
                        st = ho.st;
                        if (!st) {
                            if (ho.set_r0) REG(0) = ho.r0;
                            if (ho.tail) {  // PC = -1, then Step's bounds check on the new program
                                const DProg np = kp.progs[ho.new_prog];
                                L.tailcalls++;
                                if (np.n == 0) st = MIMIC_ERR_PC_OOB;
                                else {
                                    pn = np.n;
                                    pbase = np.base;
                                    jmp = 2;
                                    nk = np.base;
                                }
                            }
                        }
                        break;
                    }
                    case H_ERR:
                        st = (int)AUX_ARG(aux);
                        break;
                    default: {  // H_SLOW: rare forms whose error order is per lane, and END
                        const uint32_t cls = op & 7, hi = op & 0xf0;
                        const bool xsrc = (op & 0x08) != 0;
                        const uint64_t d = REG(dst < NREGS ? dst : 10);
                        const uint64_t s = REG(src < NREGS ? src : 10);
                        uint64_t wv = 0;
                        bool wr = false;
                        if (cls == 1) {  // LDX with dst >= 10, inst.go:298-318
                            const Ref R = resolve(kp, L, (uint32_t)(s + (uint64_t)(int64_t)off));
                            st = mem_load(kp, L, R, size_bytes(op), wv);
                            if (!st) st = dst > 10 ? MIMIC_PANIC_BADREG : MIMIC_ERR_R10_WRITE;
                        } else if (hi == 0xd0) {  // END, inst.go:138-198 (Q4)
                            if (dst > 10) st = MIMIC_PANIC_BADREG;
                            else {
                                wv = d;
                                if (k == 16) wv = xsrc ? (d & 0xffff) : (((d >> 8) & 0xff) | ((d & 0xff) << 8));
                                else if (k == 32) wv = xsrc ? (d & 0xffffffffull) : (uint64_t)__builtin_bswap32((uint32_t)d);
                                else if (k == 64) wv = xsrc ? (d >> 32) : (uint64_t)__builtin_bswap32((uint32_t)(d >> 32));
                                if (dst == 10) st = MIMIC_ERR_R10_WRITE;
                                else wr = true;
                            }
                        } else {  // DIV / MOD with a register divisor (per-lane Go panic)
                            const bool is64 = cls == 7;
                            if (is64 ? s == 0 : (uint32_t)s == 0) st = MIMIC_PANIC_DIV0;
                            else if (dst == 10) st = MIMIC_ERR_R10_WRITE;
                            else {
                                wv = is64 ? alu64(hi, d, s) : alu32(hi, d, s);
                                wr = true;
                            }
                        }
                        if (wr) {
                            const uint32_t wdu = (uint32_t)__builtin_amdgcn_readfirstlane((int)dst);
                            REG(wdu) = wv;
                        }
                        break;
                    }
                    }

                    if (st == EXIT_SIG) {
                        TERM(MIMIC_OK, -1);
                    } else if (st) {
                        TERM(st, pc);
                    } else if (jmp == 0) {                 // PC+1 (vm.go:328-337)
                        if (aux & AUX_FALL_OK) key = kw + 1;
                        else TERM(MIMIC_ERR_PC_OOB, pc);
                    } else if (jmp == 2) {
                        key = nk;
                    } else {                               // taken jump / BPF-to-BPF call
                        const int32_t tgt = op == 0x85 ? (int32_t)pc + (int32_t)(uint32_t)k : (int32_t)pc + off + 1;
                        if (aux & AUX_JT_OK) key = pbase + (uint32_t)tgt;
                        else if (aux & AUX_JT_NEG) {       // next Step indexes Instructions[-x] (vm.go:300)
                            if ((uint64_t)steps == kp.budget) TERM(MIMIC_ERR_STEP_LIMIT, tgt);
                            else { steps++; TERM(MIMIC_PANIC_PC, tgt); }
                        } else TERM(MIMIC_ERR_PC_OOB, pc);
                    }
                }
            }
            cand = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)__builtin_ctzll(act));
        }
#undef TERM
    }
    if (lane_valid && kp.lane_steps) kp.lane_steps[g] = lane_steps;
#undef REG
}

// Sum of a per-CPU u64 array over cpus: out[k] = sum_c base[c*stride + 8k] (the "sum over CPUs"
// readout of a per-CPU counter map).  Threads are laid out so that each owns one key k.
extern "C" __global__ void mimic_sum_u64_kernel(const uint8_t *base, uint64_t stride, uint32_t nvals, uint32_t cpus,
                                                uint64_t *out) {
    const uint32_t T = gridDim.x * blockDim.x;
    const uint32_t m = T / nvals;  // threads per key
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m * nvals) return;
    const uint32_t k = t % nvals;
    uint64_t s = 0;
    for (uint32_t c = t / nvals; c < cpus; c += m) s += *(const uint64_t *)(base + (uint64_t)c * stride + 8ull * k);
    atomicAdd((unsigned long long *)&out[k], (unsigned long long)s);
}

// One host-side hash-map operation (mimic_map_update/lookup/delete), run by the same device code
// the helpers use so that both sides share the index and the freelist.
extern "C" __global__ void mimic_hash_op_kernel(uint8_t *arena, DMap m, uint32_t op, const uint8_t *key,
                                                const uint8_t *val, int32_t cpu, int32_t *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const KeyBytes ks{key, m.key_size};
    const uint64_t h = h_hash(ks, m.key_size);
    const HT t = h_table(arena, m);
    int32_t idx;
    if (op == 0) {
        idx = h_find(t, ks, h, nullptr);
    } else if (op == 1) {
        idx = h_find(t, ks, h, nullptr);
        bool ins = false;
        if (idx < 0) idx = h_insert_locked(t, ks, h, &ins);
        if (idx >= 0) {  // keys.Write + values[cpu].Write (emulator_linux_map_hash.go:188-200)
            uint8_t *kd = arena + m.keys_dev_off + (size_t)idx * m.key_size;
            for (uint32_t i = 0; i < m.key_size; i++) kd[i] = key[i];
            uint8_t *vd = arena + m.dev_off + (m.family == FAM_PERCPU_HASH ? (size_t)cpu * m.dev_stride : 0) +
                          (size_t)idx * m.value_size;
            for (uint32_t i = 0; i < m.value_size; i++) vd[i] = val[i];
        }
    } else {
        idx = h_delete_locked(t, ks, h);
    }
    *out = idx;
}

// Tombstone compaction: when live + deleted buckets pass 3/4 of the table, rebuild it in
// place (one workgroup; launched before every batch, returns at once otherwise).
extern "C" __global__ __launch_bounds__(1024) void mimic_hash_rebuild_kernel(uint8_t *arena, DMap m, uint32_t force) {
    __shared__ uint32_t go, live;
    const HT t = h_table(arena, m);
    HashCtl *c = h_ctl(t);
    if (threadIdx.x == 0) {
        go = force || (uint64_t)c->used * 4 > (uint64_t)m.ht_cap * 3;
        live = 0;
    }
    __syncthreads();
    if (!go) return;
    uint64_t *rec = h_rec(t, 0), *tmp = h_tmp(t);
    const size_t words = (size_t)m.ht_cap * m.rec_q;
    for (size_t i = threadIdx.x; i < words; i += blockDim.x) tmp[i] = rec[i];
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < m.ht_cap; p += blockDim.x) h_st(rec + (size_t)p * m.rec_q, ~0ull);
    __syncthreads();
    const uint32_t mask = m.ht_cap - 1, nq = m.rec_q - 1;
    for (uint32_t p = threadIdx.x; p < m.ht_cap; p += blockDim.x) {
        const uint64_t *t = tmp + (size_t)p * m.rec_q;
        const uint64_t w = t[0];
        if ((uint32_t)w >= HT_BUSY) continue;
        const KeyRec kr{t};
        const uint64_t h = h_hash(kr, m.key_size);
        for (uint32_t q = (uint32_t)h & mask;; q = (q + 1) & mask) {
            uint64_t *r = rec + (size_t)q * m.rec_q;
            if (h_cas(r, ~0ull, ((uint64_t)(uint32_t)(w >> 32) << 32) | HT_BUSY)) {
                for (uint32_t k = 0; k < nq; k++) h_st(r + 1 + k, t[1 + k]);
                h_drain();
                h_st(r, w);
                break;
            }
        }
        atomicAdd(&live, 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) c->used = live;
}

extern "C" int mimic_launch_hash_op(uint8_t *arena, const DMap *m, uint32_t op, const uint8_t *key, const uint8_t *val,
                                    int32_t cpu, int32_t *out, hipStream_t st) {
    hipLaunchKernelGGL(mimic_hash_op_kernel, dim3(1), dim3(64), 0, st, arena, *m, op, key, val, cpu, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_hash_rebuild(uint8_t *arena, const DMap *m, uint32_t force, hipStream_t st) {
    hipLaunchKernelGGL(mimic_hash_rebuild_kernel, dim3(1), dim3(1024), 0, st, arena, *m, force);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_xdp(const KParams *kp, hipStream_t st) {
    const uint32_t blocks = (kp->lanes + 255) / 256;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(mimic_xdp_kernel, dim3(blocks), dim3(256), 0, st, *kp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_sum_u64(const uint8_t *base, uint64_t stride, uint32_t nvals, uint32_t cpus, uint64_t *out,
                                    hipStream_t st) {
    if (hipMemsetAsync(out, 0, (size_t)nvals * 8, st) != hipSuccess) return -1;
    uint32_t threads = nvals * std::max(1u, std::min(cpus, 65536u / std::max(1u, nvals)));
    threads = std::max(threads, nvals);
    threads = (threads / nvals) * nvals;
    const uint32_t blocks = (threads + 255) / 256;
    hipLaunchKernelGGL(mimic_sum_u64_kernel, dim3(blocks), dim3(256), 0, st, base, stride, nvals, cpus, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
