/*
 * mimic_oracle.c -- CPU restatement of dylandreimerink/mimic's Process.Run hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see mimic_oracle.h).  This file restates, as plain C,
 * the *effective* behaviour of the Go reference at /root/reference, including its
 * quirks.  It is deliberately literal -- a sorted entry
 * list with first-fit allocation, a binary search per memory access, per-process
 * heap allocations -- because it doubles as the CPU baseline ("port") that bench.py
 * times beside the GPU engine.
 *
 * Third-party algorithms restated here (not present in /root/reference, pinned by
 * the reference's go.mod): cilium/ebpf v0.9.0 asm.Instruction.Unmarshal (LD_IMM64
 * fusing, imm sign extension), OpCode.SetALUOp/SetJumpOp (InvalidOpCode=0xff for a
 * wrong class), Size.Sizeof.  Go language semantics restated: integer conversion
 * sign/zero extension, unmasked shifts, panics on divide-by-zero / negative signed
 * shift counts / out-of-range slice index.
 */
#include "mimic_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MEM_START 0xFFFFu            /* memory_controller.go:55 */
#define ORC_MAX_FRAMES 32            /* engine bound, mirrored by the product (MIMIC_MAX_FRAMES) */
#define DEFAULT_BUDGET (1ull << 22)
#define EXIT_SIGNAL (-1)

#define E2BIG_ERRNO 7u
#define EINVAL_ERRNO 22u
#define EPERM_ERRNO 1u

/* ------------------------------------------------------------------------- */
/* objects registered in the memory controller                               */
/* ------------------------------------------------------------------------- */

typedef enum { K_PLAIN, K_ARRAY, K_PERCPU_ARRAY, K_HASH, K_PERCPU_HASH, K_PROG, K_SKB, K_SK, K_FK } objkind;

typedef struct {
    uint8_t *b;
    uint32_t len;
    int big_endian;
} plain_mem; /* memory_plain.go:15-18 */

typedef struct {
    char name[64];
    uint32_t type, key_size, value_size, max_entries;
    int datasec; /* Spec.Value is *btf.Datasec, emulator_linux_map_array.go:136 */
} map_spec;

enum { FAM_ARRAY = 1, FAM_PERCPU_ARRAY, FAM_HASH, FAM_PERCPU_HASH };

typedef struct orc_map {
    int family;
    map_spec *spec;
    /* array: emulator_linux_map_array.go:21-27 */
    plain_mem backing;
    uint32_t addr;
    /* per-CPU array: :177-182 */
    struct orc_map **subs;
    int nsubs;
    /* hash: emulator_linux_map_hash.go:21-40 (+ per-CPU :417-436) */
    uint32_t tcap;      /* open-addressing table standing in for KeyToIndex (exact key, sha256 collisions ignored) */
    uint8_t *tkeys;
    int32_t *tidx;      /* -1 empty, -2 deleted, else slot index */
    uint32_t tcount, ntomb;
    int32_t *fl;        /* freelist channel, capacity E+1, FIFO */
    uint32_t fl_cap, fl_head, fl_len;
    plain_mem keys;
    uint32_t keys_addr;
    plain_mem *values;  /* 1 (hash) or V (per-CPU hash) */
    uint32_t *values_addr;
    int nvalues;
} orc_map;

typedef struct {
    uint8_t op, dst, src;
    int16_t off;
    int64_t k; /* asm.Instruction.Constant */
} insn;

typedef struct {
    char name[64];
    insn *ins;
    uint32_t n;
} program;

typedef struct {
    uint32_t addr, size;
    objkind kind;
    void *obj;
} entry;

#define MC_BLK 256
typedef struct mc_blk { entry *e; size_t n; } mc_blk;

struct orc_vm {
    int vcpus, frame_size, frame_count, max_tail_calls;
    struct mc_blk *blk; /* the entry list, sorted by address, in blocks (mc_insert_at) */
    size_t nblk, cap_blk, n;
    /* acceleration indexes of the entry list (same results as the literal loops they stand in for):
     * gaps between entries keyed by their start address in a binary trie with a per-node maximum
     * of the free bytes, so first fit is "lowest start whose gap holds size"; and entry address
     * by object pointer (open addressing), so DelEntryByObj needs no scan */
    struct gap_node { uint32_t c[2]; uint32_t mx; } *gn;
    uint32_t gn_n, gn_cap;
    void **ok; uint32_t *ov; uint8_t *os; /* object index: key, entry address, state 0 empty 1 used 2 tomb */
    uint32_t o_cap, o_used, o_fill;
    int o_dup;          /* an object was entered twice: fall back to the literal scans */
    orc_map **maps;
    int nmaps;
    program **progs;
    int nprogs;
    plain_mem **scratch;
    int nscratch;
    void **leaks;   /* sk_buff contexts' sock / flow_keys / packet objects: never freed by Cleanup */
    int nleaks, cap_leaks;
    char err[256];
};

typedef struct {
    int64_t pc;
    uint64_t r[11];
} regs;

struct orc_proc {
    orc_vm *vm;
    program *prog;
    plain_mem stack;
    regs R;
    int cpu;
    regs *frames;
    int nframes, frames_cap;
    int tailcalls;
    /* xdp_md context (context_xdp_md.go:22-34) */
    int has_ctx;
    plain_mem *pkt, *xdpmd;
    struct skb_state *skb;  /* sk_buff context (context_sk_buff.go:20-29) */
};

static void set_err(orc_vm *vm, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(vm->err, sizeof vm->err, fmt, ap);
    va_end(ap);
}

const char *orc_last_error(orc_vm *vm) { return vm->err; }

/* ------------------------------------------------------------------------- */
/* MemoryController, memory_controller.go                                     */
/* ------------------------------------------------------------------------- */

/* ---- acceleration indexes (test infrastructure speed only; the literal loops stay the spec) ---- */
static uint32_t gn_new(orc_vm *vm) {
    if (vm->gn_n == vm->gn_cap) {
        vm->gn_cap = vm->gn_cap ? vm->gn_cap * 2 : 1024;
        vm->gn = (struct gap_node *)realloc(vm->gn, vm->gn_cap * sizeof *vm->gn);
    }
    memset(&vm->gn[vm->gn_n], 0, sizeof *vm->gn);
    return vm->gn_n++;
}

/* the gap starting at `start` has `avail` bytes before the next entry (0 = no gap there) */
static void gap_set(orc_vm *vm, uint32_t start, uint32_t avail) {
    if (vm->gn_n == 0) { gn_new(vm); gn_new(vm); } /* 0 = null, 1 = root */
    if (avail == 0 && vm->gn[1].mx == 0) return;
    uint32_t path[33];
    uint32_t at = 1;
    for (int b = 31; b >= 0; b--) {
        path[31 - b] = at;
        uint32_t bit = (start >> b) & 1u;
        if (!vm->gn[at].c[bit]) {
            if (avail == 0) return; /* nothing stored there */
            uint32_t nn = gn_new(vm);
            vm->gn[at].c[bit] = nn;
        }
        at = vm->gn[at].c[bit];
    }
    vm->gn[at].mx = avail;
    for (int d = 31; d >= 0; d--) {
        uint32_t n = path[d], l = vm->gn[n].c[0], r = vm->gn[n].c[1];
        uint32_t ml = l ? vm->gn[l].mx : 0, mr = r ? vm->gn[r].mx : 0;
        vm->gn[n].mx = ml > mr ? ml : mr;
    }
}

/* lowest gap start whose gap holds `size` bytes (fits iff size < avail, as AddEntry tests) */
static int gap_first_fit(orc_vm *vm, uint32_t size, uint32_t *start) {
    if (vm->gn_n == 0 || vm->gn[1].mx <= size) return 0;
    uint32_t at = 1, key = 0;
    for (int b = 31; b >= 0; b--) {
        uint32_t l = vm->gn[at].c[0];
        if (l && vm->gn[l].mx > size) {
            at = l;
        } else {
            at = vm->gn[at].c[1];
            key |= 1u << b;
        }
    }
    *start = key;
    return 1;
}

static uint32_t obj_hash(const void *p, uint32_t cap) {
    uint64_t x = (uint64_t)(uintptr_t)p;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
    return (uint32_t)x & (cap - 1);
}

static void obj_put(orc_vm *vm, void *obj, uint32_t addr);

static void obj_grow(orc_vm *vm) {
    uint32_t oc = vm->o_cap;
    void **ok = vm->ok; uint32_t *ov = vm->ov; uint8_t *os = vm->os;
    vm->o_cap = oc ? oc * 2 : 1024;
    if (vm->o_used * 4 < oc) vm->o_cap = oc; /* mostly tombstones: rehash at the same size */
    vm->ok = (void **)calloc(vm->o_cap, sizeof(void *));
    vm->ov = (uint32_t *)calloc(vm->o_cap, sizeof(uint32_t));
    vm->os = (uint8_t *)calloc(vm->o_cap, 1);
    vm->o_used = vm->o_fill = 0;
    for (uint32_t i = 0; i < oc; i++)
        if (os[i] == 1) obj_put(vm, ok[i], ov[i]);
    free(ok); free(ov); free(os);
}

static void obj_put(orc_vm *vm, void *obj, uint32_t addr) {
    if ((vm->o_fill + 1) * 2 > vm->o_cap) obj_grow(vm);
    uint32_t i = obj_hash(obj, vm->o_cap), tomb = UINT32_MAX;
    for (;; i = (i + 1) & (vm->o_cap - 1)) {
        if (vm->os[i] == 1 && vm->ok[i] == obj) { vm->o_dup = 1; return; }
        if (vm->os[i] == 2 && tomb == UINT32_MAX) tomb = i;
        if (vm->os[i] == 0) break;
    }
    if (tomb != UINT32_MAX) i = tomb; else vm->o_fill++;
    vm->ok[i] = obj; vm->ov[i] = addr; vm->os[i] = 1;
    vm->o_used++;
}

static int obj_find(orc_vm *vm, void *obj, uint32_t *slot) {
    if (!vm->o_cap) return 0;
    for (uint32_t i = obj_hash(obj, vm->o_cap);; i = (i + 1) & (vm->o_cap - 1)) {
        if (vm->os[i] == 0) return 0;
        if (vm->os[i] == 1 && vm->ok[i] == obj) { *slot = i; return 1; }
    }
}

/* The sorted entry list (memory_controller.go's []Entry) is kept in blocks of at most MC_BLK
 * entries so an insertion or deletion moves one block's tail, not the whole list; a position is
 * (block, index in block), the end position is (nblk - 1, its n) or (0, 0) when empty. */
typedef struct { size_t b, k; } mc_pos;

static entry *mc_at(orc_vm *vm, mc_pos p) { return &vm->blk[p.b].e[p.k]; }
static int mc_is_end(orc_vm *vm, mc_pos p) { return vm->nblk == 0 || p.k >= vm->blk[p.b].n; }
static mc_pos mc_first(orc_vm *vm) { (void)vm; mc_pos p = {0, 0}; return p; }
static mc_pos mc_end(orc_vm *vm) {
    mc_pos p = {vm->nblk ? vm->nblk - 1 : 0, vm->nblk ? vm->blk[vm->nblk - 1].n : 0};
    return p;
}
static mc_pos mc_next(orc_vm *vm, mc_pos p) {
    if (++p.k >= vm->blk[p.b].n && p.b + 1 < vm->nblk) { p.b++; p.k = 0; }
    return p;
}
static int mc_prev(orc_vm *vm, mc_pos p, mc_pos *out) { /* 0 at the first entry */
    if (p.k > 0) { p.k--; *out = p; return 1; }
    if (p.b == 0) return 0;
    out->b = p.b - 1;
    out->k = vm->blk[p.b - 1].n - 1;
    return 1;
}

/* sort.Search over the list: the first entry with Addr >= addr */
static mc_pos mc_lower_bound(orc_vm *vm, uint32_t addr) {
    if (vm->n == 0) return mc_end(vm);
    size_t lo = 0, hi = vm->nblk;
    while (lo < hi) { /* first block whose last entry has Addr >= addr */
        size_t mid = (lo + hi) / 2;
        if (vm->blk[mid].e[vm->blk[mid].n - 1].addr >= addr) hi = mid; else lo = mid + 1;
    }
    if (lo == vm->nblk) return mc_end(vm);
    mc_blk *B = &vm->blk[lo];
    size_t l = 0, h = B->n;
    while (l < h) {
        size_t mid = (l + h) / 2;
        if (B->e[mid].addr >= addr) h = mid; else l = mid + 1;
    }
    mc_pos p = {lo, l};
    return p;
}

static uint32_t mc_end1(const entry *e) { /* first address after an entry and its one-byte gap */
    return e->addr + e->size + 1;
}

static void mc_insert_at(orc_vm *vm, mc_pos p, const entry *ne) {
    if (vm->nblk == 0) {
        vm->blk = (mc_blk *)calloc(1, sizeof(mc_blk));
        vm->blk[0].e = (entry *)malloc(MC_BLK * sizeof(entry));
        vm->nblk = vm->cap_blk = 1;
        p.b = p.k = 0;
    }
    if (vm->blk[p.b].n == MC_BLK) { /* split the full block in halves */
        if (vm->nblk == vm->cap_blk) {
            vm->cap_blk *= 2;
            vm->blk = (mc_blk *)realloc(vm->blk, vm->cap_blk * sizeof(mc_blk));
        }
        memmove(&vm->blk[p.b + 2], &vm->blk[p.b + 1], (vm->nblk - p.b - 1) * sizeof(mc_blk));
        vm->nblk++;
        mc_blk *A = &vm->blk[p.b], *N = &vm->blk[p.b + 1];
        N->e = (entry *)malloc(MC_BLK * sizeof(entry));
        N->n = MC_BLK / 2;
        memcpy(N->e, A->e + MC_BLK / 2, N->n * sizeof(entry));
        A->n = MC_BLK / 2;
        if (p.k > A->n) { p.b++; p.k -= MC_BLK / 2; }
    }
    mc_blk *B = &vm->blk[p.b];
    memmove(&B->e[p.k + 1], &B->e[p.k], (B->n - p.k) * sizeof(entry));
    B->e[p.k] = *ne;
    B->n++;
    vm->n++;
}

static void mc_remove_at(orc_vm *vm, mc_pos p) {
    mc_blk *B = &vm->blk[p.b];
    memmove(&B->e[p.k], &B->e[p.k + 1], (B->n - p.k - 1) * sizeof(entry));
    B->n--;
    vm->n--;
    if (B->n == 0 && vm->nblk > 1) {
        free(B->e);
        memmove(&vm->blk[p.b], &vm->blk[p.b + 1], (vm->nblk - p.b - 1) * sizeof(mc_blk));
        vm->nblk--;
    }
}

/* AddEntry, memory_controller.go:58-112 (first fit from memStart+1, one-byte gaps). */
static int mc_add(orc_vm *vm, void *obj, objkind kind, uint32_t size, uint32_t *addr_out) {
    mc_pos at = mc_end(vm);
    uint32_t addr = MEM_START + 1;
    uint64_t tail = vm->n ? (uint64_t)mc_end1(mc_at(vm, (mc_pos){vm->nblk - 1, vm->blk[vm->nblk - 1].n - 1}))
                          : MEM_START + 1;
    int fast = !vm->o_dup && tail + size <= 0xFFFFFFFFull; /* no gap start + size can wrap 32 bits */
    if (fast && vm->n > 0) {
        uint32_t g;
        if (gap_first_fit(vm, size, &g)) {   /* the first entry whose preceding gap holds size */
            addr = g;
            at = mc_lower_bound(vm, g);
        } else {                             /* past the last entry */
            addr = (uint32_t)tail;
            if (0xFFFFFFFFu - addr < size) {
                set_err(vm, "out of memory");
                return -1;
            }
        }
    } else if (vm->n > 0) {
        /* the literal loop of memory_controller.go:70-90 */
        for (mc_pos j = mc_first(vm); !mc_is_end(vm, j); j = mc_next(vm, j)) {
            entry *cur = mc_at(vm, j);
            if ((uint32_t)(addr + size) < cur->addr) {
                at = j;
                break;
            }
            addr = cur->addr + cur->size + 1;
            if (mc_is_end(vm, mc_next(vm, j))) {
                uint32_t avail = 0xFFFFFFFFu - addr;
                if (avail < size) {
                    set_err(vm, "out of memory");
                    return -1;
                }
            }
        }
    }
    entry ne = {addr, size, kind, obj};
    int in_gap = !mc_is_end(vm, at);
    mc_insert_at(vm, at, &ne);
    if (in_gap) { /* the gap this entry went into now starts after it */
        mc_pos nx = mc_lower_bound(vm, addr + 1);
        gap_set(vm, addr, 0);
        gap_set(vm, addr + size + 1, mc_at(vm, nx)->addr - (addr + size + 1));
    }
    obj_put(vm, obj, addr);
    if (addr_out) *addr_out = addr;
    return 0;
}

/* GetEntry, memory_controller.go:117-145 (inclusive upper bound at :137). */
static entry *mc_get(orc_vm *vm, uint32_t addr, uint32_t *off) {
    if (vm->n == 0) return NULL;
    mc_pos lo = mc_lower_bound(vm, addr), pv;
    if (!mc_is_end(vm, lo) && mc_at(vm, lo)->addr == addr) {
        *off = 0;
        return mc_at(vm, lo);
    }
    if (mc_prev(vm, lo, &pv)) {
        entry *prev = mc_at(vm, pv);
        if (addr >= prev->addr && (uint64_t)addr <= (uint64_t)prev->addr + prev->size) {
            *off = addr - prev->addr;
            return prev;
        }
    }
    return NULL;
}

/* DelEntryByObj, memory_controller.go:202-232. */
static void mc_del_at(orc_vm *vm, mc_pos j) {
    mc_pos pv;
    uint32_t before = mc_prev(vm, j, &pv) ? mc_end1(mc_at(vm, pv)) : MEM_START + 1;
    entry *e = mc_at(vm, j);
    uint32_t addr = e->addr;
    gap_set(vm, before, 0);
    gap_set(vm, mc_end1(e), 0);
    uint32_t slot;
    if (obj_find(vm, e->obj, &slot) && vm->ov[slot] == addr) {
        vm->os[slot] = 2;
        vm->o_used--;
    }
    mc_remove_at(vm, j);
    mc_pos nx = mc_lower_bound(vm, addr);
    if (!mc_is_end(vm, nx)) gap_set(vm, before, mc_at(vm, nx)->addr - before); /* the two gaps merge */
}

static int mc_find_obj(orc_vm *vm, void *obj, mc_pos *out) {
    uint32_t slot;
    if (!vm->o_dup) {
        if (!obj_find(vm, obj, &slot)) return 0;
        mc_pos j = mc_lower_bound(vm, vm->ov[slot]);
        if (mc_is_end(vm, j) || mc_at(vm, j)->obj != obj) return 0;
        *out = j;
        return 1;
    }
    if (vm->n == 0) return 0;
    mc_pos j = mc_end(vm), pv; /* the literal scan, last entry first */
    while (mc_prev(vm, j, &pv)) {
        if (mc_at(vm, pv)->obj == obj) { *out = pv; return 1; }
        j = pv;
    }
    return 0;
}

static void mc_del_obj(orc_vm *vm, void *obj) {
    mc_pos j;
    if (mc_find_obj(vm, obj, &j)) mc_del_at(vm, j);
}

static entry *mc_by_obj(orc_vm *vm, void *obj) {
    mc_pos j;
    return mc_find_obj(vm, obj, &j) ? mc_at(vm, j) : NULL;
}

uint32_t orc_mem_next_free(orc_vm *vm) {
    if (vm->n == 0) return MEM_START + 1;
    return mc_end1(mc_at(vm, (mc_pos){vm->nblk - 1, vm->blk[vm->nblk - 1].n - 1}));
}

/* ------------------------------------------------------------------------- */
/* PlainMemory, memory_plain.go                                               */
/* ------------------------------------------------------------------------- */

static int size_bytes(uint8_t op) { /* asm.Size.Sizeof on op&0x18 */
    switch (op & 0x18) {
    case 0x00: return 4;
    case 0x08: return 2;
    case 0x10: return 1;
    default: return 8;
    }
}

/* Load, memory_plain.go:25-52 */
static int pm_load(plain_mem *m, uint32_t off, int n, uint64_t *v) {
    if ((uint64_t)off + (uint64_t)n > m->len) return ORC_ERR_MEM_BOUNDS;
    uint64_t x = 0;
    if (m->big_endian) {
        for (int k = 0; k < n; k++) x = (x << 8) | m->b[off + k];
    } else {
        for (int k = n - 1; k >= 0; k--) x = (x << 8) | m->b[off + k];
    }
    *v = x;
    return 0;
}

/* Store, memory_plain.go:55-87 */
static int pm_store(plain_mem *m, uint32_t off, uint64_t v, int n) {
    if ((uint64_t)off + (uint64_t)n > m->len) return ORC_ERR_MEM_BOUNDS;
    for (int k = 0; k < n; k++) {
        int sh = m->big_endian ? (n - 1 - k) * 8 : k * 8;
        m->b[off + k] = (uint8_t)(v >> sh);
    }
    return 0;
}

/* Read / Write, memory_plain.go:90-119 */
static int pm_read(plain_mem *m, uint32_t off, uint8_t *out, uint32_t n) {
    if ((uint64_t)off + n > m->len) return ORC_ERR_MEM_BOUNDS;
    memcpy(out, m->b + off, n);
    return 0;
}
static int pm_write(plain_mem *m, uint32_t off, const uint8_t *in, uint32_t n) {
    if ((uint64_t)off + n > m->len) return ORC_ERR_MEM_BOUNDS;
    memcpy(m->b + off, in, n);
    return 0;
}

static plain_mem *pm_new(uint32_t len) {
    plain_mem *m = (plain_mem *)calloc(1, sizeof *m);
    m->b = (uint8_t *)calloc(len ? len : 1, 1);
    m->len = len;
    return m;
}
static void pm_free(plain_mem *m) {
    if (!m) return;
    free(m->b);
    free(m);
}

static int skb_access(void *obj, objkind kind, uint32_t off, int n, uint64_t *v, int load);

/* VMMem dispatch for an entry: PlainMemory or LinuxArrayMap (emulator_linux_map_array.go:134-168).
 * Returns ORC_ERR_MEM_NOT_VMMEM for objects that do not implement VMMem. */
static int vm_load(entry *e, uint32_t off, int n, uint64_t *v) {
    if (e->kind == K_PLAIN) return pm_load((plain_mem *)e->obj, off, n, v);
    if (e->kind == K_SKB || e->kind == K_SK || e->kind == K_FK) return skb_access(e->obj, e->kind, off, n, v, 1);
    if (e->kind == K_ARRAY) {
        orc_map *m = (orc_map *)e->obj;
        if (!m->spec->datasec) return ORC_ERR_MEM_NOT_DATASEC;
        return pm_load(&m->backing, off, n, v);
    }
    return ORC_ERR_MEM_NOT_VMMEM;
}
static int vm_store(entry *e, uint32_t off, uint64_t v, int n) {
    if (e->kind == K_PLAIN) return pm_store((plain_mem *)e->obj, off, v, n);
    if (e->kind == K_SKB || e->kind == K_SK || e->kind == K_FK) return skb_access(e->obj, e->kind, off, n, &v, 0);
    if (e->kind == K_ARRAY) {
        orc_map *m = (orc_map *)e->obj;
        if (!m->spec->datasec) return ORC_ERR_MEM_NOT_DATASEC;
        return pm_store(&m->backing, off, v, n);
    }
    return ORC_ERR_MEM_NOT_VMMEM;
}
static int vm_read(entry *e, uint32_t off, uint8_t *out, uint32_t n) {
    if (e->kind == K_PLAIN) return pm_read((plain_mem *)e->obj, off, out, n);
    if (e->kind == K_SKB || e->kind == K_SK || e->kind == K_FK) return ORC_ERR_CTX_ACCESS; /* "not implemented" */
    if (e->kind == K_ARRAY) {
        orc_map *m = (orc_map *)e->obj;
        if (!m->spec->datasec) return ORC_ERR_MEM_NOT_DATASEC;
        return pm_read(&m->backing, off, out, n);
    }
    return ORC_ERR_MEM_NOT_VMMEM;
}
static int vm_write(entry *e, uint32_t off, const uint8_t *in, uint32_t n) {
    if (e->kind == K_PLAIN) return pm_write((plain_mem *)e->obj, off, in, n);
    if (e->kind == K_SKB || e->kind == K_SK || e->kind == K_FK) return ORC_ERR_CTX_ACCESS;
    if (e->kind == K_ARRAY) {
        orc_map *m = (orc_map *)e->obj;
        if (!m->spec->datasec) return ORC_ERR_MEM_NOT_DATASEC;
        return pm_write(&m->backing, off, in, n);
    }
    return ORC_ERR_MEM_NOT_VMMEM;
}
static int is_vmmem(objkind k) { return k == K_PLAIN || k == K_ARRAY || k == K_SKB || k == K_SK || k == K_FK; }
static int is_linuxmap(objkind k) { return k == K_ARRAY || k == K_PERCPU_ARRAY || k == K_HASH || k == K_PERCPU_HASH; }

/* ------------------------------------------------------------------------- */
/* VM                                                                          */
/* ------------------------------------------------------------------------- */

orc_vm *orc_vm_new(int vcpus, int frame_size, int frame_count, int max_tail_calls) {
    orc_vm *vm = (orc_vm *)calloc(1, sizeof *vm);
    vm->vcpus = vcpus;                     /* VMOptSetvCPUs, vm.go:36-40 */
    vm->frame_size = frame_size > 0 ? frame_size : 256;  /* vm.go:60 */
    vm->frame_count = frame_count > 0 ? frame_count : 8; /* vm.go:62 */
    vm->max_tail_calls = max_tail_calls;   /* emulator_linux_.go:78 default 33 */
    /* MIMIC_ORACLE_LITERAL_MC=1: first fit and DelEntryByObj by the literal scans only (the tests
     * check the indexes against them) */
    const char *lit = getenv("MIMIC_ORACLE_LITERAL_MC");
    if (lit && lit[0] == '1') vm->o_dup = 1;
    return vm;
}

static void map_free(orc_map *m) {
    if (!m) return;
    free(m->backing.b);
    if (m->subs) {
        for (int i = 0; i < m->nsubs; i++) {
            free(m->subs[i]->backing.b);
            free(m->subs[i]);
        }
        free(m->subs);
    }
    free(m->tkeys);
    free(m->tidx);
    free(m->fl);
    free(m->keys.b);
    if (m->values) {
        for (int i = 0; i < m->nvalues; i++) free(m->values[i].b);
        free(m->values);
    }
    free(m->values_addr);
    free(m->spec);
    free(m);
}

void orc_vm_free(orc_vm *vm) {
    if (!vm) return;
    for (int i = 0; i < vm->nmaps; i++) map_free(vm->maps[i]);
    for (int i = 0; i < vm->nprogs; i++) {
        free(vm->progs[i]->ins);
        free(vm->progs[i]);
    }
    for (int i = 0; i < vm->nscratch; i++) pm_free(vm->scratch[i]);
    free(vm->scratch);
    for (int i = 0; i < vm->nleaks; i++) free(vm->leaks[i]);
    free(vm->leaks);
    free(vm->maps);
    free(vm->progs);
    for (size_t b = 0; b < vm->nblk; b++) free(vm->blk[b].e);
    free(vm->blk);
    free(vm->gn);
    free(vm->ok);
    free(vm->ov);
    free(vm->os);
    free(vm);
}

/* ------------------------------------------------------------------------- */
/* Maps                                                                        */
/* ------------------------------------------------------------------------- */

/* LinuxArrayMap.Init, emulator_linux_map_array.go:30-54 */
static int array_init(orc_vm *vm, orc_map *m) {
    uint32_t size = m->spec->max_entries * m->spec->value_size;
    m->backing.b = (uint8_t *)calloc(size ? size : 1, 1);
    m->backing.len = size;
    if (mc_add(vm, m, K_ARRAY, 8, NULL)) return -1;
    if (mc_add(vm, &m->backing, K_PLAIN, size, &m->addr)) return -1;
    return 0;
}

static uint32_t fnv(const uint8_t *k, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; i++) h = (h ^ k[i]) * 16777619u;
    return h;
}

/* LinuxHashMap.Init, emulator_linux_map_hash.go:43-97; LinuxPerCPUHashMap.Init :439-500 */
static int hash_init(orc_vm *vm, orc_map *m, int percpu) {
    map_spec *s = m->spec;
    uint32_t E = s->max_entries;
    m->tcap = 16;
    while (m->tcap < 2 * E + 2) m->tcap <<= 1;
    m->tkeys = (uint8_t *)calloc((size_t)m->tcap * (s->key_size ? s->key_size : 1), 1);
    m->tidx = (int32_t *)malloc(sizeof(int32_t) * m->tcap);
    for (uint32_t i = 0; i < m->tcap; i++) m->tidx[i] = -1;
    m->fl_cap = E + 1;
    m->fl = (int32_t *)malloc(sizeof(int32_t) * m->fl_cap);
    for (uint32_t i = 0; i < E; i++) m->fl[i] = (int32_t)i;
    m->fl_head = 0;
    m->fl_len = E;
    m->keys.b = (uint8_t *)calloc((size_t)E * s->key_size + 1, 1);
    m->keys.len = E * s->key_size;
    m->nvalues = percpu ? vm->vcpus : 1;
    m->values = (plain_mem *)calloc((size_t)m->nvalues, sizeof(plain_mem));
    m->values_addr = (uint32_t *)calloc((size_t)m->nvalues, sizeof(uint32_t));
    for (int i = 0; i < m->nvalues; i++) {
        m->values[i].b = (uint8_t *)calloc((size_t)E * s->value_size + 1, 1);
        m->values[i].len = E * s->value_size;
    }
    if (percpu) {
        for (int i = 0; i < m->nvalues; i++)
            if (mc_add(vm, &m->values[i], K_PLAIN, m->values[i].len, &m->values_addr[i])) return -1;
        if (mc_add(vm, m, K_PERCPU_HASH, 8, NULL)) return -1;
        if (mc_add(vm, &m->keys, K_PLAIN, m->keys.len, &m->keys_addr)) return -1;
    } else {
        if (mc_add(vm, m, K_HASH, 8, NULL)) return -1;
        if (mc_add(vm, &m->keys, K_PLAIN, m->keys.len, &m->keys_addr)) return -1;
        if (mc_add(vm, &m->values[0], K_PLAIN, m->values[0].len, &m->values_addr[0])) return -1;
    }
    return 0;
}

static int32_t ht_find(orc_map *m, const uint8_t *key, uint32_t *pos_out) {
    uint32_t K = m->spec->key_size;
    uint32_t p = fnv(key, K) & (m->tcap - 1);
    for (;;) {
        int32_t t = m->tidx[p];
        if (t == -1) {
            if (pos_out) *pos_out = p;
            return -1;
        }
        if (t >= 0 && memcmp(m->tkeys + (size_t)p * K, key, K) == 0) {
            if (pos_out) *pos_out = p;
            return t;
        }
        p = (p + 1) & (m->tcap - 1);
    }
}

static void ht_place(orc_map *m, const uint8_t *key, int32_t idx) {
    uint32_t K = m->spec->key_size;
    uint32_t p = fnv(key, K) & (m->tcap - 1);
    while (m->tidx[p] >= 0) p = (p + 1) & (m->tcap - 1);
    if (m->tidx[p] == -2) m->ntomb--;
    m->tidx[p] = idx;
    memcpy(m->tkeys + (size_t)p * K, key, K);
    m->tcount++;
}

/* rebuild the probe table when deletions have left too many tombstones */
static void ht_rehash(orc_map *m) {
    uint32_t K = m->spec->key_size, cap = m->tcap;
    uint8_t *ok = m->tkeys;
    int32_t *oi = m->tidx;
    m->tkeys = (uint8_t *)calloc((size_t)cap * (K ? K : 1), 1);
    m->tidx = (int32_t *)malloc(sizeof(int32_t) * cap);
    for (uint32_t i = 0; i < cap; i++) m->tidx[i] = -1;
    m->tcount = 0;
    m->ntomb = 0;
    for (uint32_t i = 0; i < cap; i++)
        if (oi[i] >= 0) ht_place(m, ok + (size_t)i * K, oi[i]);
    free(ok);
    free(oi);
}

static void ht_insert(orc_map *m, const uint8_t *key, int32_t idx) {
    if ((m->tcount + m->ntomb + 1) * 4 > m->tcap * 3) ht_rehash(m);
    ht_place(m, key, idx);
}

/* MapSpecToLinuxMap, emulator_linux_map.go:57-113 + LinuxEmulator.AddMap, emulator_linux_.go:97-116 */
int orc_map_create(orc_vm *vm, const char *name, uint32_t type, uint32_t key_size, uint32_t value_size,
                   uint32_t max_entries, int datasec) {
    for (int i = 0; i < vm->nmaps; i++) {
        if (strcmp(vm->maps[i]->spec->name, name) == 0) {
            set_err(vm, "map with name '%s' already exists in emulator", name);
            return -1;
        }
    }
    orc_map *m = (orc_map *)calloc(1, sizeof *m);
    m->spec = (map_spec *)calloc(1, sizeof *m->spec);
    snprintf(m->spec->name, sizeof m->spec->name, "%s", name);
    m->spec->type = type;
    m->spec->key_size = key_size;
    m->spec->value_size = value_size;
    m->spec->max_entries = max_entries;
    m->spec->datasec = datasec;
    int rc;
    switch (type) {
    case ORC_MAP_ARRAY: case ORC_MAP_PROG_ARRAY: case ORC_MAP_ARRAY_OF_MAPS: case ORC_MAP_DEVMAP:
    case ORC_MAP_SOCKMAP: case ORC_MAP_CPUMAP: case ORC_MAP_XSKMAP: case ORC_MAP_CGROUP_ARRAY:
    case ORC_MAP_REUSEPORT_SOCKARRAY:
        m->family = FAM_ARRAY;
        rc = array_init(vm, m);
        break;
    case ORC_MAP_PERCPU_ARRAY:
        /* LinuxPerCPUArrayMap.Init, emulator_linux_map_array.go:185-215 */
        m->family = FAM_PERCPU_ARRAY;
        rc = mc_add(vm, m, K_PERCPU_ARRAY, 8, NULL);
        m->subs = (orc_map **)calloc((size_t)(vm->vcpus > 0 ? vm->vcpus : 1), sizeof(orc_map *));
        for (int i = 0; rc == 0 && i < vm->vcpus; i++) {
            orc_map *sub = (orc_map *)calloc(1, sizeof *sub);
            sub->family = FAM_ARRAY;
            sub->spec = m->spec; /* Spec: m.Spec (shared, parent's type) */
            rc = array_init(vm, sub);
            m->subs[m->nsubs++] = sub;
        }
        break;
    case ORC_MAP_HASH: case ORC_MAP_HASH_OF_MAPS: case ORC_MAP_SOCKHASH: case ORC_MAP_CGROUP_STORAGE:
    case ORC_MAP_SK_STORAGE: case ORC_MAP_DEVMAP_HASH: case ORC_MAP_STRUCT_OPS: case ORC_MAP_INODE_STORAGE:
    case ORC_MAP_TASK_STORAGE:
        m->family = FAM_HASH;
        rc = hash_init(vm, m, 0);
        break;
    case ORC_MAP_PERCPU_HASH: case ORC_MAP_PERCPU_CGROUP_STORAGE:
        m->family = FAM_PERCPU_HASH;
        rc = hash_init(vm, m, 1);
        break;
    default:
        set_err(vm, "unsupported map type '%u'", type);
        free(m->spec);
        free(m);
        return -1;
    }
    if (rc) {
        set_err(vm, "map init: out of memory");
        return -1;
    }
    vm->maps = (orc_map **)realloc(vm->maps, sizeof(orc_map *) * (size_t)(vm->nmaps + 1));
    vm->maps[vm->nmaps] = m;
    return vm->nmaps++;
}

/* status codes for map ops: 0 ok, >0 errno (graceful), <0 fatal */
#define MAPOP_FATAL (-1)

/* LinuxArrayMap.Lookup :78-94 / LinuxPerCPUArrayMap.Lookup :235-241 / LinuxHashMap.Lookup
 * emulator_linux_map_hash.go:134-155 / LinuxPerCPUHashMap.Lookup :537-561 */
static int map_lookup(orc_vm *vm, orc_map *m, const uint8_t *key, uint32_t klen, int cpu, uint32_t *addr) {
    (void)vm;
    switch (m->family) {
    case FAM_ARRAY: {
        if (klen != 4) return MAPOP_FATAL;
        uint32_t k;
        memcpy(&k, key, 4);
        *addr = k >= m->spec->max_entries ? 0 : m->addr + k * m->spec->value_size;
        return 0;
    }
    case FAM_PERCPU_ARRAY:
        if (cpu < 0 || cpu >= m->nsubs) return MAPOP_FATAL;
        return map_lookup(vm, m->subs[cpu], key, klen, cpu, addr);
    case FAM_HASH: {
        if (klen != m->spec->key_size) return MAPOP_FATAL;
        int32_t idx = ht_find(m, key, NULL);
        *addr = idx < 0 ? 0 : m->values_addr[0] + (uint32_t)idx * m->spec->value_size;
        return 0;
    }
    case FAM_PERCPU_HASH: {
        if (klen != m->spec->key_size) return MAPOP_FATAL;
        if (cpu < 0 || cpu >= m->nvalues) return MAPOP_FATAL;
        int32_t idx = ht_find(m, key, NULL);
        *addr = idx < 0 ? 0 : m->values_addr[cpu] + (uint32_t)idx * m->spec->value_size;
        return 0;
    }
    }
    return MAPOP_FATAL;
}

/* Update: emulator_linux_map_array.go:97-113, :244-250; emulator_linux_map_hash.go:158-203, :564-612 */
static int map_update(orc_vm *vm, orc_map *m, const uint8_t *key, uint32_t klen, const uint8_t *val,
                      uint32_t vlen, uint32_t flags, int cpu) {
    (void)flags; /* Q10: flags are ignored by every map */
    switch (m->family) {
    case FAM_ARRAY: {
        if (klen != 4) return MAPOP_FATAL;
        if (vlen != m->spec->value_size) return MAPOP_FATAL;
        uint32_t k;
        memcpy(&k, key, 4);
        if (k >= m->spec->max_entries) return (int)E2BIG_ERRNO;
        if (pm_write(&m->backing, k * m->spec->value_size, val, vlen)) return MAPOP_FATAL;
        return 0;
    }
    case FAM_PERCPU_ARRAY:
        if (cpu < 0 || cpu >= m->nsubs) return MAPOP_FATAL;
        return map_update(vm, m->subs[cpu], key, klen, val, vlen, flags, cpu);
    case FAM_HASH:
    case FAM_PERCPU_HASH: {
        int percpu = m->family == FAM_PERCPU_HASH;
        if (klen != m->spec->key_size) return MAPOP_FATAL;
        if (vlen != m->spec->value_size) return MAPOP_FATAL;
        if (percpu && (cpu < 0 || cpu >= m->nvalues)) return MAPOP_FATAL;
        int32_t idx = ht_find(m, key, NULL);
        if (idx < 0) {
            if (m->fl_len == 0) return (int)E2BIG_ERRNO;
            idx = m->fl[m->fl_head];
            m->fl_head = (m->fl_head + 1) % m->fl_cap;
            m->fl_len--;
            ht_insert(m, key, idx);
        }
        if (pm_write(&m->keys, (uint32_t)idx * m->spec->key_size, key, klen)) return MAPOP_FATAL;
        if (pm_write(&m->values[percpu ? cpu : 0], (uint32_t)idx * m->spec->value_size, val, vlen)) return MAPOP_FATAL;
        return 0;
    }
    }
    return MAPOP_FATAL;
}

/* Delete: emulator_linux_map_hash.go:225-255, :634-664 (arrays are not LinuxMapDeleter) */
static int map_delete(orc_map *m, const uint8_t *key, uint32_t klen) {
    if (m->family != FAM_HASH && m->family != FAM_PERCPU_HASH) return MAPOP_FATAL;
    if (klen != m->spec->key_size) return MAPOP_FATAL;
    uint32_t pos;
    int32_t idx = ht_find(m, key, &pos);
    if (idx < 0) return 0;
    m->tidx[pos] = -2;
    m->tcount--;
    m->ntomb++;
    if (m->fl_len == m->fl_cap) abort(); /* panic("freelist is full") -- unreachable */
    m->fl[(m->fl_head + m->fl_len) % m->fl_cap] = idx;
    m->fl_len++;
    return 0;
}

int orc_map_update(orc_vm *vm, int id, const void *key, const void *value, uint32_t flags, int cpu) {
    orc_map *m = vm->maps[id];
    return map_update(vm, m, (const uint8_t *)key, m->spec->key_size, (const uint8_t *)value, m->spec->value_size, flags, cpu);
}
int orc_map_lookup(orc_vm *vm, int id, const void *key, int cpu, uint32_t *addr_out) {
    orc_map *m = vm->maps[id];
    return map_lookup(vm, m, (const uint8_t *)key, m->spec->key_size, cpu, addr_out);
}
int orc_map_delete(orc_vm *vm, int id, const void *key) {
    orc_map *m = vm->maps[id];
    return map_delete(m, (const uint8_t *)key, m->spec->key_size);
}
uint32_t orc_map_addr(orc_vm *vm, int id) {
    entry *e = mc_by_obj(vm, vm->maps[id]);
    return e ? e->addr : 0;
}
int orc_map_values(orc_vm *vm, int id, int cpu, void *out, size_t cap) {
    orc_map *m = vm->maps[id];
    plain_mem *b;
    switch (m->family) {
    case FAM_ARRAY: b = &m->backing; break;
    case FAM_PERCPU_ARRAY:
        if (cpu < 0 || cpu >= m->nsubs) return -1;
        b = &m->subs[cpu]->backing;
        break;
    case FAM_HASH: b = &m->values[0]; break;
    case FAM_PERCPU_HASH:
        if (cpu < 0 || cpu >= m->nvalues) return -1;
        b = &m->values[cpu];
        break;
    default: return -1;
    }
    if (cap < b->len) return -1;
    memcpy(out, b->b, b->len);
    return (int)b->len;
}
int orc_map_slots(orc_vm *vm, int id, int32_t *slot_out, uint8_t *keys_out, size_t cap_keys) {
    orc_map *m = vm->maps[id];
    if (m->family != FAM_HASH && m->family != FAM_PERCPU_HASH) return -1;
    uint32_t K = m->spec->key_size;
    int n = 0;
    for (uint32_t p = 0; p < m->tcap; p++) {
        if (m->tidx[p] < 0) continue;
        if ((size_t)n >= cap_keys) return -1;
        slot_out[n] = m->tidx[p];
        memcpy(keys_out + (size_t)n * K, m->tkeys + (size_t)p * K, K);
        n++;
    }
    return n;
}

/* ------------------------------------------------------------------------- */
/* Programs: VM.AddProgram, vm.go:98-139; RewriteProgram, emulator_linux_.go:292-339 */
/* ------------------------------------------------------------------------- */

int orc_prog_load(orc_vm *vm, const char *name, const uint8_t *raw, uint32_t n_slots,
                  const orc_reloc *relocs, uint32_t n_relocs) {
    program *p = (program *)calloc(1, sizeof *p);
    snprintf(p->name, sizeof p->name, "%s", name ? name : "");
    p->ins = (insn *)calloc(n_slots ? n_slots : 1, sizeof(insn));
    p->n = n_slots;
    /* cilium/ebpf v0.9.0 asm.Instruction.Unmarshal (little endian), then the Nop
     * re-inserted after every LD_IMM64 by AddProgram (vm.go:102-112). */
    for (uint32_t i = 0; i < n_slots; i++) {
        const uint8_t *b = raw + 8 * (size_t)i;
        insn *x = &p->ins[i];
        x->op = b[0];
        x->dst = b[1] & 0xf;
        x->src = b[1] >> 4;
        x->off = (int16_t)(uint16_t)(b[2] | (b[3] << 8));
        int32_t imm = (int32_t)((uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24));
        x->k = (int64_t)imm;
        if (x->op == 0x18) {
            if (i + 1 >= n_slots) {
                set_err(vm, "64bit immediate is missing second half");
                free(p->ins);
                free(p);
                return -1;
            }
            const uint8_t *c = raw + 8 * (size_t)(i + 1);
            if (c[0] | c[1] | c[2] | c[3]) {
                set_err(vm, "64bit immediate has non-zero fields");
                free(p->ins);
                free(p);
                return -1;
            }
            uint32_t hi = (uint32_t)c[4] | ((uint32_t)c[5] << 8) | ((uint32_t)c[6] << 16) | ((uint32_t)c[7] << 24);
            x->k = (int64_t)(((uint64_t)hi << 32) | (uint32_t)imm);
            i++;
            memset(&p->ins[i], 0, sizeof(insn)); /* asm.Instruction{OpCode: 0} */
        }
    }
    /* RewriteProgram: map references -> map object address */
    for (uint32_t r = 0; r < n_relocs; r++) {
        uint32_t s = relocs[r].slot;
        if (s >= p->n) {
            set_err(vm, "relocation slot %u out of range", s);
            free(p->ins);
            free(p);
            return -1;
        }
        insn *x = &p->ins[s];
        if (!(x->op == 0x18 && (x->src == 1 || x->src == 2))) continue; /* !IsLoadFromMap */
        if (relocs[r].map_id >= (uint32_t)vm->nmaps) {
            set_err(vm, "program references a map that does not exist in the emulator");
            free(p->ins);
            free(p);
            return -1;
        }
        entry *e = mc_by_obj(vm, vm->maps[relocs[r].map_id]);
        if (x->src == 1) x->k = (int64_t)e->addr;               /* PseudoMapFD */
        else x->k = (int64_t)e->addr + (int64_t)x->off;         /* PseudoMapValue (Q16) */
    }
    /* fixupJumpsAndCalls (vm.go:142-194) is the identity on raw bytecode whose call/jump
     * immediates are already relative; AddEntry(prog, 8) (vm.go:131). */
    if (mc_add(vm, p, K_PROG, 8, NULL)) {
        free(p->ins);
        free(p);
        return -1;
    }
    vm->progs = (program **)realloc(vm->progs, sizeof(program *) * (size_t)(vm->nprogs + 1));
    vm->progs[vm->nprogs] = p;
    return vm->nprogs++;
}

uint32_t orc_prog_addr(orc_vm *vm, int id) {
    entry *e = mc_by_obj(vm, vm->progs[id]);
    return e ? e->addr : 0;
}

uint32_t orc_mem_add_scratch(orc_vm *vm, uint32_t size) {
    plain_mem *m = pm_new(size);
    uint32_t a = 0;
    if (mc_add(vm, m, K_PLAIN, size, &a)) {
        pm_free(m);
        return 0;
    }
    vm->scratch = (plain_mem **)realloc(vm->scratch, sizeof(plain_mem *) * (size_t)(vm->nscratch + 1));
    vm->scratch[vm->nscratch++] = m;
    return a;
}
int orc_mem_read(orc_vm *vm, uint32_t addr, void *buf, uint32_t len) {
    uint32_t off;
    entry *e = mc_get(vm, addr, &off);
    if (!e) return ORC_ERR_MEM_UNRESOLVED;
    return vm_read(e, off, (uint8_t *)buf, len);
}
int orc_mem_write(orc_vm *vm, uint32_t addr, const void *buf, uint32_t len) {
    uint32_t off;
    entry *e = mc_get(vm, addr, &off);
    if (!e) return ORC_ERR_MEM_UNRESOLVED;
    return vm_write(e, off, (const uint8_t *)buf, len);
}
int orc_mem_load(orc_vm *vm, uint32_t addr, int size, uint64_t *out) {
    uint32_t off;
    entry *e = mc_get(vm, addr, &off);
    if (!e) return ORC_ERR_MEM_UNRESOLVED;
    return vm_load(e, off, size, out);
}

/* ------------------------------------------------------------------------- */
/* Registers, vm.go:407-466                                                    */
/* ------------------------------------------------------------------------- */

#define GET(reg, out)                                              \
    do {                                                           \
        if ((reg) > 10) return ORC_PANIC_BADREG;                   \
        (out) = p->R.r[(reg)];                                     \
    } while (0)
#define SET(reg, val)                                              \
    do {                                                           \
        if ((reg) == 10) return ORC_ERR_R10_WRITE;                 \
        if ((reg) > 10) return ORC_PANIC_BADREG;                   \
        p->R.r[(reg)] = (val);                                     \
    } while (0)

/* ------------------------------------------------------------------------- */
/* Instruction handlers                                                        */
/* ------------------------------------------------------------------------- */

/* Generated ALU handlers, inst_gen.go:7-225 (ADD..XOR, x{32,64}x{IMM,Reg}).
 * ALU32: uint64(uint32(dst) op uint32(x)); ALU64: dst op x with x = uint64(Constant). */
static int h_alu_gen(orc_proc *p, const insn *i) {
    int is64 = (i->op & 7) == 7;
    int reg = (i->op & 0x08) != 0;
    int aop = i->op & 0xf0;
    uint64_t d, s;
    GET(i->dst, d);
    if (reg) GET(i->src, s);
    else s = (uint64_t)i->k;
    uint64_t r;
    if (is64) {
        switch (aop) {
        case 0x00: r = d + s; break;
        case 0x10: r = d - s; break;
        case 0x20: r = d * s; break;
        case 0x30: if (s == 0) return ORC_PANIC_DIV0; r = d / s; break;
        case 0x40: r = d | s; break;
        case 0x50: r = d & s; break;
        case 0x60: r = s >= 64 ? 0 : d << s; break;   /* Go: shifts >= width yield 0 */
        case 0x70: r = s >= 64 ? 0 : d >> s; break;
        case 0x90: if (s == 0) return ORC_PANIC_DIV0; r = d % s; break;
        default: r = d ^ s; break; /* 0xa0 */
        }
    } else {
        uint32_t a = (uint32_t)d, b = (uint32_t)s, x;
        switch (aop) {
        case 0x00: x = a + b; break;
        case 0x10: x = a - b; break;
        case 0x20: x = a * b; break;
        case 0x30: if (b == 0) return ORC_PANIC_DIV0; x = a / b; break;
        case 0x40: x = a | b; break;
        case 0x50: x = a & b; break;
        case 0x60: x = b >= 32 ? 0 : a << b; break;   /* uint32(dst) << uint32(x) */
        case 0x70: x = b >= 32 ? 0 : a >> b; break;
        case 0x90: if (b == 0) return ORC_PANIC_DIV0; x = a % b; break;
        default: x = a ^ b; break;
        }
        r = (uint64_t)x;
    }
    SET(i->dst, r);
    return 0;
}

/* inst.go:86-94 (Q6: ALU32 NEG sign-extends) */
static int h_neg(orc_proc *p, const insn *i) {
    uint64_t d;
    GET(i->dst, d);
    uint64_t r;
    if ((i->op & 7) == 7) r = (uint64_t)(-(int64_t)d);
    else r = (uint64_t)(int64_t)(int32_t)(0u - (uint32_t)d);
    SET(i->dst, r);
    return 0;
}

/* inst.go:96-114 */
static int h_mov(orc_proc *p, const insn *i) {
    int is64 = (i->op & 7) == 7;
    uint64_t v;
    if (i->op & 0x08) {
        GET(i->src, v);
        if (!is64) v = (uint32_t)v;
    } else {
        v = is64 ? (uint64_t)i->k : (uint64_t)(uint32_t)i->k;
    }
    SET(i->dst, v);
    return 0;
}

/* inst.go:116-136 (Q5/Q6: Go signed shift; negative IMM count panics; ALU32 result sign-extends) */
static int h_arsh(orc_proc *p, const insn *i) {
    int is64 = (i->op & 7) == 7;
    uint64_t d, s;
    int reg = (i->op & 0x08) != 0;
    if (reg) {
        GET(i->src, s);
        GET(i->dst, d);
    } else {
        GET(i->dst, d);
        if (i->k < 0) return ORC_PANIC_SHIFT;
        s = (uint64_t)i->k;
    }
    uint64_t r;
    if (is64) {
        int64_t x = (int64_t)d;
        r = (uint64_t)(s >= 64 ? (x < 0 ? -1 : 0) : (x >> s));
    } else {
        int32_t x = (int32_t)(uint32_t)d;
        int32_t y = s >= 32 ? (x < 0 ? -1 : 0) : (x >> s);
        r = (uint64_t)(int64_t)y;
    }
    SET(i->dst, r);
    return 0;
}

static uint64_t bswap16(uint64_t x) { return ((x >> 8) & 0xff) | ((x & 0xff) << 8); }
static uint64_t bswap32(uint64_t x) {
    return ((x >> 24) & 0xff) | ((x >> 8) & 0xff00) | ((x << 8) & 0xff0000) | ((x << 24) & 0xff000000u);
}

/* inst.go:138-198 (Q4) */
static int h_end(orc_proc *p, const insn *i) {
    uint64_t d;
    GET(i->dst, d);
    int to_be = (i->op & 0x08) != 0;
    switch (i->k) {
    case 16: d = to_be ? (d & 0xffff) : bswap16(d & 0xffff); break;
    case 32: d = to_be ? (d & 0xffffffffu) : bswap32(d & 0xffffffffu); break;
    case 64: d = to_be ? (d >> 32) : bswap32(d >> 32); break;
    default: break;
    }
    SET(i->dst, d);
    return 0;
}

/* Conditional jumps, inst_gen.go:227-605 and inst.go:205-241.
 * width32: compare uint32/int32 views.  Taken => PC += Offset. */
static int jump_cond(int jop, uint64_t d, uint64_t s, int width32) {
    if (width32) {
        uint32_t a = (uint32_t)d, b = (uint32_t)s;
        int32_t sa = (int32_t)a, sb = (int32_t)b;
        switch (jop) {
        case 0x10: return a == b;
        case 0x20: return a > b;
        case 0x30: return a >= b;
        case 0x40: return (a & b) == 0; /* Q3: inverted JSET */
        case 0x50: return a != b;
        case 0x60: return sa > sb;
        case 0x70: return sa >= sb;
        case 0xa0: return a < b;
        case 0xb0: return a <= b;
        case 0xc0: return sa < sb;
        case 0xd0: return sa <= sb;
        }
    } else {
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
        case 0xd0: return sa <= sb;
        }
    }
    return 0;
}

/* width: 32 or 64.  Register-source handlers read Src first (inst_gen.go:246-247). */
static int h_jcond(orc_proc *p, const insn *i, int width32, int jop) {
    uint64_t d, s;
    if (i->op & 0x08) {
        GET(i->src, s);
        GET(i->dst, d);
    } else {
        GET(i->dst, d);
        s = (uint64_t)i->k;
    }
    if (jump_cond(jop, d, s, width32)) p->R.pc += i->off;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Helpers, emulator_linux_helpers.go                                          */
/* ------------------------------------------------------------------------- */

/* regToMap, emulator_linux_helpers.go:415-447 */
static orc_map *reg_to_map(orc_proc *p, uint64_t regval) {
    uint32_t off;
    entry *e = mc_get(p->vm, (uint32_t)regval, &off);
    if (!e) return NULL;
    if (is_linuxmap(e->kind)) return (orc_map *)e->obj;
    if (is_vmmem(e->kind)) {
        uint64_t a;
        if (vm_load(e, off, 4, &a)) return NULL;
        e = mc_get(p->vm, (uint32_t)a, &off);
        if (!e) return NULL;
        if (is_linuxmap(e->kind)) return (orc_map *)e->obj;
    }
    return NULL;
}

/* derefMapKey, :449-471 (also the value deref of :525-541) */
static int deref_bytes(orc_proc *p, uint64_t regval, uint32_t n, uint8_t *out) {
    uint32_t off;
    entry *e = mc_get(p->vm, (uint32_t)regval, &off);
    if (!e) return -1;
    if (!is_vmmem(e->kind)) return -1;
    if (vm_read(e, off, out, n)) return -1;
    return 0;
}

static int helper_lookup(orc_proc *p) { /* :477-504 */
    orc_map *m = reg_to_map(p, p->R.r[1]);
    if (!m) return ORC_ERR_HELPER_MAP_PTR;
    uint8_t kb[512];
    uint8_t *key = m->spec->key_size <= sizeof kb ? kb : (uint8_t *)malloc(m->spec->key_size);
    int rc = 0;
    if (deref_bytes(p, p->R.r[2], m->spec->key_size, key)) {
        rc = ORC_ERR_HELPER_KEY;
    } else {
        uint32_t a = 0;
        int r = map_lookup(p->vm, m, key, m->spec->key_size, p->cpu, &a);
        if (r < 0) rc = ORC_ERR_HELPER_MAP_OP;
        else if (r > 0) p->R.r[0] = (uint64_t)r; /* Q9 (lookups never return an errno) */
        else p->R.r[0] = a;
    }
    if (key != kb) free(key);
    return rc;
}

static int helper_update(orc_proc *p) { /* :506-555 */
    orc_map *m = reg_to_map(p, p->R.r[1]);
    if (!m) return ORC_ERR_HELPER_MAP_PTR;
    uint32_t K = m->spec->key_size, S = m->spec->value_size;
    uint8_t *key = (uint8_t *)malloc(K + 1), *val = (uint8_t *)malloc(S + 1);
    int rc = 0;
    if (deref_bytes(p, p->R.r[2], K, key)) rc = ORC_ERR_HELPER_KEY;
    else if (deref_bytes(p, p->R.r[3], S, val)) rc = ORC_ERR_HELPER_VALUE;
    else {
        int r = map_update(p->vm, m, key, K, val, S, (uint32_t)p->R.r[4], p->cpu);
        if (r < 0) rc = ORC_ERR_HELPER_MAP_OP;
        else p->R.r[0] = (uint64_t)(uint32_t)r; /* Q9: R0 = uint64(errno), positive */
    }
    free(key);
    free(val);
    return rc;
}

static int helper_delete(orc_proc *p) { /* :557-586 */
    orc_map *m = reg_to_map(p, p->R.r[1]);
    if (!m) return ORC_ERR_HELPER_MAP_PTR;
    if (m->family != FAM_HASH && m->family != FAM_PERCPU_HASH) return ORC_ERR_HELPER_MAP_OP;
    uint32_t K = m->spec->key_size;
    uint8_t *key = (uint8_t *)malloc(K + 1);
    int rc = 0;
    if (deref_bytes(p, p->R.r[2], K, key)) rc = ORC_ERR_HELPER_KEY;
    else {
        int r = map_delete(m, key, K);
        if (r < 0) rc = ORC_ERR_HELPER_MAP_OP;
        else p->R.r[0] = (uint64_t)(uint32_t)r;
    }
    free(key);
    return rc;
}

static int helper_tailcall(orc_proc *p) { /* :649-738 */
    if (p->tailcalls >= p->vm->max_tail_calls) {
        p->R.r[0] = (uint64_t)(0 - (uint64_t)EPERM_ERRNO);
        return 0;
    }
    orc_map *m = reg_to_map(p, p->R.r[2]);
    if (!m) return ORC_ERR_HELPER_MAP_PTR;
    if (m->spec->type != ORC_MAP_PROG_ARRAY || m->spec->key_size != 4) return ORC_ERR_HELPER_TAILCALL;
    if (m->family != FAM_ARRAY) return ORC_ERR_HELPER_TAILCALL;
    uint32_t k = (uint32_t)p->R.r[3];
    uint32_t ptr = 0;
    if (map_lookup(p->vm, m, (uint8_t *)&k, 4, p->cpu, &ptr) < 0) return ORC_ERR_HELPER_TAILCALL;
    uint32_t off;
    entry *e = mc_get(p->vm, ptr, &off);
    if (!e) {
        p->R.r[0] = (uint64_t)(0 - (uint64_t)EINVAL_ERRNO);
        return 0;
    }
    if (!is_vmmem(e->kind)) return ORC_ERR_HELPER_TAILCALL;
    uint64_t pa = 0;
    if (vm_load(e, off, 4, &pa)) pa = 0; /* error ignored (checks `ok` instead of err, :708) */
    e = mc_get(p->vm, (uint32_t)pa, &off);
    if (!e || e->kind != K_PROG) {
        p->R.r[0] = (uint64_t)(0 - (uint64_t)EINVAL_ERRNO);
        return 0;
    }
    p->prog = (program *)e->obj;
    p->R.pc = -1;
    p->tailcalls++;
    return 0;
}

/* bpf_xdp_adjust_tail, :842-861 (only the always-EINVAL prefix; a 20-byte PlainMemory ctx
 * is outside the engine's supported set) */
static int helper_xdp_adjust_tail(orc_proc *p) {
    uint32_t off;
    entry *e = mc_get(p->vm, (uint32_t)p->R.r[1], &off);
    if (!e || e->kind != K_PLAIN || ((plain_mem *)e->obj)->len != 20) {
        p->R.r[0] = (uint64_t)(0 - (uint64_t)EINVAL_ERRNO);
        return 0;
    }
    return ORC_ERR_ENGINE_HELPER;
}

static int helper_class(int32_t n) {
    /* emulatedLinuxHelpers table, emulator_linux_helpers.go:28-204: 0 nil, 1 emulated, 2 CantEmulate */
    static const int ce[] = {4, 14, 15, 16, 17, 22, 24, 27, 35, 36, 42, 45, 46, 47, 55, 56, 67, 69, 80,
                             112, 113, 114, 115, 119, 120, 122, 123, 128, 129, 141, 148, 151};
    static const int em[] = {1, 2, 3, 5, 7, 8, 9, 12, 25, 38, 65, 87, 88, 89, 125, 160};
    for (size_t k = 0; k < sizeof ce / sizeof ce[0]; k++) if (ce[k] == n) return 2;
    for (size_t k = 0; k < sizeof em / sizeof em[0]; k++) if (em[k] == n) return 1;
    return 0;
}

/* LinuxEmulator.CallHelperFunction, emulator_linux_.go:125-194 */
static int call_helper(orc_proc *p, int32_t n) {
    if (n < 0) return ORC_PANIC_HELPER_NEG;             /* replayableHelpers[n] index panic */
    if (n >= 176) return ORC_ERR_HELPER_UNIMPLEMENTED;  /* len(emulatedLinuxHelpers) == 176 */
    int c = helper_class(n);
    if (c == 0) return ORC_ERR_HELPER_UNIMPLEMENTED;
    if (c == 2) return ORC_ERR_HELPER_CANT_EMULATE;
    switch (n) {
    case 1: return helper_lookup(p);
    case 2: return helper_update(p);
    case 3: return helper_delete(p);
    case 8: p->R.r[0] = (uint64_t)(int64_t)p->cpu; return 0; /* :603-606 */
    case 12: return helper_tailcall(p);
    case 65: return helper_xdp_adjust_tail(p);
    default: return ORC_ERR_ENGINE_HELPER; /* ktime, prandom, skb_store_bytes, perf output, ... */
    }
}

/* inst.go:243-266 */
static int h_call(orc_proc *p, const insn *i) {
    if (i->src == 1) { /* PseudoCall: BPF-to-BPF */
        if (p->nframes >= ORC_MAX_FRAMES) return ORC_ERR_CALL_DEPTH;
        if (p->nframes == p->frames_cap) {
            p->frames_cap = p->frames_cap ? p->frames_cap * 2 : 4;
            p->frames = (regs *)realloc(p->frames, sizeof(regs) * (size_t)p->frames_cap);
        }
        p->frames[p->nframes++] = p->R;
        p->R.pc += (int64_t)i->k - 1;
        p->R.r[10] += (uint64_t)p->vm->frame_size;
        return 0;
    }
    return call_helper(p, (int32_t)i->k);
}

/* inst.go:277-296 */
static int h_exit(orc_proc *p) {
    if (p->nframes > 0) {
        regs *s = &p->frames[p->nframes - 1];
        p->R.pc = s->pc;
        p->R.r[6] = s->r[6];
        p->R.r[7] = s->r[7];
        p->R.r[8] = s->r[8];
        p->R.r[9] = s->r[9];
        p->nframes--;
        p->R.r[10] -= (uint64_t)p->vm->frame_size;
        return 0;
    }
    return EXIT_SIGNAL;
}

/* inst.go:298-363 */
static int h_ldx(orc_proc *p, const insn *i) {
    uint64_t s;
    GET(i->src, s);
    uint32_t addr = (uint32_t)(s + (uint64_t)(int64_t)i->off);
    uint32_t off;
    entry *e = mc_get(p->vm, addr, &off);
    if (!e) return ORC_ERR_MEM_UNRESOLVED;
    if (!is_vmmem(e->kind)) return ORC_ERR_MEM_NOT_VMMEM;
    uint64_t v;
    int rc = vm_load(e, off, size_bytes(i->op), &v);
    if (rc) return rc;
    SET(i->dst, v);
    return 0;
}

static int h_st(orc_proc *p, const insn *i, int reg) {
    uint64_t s = 0, d;
    if (reg) GET(i->src, s);
    GET(i->dst, d);
    if (!reg) s = (uint64_t)i->k;
    uint32_t addr = (uint32_t)(d + (uint64_t)(int64_t)i->off);
    uint32_t off;
    entry *e = mc_get(p->vm, addr, &off);
    if (!e) return ORC_ERR_MEM_UNRESOLVED;
    if (!is_vmmem(e->kind)) return ORC_ERR_MEM_NOT_VMMEM;
    return vm_store(e, off, s, size_bytes(i->op));
}

/* LinuxEmulator.CustomInstruction, emulator_linux_.go:198-288: LD_ABS / LD_IND read the
 * __sk_buff's packet (R6 must resolve to the *SKBuff entry), R0 = big-endian load at
 * skb.data + [src] + imm, then R1-R5 are clobbered.  Every failure is one error status. */
static uint32_t skb_data_addr(void *skb);
static int h_custom(orc_proc *p, const insn *i) {
    switch (i->op) {
    case 0x20: case 0x28: case 0x30: case 0x38:
    case 0x40: case 0x48: case 0x50: case 0x58: {
        uint32_t off;
        entry *e = mc_get(p->vm, (uint32_t)p->R.r[6], &off);
        if (!e || e->kind != K_SKB) return ORC_ERR_LDABS;
        uint32_t addr = skb_data_addr(e->obj) + (uint32_t)i->k;
        if (i->op & 0x40) {
            uint64_t s;
            GET(i->src, s); /* Registers.Get panics on a bad register (vm.go:431-432) */
            addr = skb_data_addr(e->obj) + (uint32_t)s + (uint32_t)i->k;
        }
        entry *pe = mc_get(p->vm, addr, &off);
        if (!pe || !is_vmmem(pe->kind)) return ORC_ERR_LDABS;
        uint64_t v;
        int rc = vm_load(pe, off, size_bytes(i->op), &v);
        if (rc == ORC_PANIC_SLICE) return rc; /* a Go panic propagates as a panic */
        if (rc) return ORC_ERR_LDABS;
        p->R.r[0] = v;
        for (int r = 1; r <= 5; r++) p->R.r[r] = 0;
        return 0;
    }
    }
    return ORC_ERR_UNSUPPORTED_OP;
}

/* Effective dispatch table (inst.go:15-78 after inst_gen.go:607-688), SURVEY Appendix A. */
static int exec_insn(orc_proc *p, const insn *i) {
    uint8_t op = i->op;
    switch (op) {
    case 0x00: return 0; /* instNop */
    case 0x18: SET(i->dst, (uint64_t)i->k); return 0; /* instLoad64Imm */
    case 0x61: case 0x69: case 0x71: case 0x79: return h_ldx(p, i);
    case 0x62: case 0x6a: case 0x72: case 0x7a: return h_st(p, i, 0);
    case 0x63: case 0x6b: case 0x73: case 0x7b: return h_st(p, i, 1);
    case 0x84: case 0x8c: case 0x87: case 0x8f: return h_neg(p, i);
    case 0xb4: case 0xbc: case 0xb7: case 0xbf: return h_mov(p, i);
    case 0xc4: case 0xcc: case 0xc7: case 0xcf: return h_arsh(p, i);
    case 0xd4: case 0xdc: return h_end(p, i);
    case 0x05: p->R.pc += i->off; return 0; /* instJump */
    case 0x85: return h_call(p, i);
    case 0x8d: return ORC_PANIC_CALLX;
    case 0x95: return h_exit(p);
    case 0xff: return h_jcond(p, i, 0, 0xd0); /* Q: 0xff = instJump64JSLEReg (last write wins) */
    default: break;
    }
    uint8_t cls = op & 7, hi = op & 0xf0;
    if (cls == 4 || cls == 7) { /* ALU / ALU64 generated ops */
        switch (hi) {
        case 0x00: case 0x10: case 0x20: case 0x30: case 0x40: case 0x50:
        case 0x60: case 0x70: case 0x90: case 0xa0:
            return h_alu_gen(p, i);
        }
        return h_custom(p, i);
    }
    if (cls == 5) { /* JMP: K = 64-bit; X = 32-bit (Q1) except JSET X (64-bit) */
        switch (hi) {
        case 0x10: case 0x20: case 0x30: case 0x50: case 0x60: case 0x70:
        case 0xa0: case 0xb0: case 0xc0: case 0xd0:
            return h_jcond(p, i, (op & 0x08) != 0, hi);
        case 0x40:
            return h_jcond(p, i, 0, hi);
        }
        return h_custom(p, i);
    }
    if (cls == 6) { /* JMP32: K = 32-bit; X = nil except JSET X (Q2) */
        switch (hi) {
        case 0x10: case 0x20: case 0x30: case 0x50: case 0x60: case 0x70:
        case 0xa0: case 0xb0: case 0xc0: case 0xd0:
            if (op & 0x08) return h_custom(p, i);
            return h_jcond(p, i, 1, hi);
        case 0x40:
            return h_jcond(p, i, 1, hi);
        }
        return h_custom(p, i);
    }
    return h_custom(p, i);
}

/* Process.Step, vm.go:291-340.  Returns 0 = continue, EXIT_SIGNAL = exited, >0 status. */
static int step(orc_proc *p, int32_t *err_pc) {
    program *prog = p->prog;
    if ((int64_t)prog->n <= p->R.pc) {
        *err_pc = (int32_t)p->R.pc;
        return ORC_ERR_PC_OOB;
    }
    if (p->R.pc < 0) {
        *err_pc = (int32_t)p->R.pc;
        return ORC_PANIC_PC;
    }
    int64_t pc = p->R.pc;
    int rc = exec_insn(p, &prog->ins[pc]);
    if (rc == EXIT_SIGNAL) return EXIT_SIGNAL;
    if (rc) {
        *err_pc = (int32_t)pc;
        return rc;
    }
    if ((int64_t)p->prog->n <= p->R.pc + 1) {
        p->R.pc = pc;
        *err_pc = (int32_t)pc;
        return ORC_ERR_PC_OOB;
    }
    p->R.pc++;
    return 0;
}

/* Process.Run, vm.go:343-360: before every step the ctx is checked (done = 0: not done, 1:
 * canceled, 2: deadline exceeded -- Run returns ctx.Err() with the process where it stopped); the
 * step budget is the engine's watchdog */
static int run(orc_proc *p, uint64_t budget, int done, uint32_t done_step, uint32_t *steps, int32_t *err_pc) {
    uint64_t n = 0;
    int st;
    *err_pc = -1;
    for (;;) {
        if (done && n >= done_step) {   /* select { case <-done: return ctx.Err() } (vm.go:346-349) */
            st = ORC_ERR_CANCELED - 1 + done;
            *err_pc = (int32_t)p->R.pc;
            break;
        }
        if (n == budget) {
            st = ORC_ERR_STEP_LIMIT;
            *err_pc = (int32_t)p->R.pc;
            break;
        }
        n++;
        int rc = step(p, err_pc);
        if (rc == 0) continue;
        st = rc == EXIT_SIGNAL ? ORC_OK : rc;
        break;
    }
    *steps = (uint32_t)n;
    return st;
}

/* VM.NewProcess, vm.go:198-235 (without a context) */
static orc_proc *proc_new(orc_vm *vm, int prog_id) {
    orc_proc *p = (orc_proc *)calloc(1, sizeof *p);
    p->vm = vm;
    p->prog = vm->progs[prog_id];
    uint32_t sz = (uint32_t)(vm->frame_count * vm->frame_size);
    p->stack.b = (uint8_t *)calloc(sz ? sz : 1, 1);
    p->stack.len = sz;
    p->cpu = -1;
    uint32_t a;
    mc_add(vm, &p->stack, K_PLAIN, sz, &a);
    p->R.r[10] = (uint64_t)(a + (uint32_t)vm->frame_size);
    return p;
}

orc_proc *orc_proc_new(orc_vm *vm, int prog_id) {
    if (prog_id < 0 || prog_id >= vm->nprogs) return NULL;
    return proc_new(vm, prog_id);
}

/* Process.Cleanup, vm.go:363-374 + LinuxContextXDP.Cleanup, context_xdp_md.go:118-133 */
static void proc_cleanup(orc_proc *p) {
    mc_del_obj(p->vm, &p->stack);
    if (p->has_ctx) {
        mc_del_obj(p->vm, p->pkt);
        mc_del_obj(p->vm, p->xdpmd);
        pm_free(p->pkt);
        pm_free(p->xdpmd);
    }
    free(p->stack.b);
    free(p->frames);
}

void orc_proc_free(orc_proc *p) {
    if (!p) return;
    /* LinuxContextSKBuff.Cleanup (context_sk_buff.go:110-119): the sk_buff entry only; the sock,
     * flow keys and packet entries leak */
    if (p->skb) {
        mc_del_obj(p->vm, p->skb);
        free(p->skb);
        p->skb = NULL;
    }
    proc_cleanup(p);
    free(p);
}

int orc_proc_set_cpu(orc_proc *p, int id) { /* vm.go:268-283 (Q18: id == V accepted) */
    if (id < 0) return -1;
    if (id > p->vm->vcpus) return -1;
    p->cpu = id;
    return 0;
}
uint64_t orc_proc_get_reg(orc_proc *p, int r) { return p->R.r[r]; }
void orc_proc_set_reg(orc_proc *p, int r, uint64_t v) { p->R.r[r] = v; }
int orc_proc_call_helper(orc_proc *p, int32_t helper) { return call_helper(p, helper); }

/* LinuxContextXDP.Load, context_xdp_md.go:47-115 */
static void xdp_load(orc_proc *p, const uint8_t *pkt, uint32_t L, uint32_t H, uint32_t T, int32_t ingress,
                     int32_t rxq, int32_t egress) {
    p->has_ctx = 1;
    p->pkt = pm_new(H + L + T);
    p->xdpmd = pm_new(24);
    memcpy(p->pkt->b + H, pkt, L);
    uint32_t pa;
    mc_add(p->vm, p->pkt, K_PLAIN, H + L + T, &pa);
    pm_store(p->xdpmd, 0, (uint64_t)pa + H, 4);
    pm_store(p->xdpmd, 4, (uint64_t)pa + H + L, 4);
    pm_store(p->xdpmd, 8, (uint64_t)pa + H, 4);
    pm_store(p->xdpmd, 12, (uint64_t)(int64_t)ingress, 4);
    pm_store(p->xdpmd, 16, (uint64_t)(int64_t)rxq, 4);
    pm_store(p->xdpmd, 20, (uint64_t)(int64_t)egress, 4);
    uint32_t xa;
    mc_add(p->vm, p->xdpmd, K_PLAIN, 24, &xa);
    p->R.r[1] = xa;
}

/* NewProcess(prog, &LinuxContextXDP{...}) for single-process stepping (vm.go:198-235) */
orc_proc *orc_proc_new_xdp(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t H, uint32_t T,
                           int32_t ingress, int32_t rxq, int32_t egress) {
    if (prog_id < 0 || prog_id >= vm->nprogs) return NULL;
    orc_proc *p = proc_new(vm, prog_id);
    xdp_load(p, pkt, L, H, T, ingress, rxq, egress);
    return p;
}

/* Process.Step (vm.go:291-340): 0 = continue, -1 = exited, > 0 = fatal status */
int orc_proc_step(orc_proc *p, int32_t *err_pc) {
    int32_t e = -1;
    const int rc = step(p, &e);
    if (err_pc) *err_pc = e;
    return rc;
}

int64_t orc_proc_get_pc(orc_proc *p) { return p->R.pc; }

int orc_proc_get_prog(orc_proc *p) {
    for (int i = 0; i < p->vm->nprogs; i++)
        if (p->vm->progs[i] == p->prog) return i;
    return -1;
}

int orc_run_xdp_batch(orc_vm *vm, int prog_id, const orc_xdp_batch *b, orc_results *out) {
    if (prog_id < 0 || prog_id >= vm->nprogs) {
        set_err(vm, "no program with id '%d' is loaded", prog_id);
        return -1;
    }
    uint64_t budget = b->step_budget ? b->step_budget : DEFAULT_BUDGET;
    for (uint32_t i = 0; i < b->n; i++) {
        uint32_t H = b->headroom_arr ? b->headroom_arr[i] : b->headroom;
        uint32_t T = b->tailroom_arr ? b->tailroom_arr[i] : b->tailroom;
        uint32_t L = b->pkt_len[i];
        uint8_t *mem = b->pkt_data + b->pkt_off[i];
        orc_proc *p = proc_new(vm, prog_id);
        xdp_load(p, mem + H, L, H, T, b->ingress_ifindex ? b->ingress_ifindex[i] : 0,
                 b->rx_queue_index ? b->rx_queue_index[i] : 0, b->egress_ifindex ? b->egress_ifindex[i] : 0);
        int cpu = b->cpu ? b->cpu[i] : 0;
        uint32_t steps = 0;
        int32_t epc = -1;
        int st;
        /* cpu -1: SetCPUID was never called, the process keeps cpuID -1 (vm.go:214); only the
         * per-CPU map operations fail then (emulator_linux_map_array.go:236-238) */
        if (cpu != -1 && orc_proc_set_cpu(p, cpu)) {
            st = ORC_ERR_NO_CPU;
        } else {
            st = run(p, budget, b->ctx_done ? b->ctx_done[i] : 0, b->ctx_done_step ? b->ctx_done_step[i] : 0, &steps, &epc);
        }
        if (out->r0) out->r0[i] = p->R.r[0];
        if (out->status) out->status[i] = (uint8_t)st;
        if (out->steps) out->steps[i] = steps;
        if (out->err_pc) out->err_pc[i] = st == ORC_OK ? -1 : epc;
        if (b->write_back) memcpy(mem, p->pkt->b, H + L + T);
        orc_proc_free(p);
    }
    return 0;
}

/* ========================================================================= */
/* sk_buff context: context_sk_buff.go + emulator_linux_sk_buff.go           */
/* ========================================================================= */

/* A net.IP as the reference holds it: kind 0 = make(net.IP, n) (zeros, cap n), 1 = nil
 * (cap 0), 2 = a slice of gopacket's copy of the packet starting at byte `off` (cap = L - off;
 * Go lets s[a:b] reach up to the capacity, so reads may run past the address), 3 = n bytes of
 * its own (a user-given SK's address as SK.UnmarshalJSON parsed it, emulator_linux_sk_buff.go:721-757). */
typedef struct {
    int kind;
    uint32_t off, n;
    uint8_t own[16];
} go_ip;

typedef struct sk_state { /* SK, emulator_linux_sk_buff.go:700-720 */
    uint32_t bound_dev_if, family, sock_type, protocol, mark, priority;
    go_ip src4, src6, dst4, dst6;
    uint32_t src_port, dst_port, state;
    int32_t rx_queue_mapping;
    const uint8_t *pkt; /* gopacket's copy of the packet (immutable) */
    uint32_t L;
} sk_state;

typedef struct fk_state { /* FlowKeys, :1003-1019 */
    uint16_t nhoff, thoff, addr_proto;
    uint8_t is_frag, is_first_frag, is_encap, ip_proto;
    uint16_t n_proto, sport, dport;
    uint32_t flags, flow_label;
} fk_state;

typedef struct skb_state { /* SKBuff, :35-103 */
    uint32_t len;
    uint16_t queue_mapping;
    uint8_t pkt_type;
    int vlan_present;
    uint16_t tc_index;
    uint32_t priority;
    int32_t skb_iif;
    uint32_t hash;
    uint16_t vlan_proto, vlan_tci;
    uint32_t napi_id, mark;
    uint16_t protocol;
    uint8_t cb[48];
    int64_t tstamp;     /* time.Time as Unix seconds; the zero Time is -62135596800 */
    uint32_t head, data, tail, end;
    uint32_t sk_addr, fk_addr, dev_ifindex;
    sk_state *sk;
    fk_state *fk;
    plain_mem *pkt;
} skb_state;

static uint32_t skb_data_addr(void *skb) { return ((skb_state *)skb)->data; }

static uint64_t to_size(uint64_t v, int n) {
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}

/* b2i over n bytes, big endian (the convertAccess helpers) */
static uint64_t be_bytes(const uint8_t *b, int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; k++) v = (v << 8) | b[k];
    return v;
}

/* copy(v, ip[start:start+n]) then b2i: a slice-bounds panic when start+n exceeds the capacity */
static int ip_load(const sk_state *sk, const go_ip *ip, uint64_t start, int n, uint64_t *v) {
    uint64_t cap = ip->kind == 0 || ip->kind == 3 ? ip->n : ip->kind == 1 ? 0 : (uint64_t)sk->L - ip->off;
    if (start + (uint64_t)n > cap) return ORC_PANIC_SLICE;
    uint8_t b[8] = {0};
    if (ip->kind == 2)
        for (int k = 0; k < n; k++) b[k] = sk->pkt[ip->off + start + k];
    if (ip->kind == 3)
        for (int k = 0; k < n; k++) b[k] = ip->own[start + k];
    *v = be_bytes(b, n);
    return 0;
}

#define RO() do { if (!load) return ORC_ERR_CTX_ACCESS; } while (0)

/* SKBuff.convertAccess, emulator_linux_sk_buff.go:295-676 */
static int skb_convert(skb_state *s, uint32_t off, int n, uint64_t *v, int load) {
    uint64_t val = *v;
    switch (off) {
    case 0: RO(); *v = to_size(s->len, n); return 0;                            /* len */
    case 4: RO(); *v = to_size(s->pkt_type & 7, n); return 0;                   /* pkt_type */
    case 8: if (load) *v = to_size(s->mark, n); else s->mark = (uint32_t)to_size(val, n); return 0;
    case 12: if (load) *v = to_size(s->queue_mapping, n); else s->queue_mapping = (uint16_t)to_size(val, n); return 0;
    case 16: RO(); *v = to_size(s->protocol, n); return 0;
    case 20: RO(); *v = s->vlan_present ? 1 : 0; return 0;
    case 24: RO(); *v = to_size(s->vlan_tci, n); return 0;
    case 28: RO(); *v = to_size(s->vlan_proto, n); return 0;
    case 32: if (load) *v = to_size(s->priority, n); else s->priority = (uint32_t)to_size(val, n); return 0;
    case 36: RO(); *v = to_size((uint64_t)(int64_t)s->skb_iif, n); return 0;  /* ingress_ifindex */
    case 40: RO(); *v = to_size(s->dev_ifindex, n); return 0;                 /* ifindex */
    case 44: if (load) *v = to_size(s->tc_index, n); else s->tc_index = (uint16_t)to_size(val, n); return 0;
    case 68: RO(); *v = to_size(s->hash, n); return 0;
    case 72: /* tc_classid: native u16 at cb[6:8] */
        if (load) *v = (uint64_t)(s->cb[6] | (s->cb[7] << 8));
        else { s->cb[6] = (uint8_t)val; s->cb[7] = (uint8_t)(val >> 8); }
        return 0;
    case 76: RO(); *v = to_size(s->data, n); return 0;                         /* data */
    case 80: RO(); *v = (uint64_t)s->cb[32] | ((uint64_t)s->cb[33] << 8) | ((uint64_t)s->cb[34] << 16) |
                        ((uint64_t)s->cb[35] << 24); return 0;                  /* data_end: cb[32:36] */
    case 84: RO(); *v = to_size(s->napi_id, n); return 0;
    case 88: RO(); *v = to_size(s->sk->family, n); return 0;
    case 132: RO(); *v = to_size(s->sk->dst_port, n); return 0;                /* remote_port */
    case 136: RO(); *v = to_size(s->sk->src_port, n); return 0;                /* local_port */
    case 140: RO(); *v = (uint64_t)(s->cb[36] | (s->cb[37] << 8)); return 0;  /* data_meta: cb[36:38] */
    case 144: case 148: RO(); *v = s->fk_addr; return 0;                       /* flow_keys */
    case 152: case 156:                                                         /* tstamp */
        if (load) *v = (uint64_t)s->tstamp; else s->tstamp = (int64_t)val;
        return 0;
    case 160: RO(); *v = (uint64_t)s->cb[0] | ((uint64_t)s->cb[1] << 8) | ((uint64_t)s->cb[2] << 16) |
                         ((uint64_t)s->cb[3] << 24); return 0;                  /* wire_len: cb[0:4] */
    case 164: case 176: case 184: case 188: return ORC_ERR_CTX_ACCESS;        /* gso_segs/gso_size/hwtstamp: "not yet implemented" */
    case 168: case 172: RO(); *v = s->sk_addr; return 0;                       /* sk */
    }
    if (off >= 48 && off < 68) {   /* cb[5]: load = cb[offset:size] -> low > high -> panic; store = no-op */
        if (load) return ORC_PANIC_SLICE;
        return 0;
    }
    if (off >= 92 && off < 96) { RO(); return ip_load(s->sk, &s->sk->dst4, off - 92, n, v); }   /* remote_ip4 */
    if (off >= 96 && off < 100) { RO(); return ip_load(s->sk, &s->sk->src4, off - 96, n, v); }  /* local_ip4 */
    if (off >= 100 && off < 116) { RO(); return ip_load(s->sk, &s->sk->dst6, off - 100, n, v); } /* remote_ip6 */
    if (off >= 116 && off < 132) { RO(); return ip_load(s->sk, &s->sk->src6, off - 116, n, v); } /* local_ip6 */
    return ORC_ERR_CTX_ACCESS; /* "invalid offset" */
}

/* SK.convertAccess, :772-918 */
static int sk_convert(sk_state *s, uint32_t off, int n, uint64_t *v, int load) {
    uint64_t val = *v;
    switch (off) {
    case 0: if (load) *v = to_size(s->bound_dev_if, n); else s->bound_dev_if = (uint32_t)to_size(val, n); return 0;
    case 4: RO(); *v = to_size(s->family, n); return 0;
    case 8: RO(); *v = to_size(s->sock_type, n); return 0;
    case 12: RO(); *v = to_size(s->protocol, n); return 0;
    case 16: if (load) *v = to_size(s->mark, n); else s->mark = (uint32_t)to_size(val, n); return 0;
    case 20: if (load) *v = to_size(s->priority, n); else s->priority = (uint32_t)to_size(val, n); return 0;
    case 44: RO(); *v = to_size(s->src_port, n); return 0;
    case 48: RO(); *v = to_size(s->dst_port, n); return 0;
    case 72: RO(); *v = to_size(s->state, n); return 0;
    case 76: RO(); *v = to_size((uint64_t)(int64_t)s->rx_queue_mapping, n); return 0;
    }
    if (off >= 24 && off < 28) { RO(); return ip_load(s, &s->src4, off - 24, n, v); }
    if (off >= 28 && off < 44) { RO(); return ip_load(s, &s->src6, off - 28, n, v); }
    if (off >= 52 && off < 56) { RO(); return ip_load(s, &s->dst4, off - 52, n, v); }
    if (off >= 56 && off < 72) {   /* dst_ipv6: start := offset - 17*4 (:889), a uint32 that wraps below 68 */
        RO();
        uint32_t start = off - 68;
        return ip_load(s, &s->dst6, (uint64_t)start, n, v);
    }
    return ORC_ERR_CTX_ACCESS;
}

/* FlowKeys.convertAccess, :1031-1175 */
static int fk_convert(fk_state *f, uint32_t off, int n, uint64_t *v, int load) {
    uint64_t val = *v;
#define FK_FIELD(fld, T) do { if (load) *v = to_size(f->fld, n); else f->fld = (T)to_size(val, n); return 0; } while (0)
    switch (off) {
    case 0: case 1: FK_FIELD(nhoff, uint16_t);
    case 2: case 3: FK_FIELD(thoff, uint16_t);
    case 4: case 5: FK_FIELD(addr_proto, uint16_t);
    case 6: FK_FIELD(is_frag, uint8_t);
    case 7: FK_FIELD(is_first_frag, uint8_t);
    case 8: FK_FIELD(is_encap, uint8_t);
    case 9: FK_FIELD(ip_proto, uint8_t);
    case 10: case 11: FK_FIELD(n_proto, uint16_t);
    case 12: case 13: FK_FIELD(sport, uint16_t);
    case 14: case 15: FK_FIELD(dport, uint16_t);
    case 32: case 33: case 34: case 35: FK_FIELD(flags, uint32_t);
    case 36: case 37: case 38: case 39: FK_FIELD(flow_label, uint32_t);
    }
#undef FK_FIELD
    if (off >= 16 && off < 32) return ORC_PANIC_SLICE; /* ip[offset:...] on a 16-byte slice, offset >= 16 */
    return ORC_ERR_CTX_ACCESS;
}

static int skb_access(void *obj, objkind kind, uint32_t off, int n, uint64_t *v, int load) {
    if (kind == K_SKB) return skb_convert((skb_state *)obj, off, n, v, load);
    if (kind == K_SK) return sk_convert((sk_state *)obj, off, n, v, load);
    return fk_convert((fk_state *)obj, off, n, v, load);
}

/* ---- SKBuffFromBytes (:108-265) over gopacket v1.1.19's eager decoding ------------------
 * gopacket is not vendored (go.mod pins v1.1.19); its decoders are restated for the layers
 * that decide the SKBuff fields: Ethernet (+802.3 length), Dot1Q/QinQ, IPv4 (+options),
 * IPv6 (+Routing / Destination-options headers), TCP, UDP, and UDP tunnels that would add a
 * second link / network layer (VXLAN 4789, Geneve 6081, GTPv1-U 2152).  Other layers
 * (ARP, LLC, ICMP, payloads) end the walk; they set no field.  Parity for this walk is
 * unpinned: no reference test calls SKBuffFromBytes. */
typedef struct {
    const uint8_t *pkt;
    uint32_t L;
    int err;                /* a second link / network / transport layer */
    int link, net, trans;
    uint16_t protocol, vlan_proto, vlan_tci;
    int vlan_present;
    uint32_t family;
    go_ip s4, d4, s6, d6;
    uint32_t sport, dport;
} skb_walk;

static uint16_t rd16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

static void walk_ethertype(skb_walk *w, uint32_t t, uint32_t o, uint32_t len);
static void walk_ethernet(skb_walk *w, uint32_t o, uint32_t len);
static void walk_ip(skb_walk *w, uint32_t o, uint32_t len);

static void walk_tcp(skb_walk *w, uint32_t o, uint32_t len) {
    /* decodeTCP adds the layer even when DecodeFromBytes fails; ports are read first */
    if (w->trans++) { w->err = 1; return; }
    if (len >= 20) {
        w->sport = rd16(w->pkt + o);
        w->dport = rd16(w->pkt + o + 2);
    }
}

static void walk_udp(skb_walk *w, uint32_t o, uint32_t len) {
    if (w->trans++) { w->err = 1; return; }
    if (len < 8) return;
    const uint8_t *d = w->pkt + o;
    w->sport = rd16(d);
    w->dport = rd16(d + 2);
    uint32_t ulen = rd16(d + 4), plen;
    if (ulen >= 8) plen = (ulen > len ? len : ulen) - 8;
    else if (ulen == 0) plen = len - 8;
    else return; /* "UDP packet too small" */
    if (plen == 0) return;
    uint32_t po = o + 8;
    /* NextLayerType: the destination port's layer type unless it is LayerTypePayload, else the
     * source port's (udp.go); gopacket's UDPPortLayerType table (ports.go) */
    static const uint32_t known[] = {53, 123, 4789, 67, 68, 546, 547, 5060, 6343, 6081, 3784, 2152, 623, 1812};
    uint32_t port = w->sport;
    for (unsigned k = 0; k < sizeof known / sizeof *known; k++)
        if (w->dport == known[k]) port = w->dport;
    const uint8_t *q = w->pkt + po;
    if (port == 4789) {        /* VXLAN: 8-byte header, then Ethernet */
        if (plen < 8) return;
        walk_ethernet(w, po + 8, plen - 8);
    } else if (port == 6081) { /* Geneve: 8 + options, then the protocol's EthernetType */
        if (plen < 8) return;
        uint32_t hl = 8 + (q[0] & 0x3f) * 4u;
        if (plen < hl) return;
        walk_ethertype(w, rd16(q + 2), po + hl, plen - hl);
    } else if (port == 2152) { /* GTPv1-U: 8 bytes (+4 with E/S/PN), then IPv4 / IPv6 */
        if (plen < 8) return;
        uint32_t hl = (q[0] & 0x07) ? 12 : 8;
        if ((q[0] & 0x04) || plen <= hl) return; /* extension headers: not restated */
        walk_ip(w, po + hl, plen - hl);
    }
}

static void walk_proto(skb_walk *w, uint32_t proto, uint32_t o, uint32_t len) {
    if (len == 0) return; /* NextDecoder with an empty payload decodes nothing */
    switch (proto) {
    case 6: walk_tcp(w, o, len); return;
    case 17: walk_udp(w, o, len); return;
    case 4: case 41: walk_ip(w, o, len); return; /* IPIP / IPv6-in-IP: a second network layer */
    }
}

static void walk_ipv4(skb_walk *w, uint32_t o, uint32_t len) {
    if (w->net++) { w->err = 1; return; }
    w->family = 2; /* AF_INET */
    if (len < 20) { w->s4.kind = 1; w->d4.kind = 1; return; } /* SrcIP / DstIP stay nil */
    const uint8_t *d = w->pkt + o;
    w->s4.kind = 2; w->s4.off = o + 12;
    w->d4.kind = 2; w->d4.off = o + 16;
    uint32_t ihl = d[0] & 0x0f, tl = rd16(d + 2);
    uint32_t ff = rd16(d + 6);
    if (tl == 0) tl = len;
    if (tl < 20 || ihl < 5 || ihl * 4 > tl) return;
    uint32_t dl = len;
    if (len > tl) dl = tl;
    else if (len < tl && ihl * 4 > len) return;
    /* options, ip4.go: a malformed option ends the decode */
    uint32_t q = 20;
    while (q < ihl * 4) {
        uint8_t t = d[q];
        if (t == 0) break;
        if (t == 1) { q++; continue; }
        if (ihl * 4 - q < 2) return;
        uint8_t ol = d[q + 1];
        if (ihl * 4 - q < ol) return;
        if (ol <= 2) return;
        q += ol;
    }
    if ((ff & 0x2000) || (ff & 0x1fff)) return; /* a fragment: LayerTypeFragment */
    walk_proto(w, d[9], o + ihl * 4, dl - ihl * 4);
}

static void walk_ipv6(skb_walk *w, uint32_t o, uint32_t len) {
    if (w->net++) { w->err = 1; return; }
    w->family = 10; /* AF_INET6 */
    if (len < 40) { w->s6.kind = 1; w->d6.kind = 1; return; }
    const uint8_t *d = w->pkt + o;
    w->s6.kind = 2; w->s6.off = o + 8;
    w->d6.kind = 2; w->d6.off = o + 24;
    uint32_t next = d[6], plen = rd16(d + 4);
    if (next == 0) return;  /* Hop-by-Hop / jumbograms: not restated */
    if (plen == 0) return;  /* "IPv6 length 0, but next header is ..." */
    uint32_t po = o + 40, pl = len - 40;
    if (pl > plen) pl = plen;
    for (int guard = 0; guard < 16; guard++) {
        if (next == 43 || next == 60) { /* Routing / Destination options: (d[1]+1)*8 bytes */
            if (pl < 2) return;
            uint32_t hl = (w->pkt[po + 1] + 1u) * 8;
            if (pl < hl) return;
            next = w->pkt[po];
            po += hl;
            pl -= hl;
            continue;
        }
        if (next == 44) return; /* Fragment */
        break;
    }
    walk_proto(w, next, po, pl);
}

static void walk_ip(skb_walk *w, uint32_t o, uint32_t len) { /* decodeIPv4orIPv6 */
    if (len == 0) return;
    uint32_t v = w->pkt[o] >> 4;
    if (v == 4) walk_ipv4(w, o, len);
    else if (v == 6) walk_ipv6(w, o, len);
}

static void walk_dot1q(skb_walk *w, uint32_t o, uint32_t len) {
    if (len < 4) return;
    const uint8_t *d = w->pkt + o;
    w->vlan_proto = rd16(d + 2); /* Dot1Q.Type: the inner EthernetType (:182) */
    w->vlan_tci = rd16(d);
    w->vlan_present = 1;
    walk_ethertype(w, rd16(d + 2), o + 4, len - 4);
}

/* LLC (llc.go) and SNAP: 802.3 frames reach a network layer through LLC 0xAA/0xAA + SNAP */
static void walk_llc(skb_walk *w, uint32_t o, uint32_t len) {
    if (len < 3) return;
    const uint8_t *d = w->pkt + o;
    uint32_t hl = 3;
    if (!(d[2] & 1) || (d[2] & 3) == 1) {  /* I- or S-format: 2-byte control */
        if (len < 4) return;
        hl = 4;
    }
    if ((d[0] & 0xfe) != 0xaa || (d[1] & 0xfe) != 0xaa) return;  /* not SNAP */
    if (len - hl == 0) return;
    if (len - hl < 5) return;
    walk_ethertype(w, rd16(d + hl + 3), o + hl + 5, len - hl - 5);
}

static void walk_ethertype(skb_walk *w, uint32_t t, uint32_t o, uint32_t len) {
    if (len == 0) return;
    switch (t) {
    case 0x0000: walk_llc(w, o, len); return;
    case 0x0800: case 0x86DD: walk_ip(w, o, len); return;
    case 0x8100: case 0x88a8: walk_dot1q(w, o, len); return;
    case 0x6558: walk_ethernet(w, o, len); return; /* transparent Ethernet bridging */
    }
}

static void walk_ethernet(skb_walk *w, uint32_t o, uint32_t len) {
    if (len < 14) return; /* "Ethernet packet too small": no layer */
    if (w->link++) { w->err = 1; return; }
    const uint8_t *d = w->pkt + o;
    uint32_t t = rd16(d + 12);
    uint32_t pl = len - 14;
    if (t < 0x0600) { /* 802.3 length: EthernetTypeLLC (0); the payload is trimmed to the length */
        if (pl > t) pl = t;
        t = 0;
    }
    if (w->link == 1) w->protocol = (uint16_t)t;
    walk_ethertype(w, t, o + 14, pl);
}

/* LinuxContextSKBuff.Load, context_sk_buff.go:42-107.  Returns 0 or ORC_ERR_CTX_LOAD. */
/* a user-given SK's net.IP: its own bytes, or nil */
static go_ip custom_ip(const orc_skb_custom *c, int k) {
    go_ip ip;
    memset(&ip, 0, sizeof ip);
    ip.kind = c->sk_ip_len[k] ? 3 : 1;
    ip.n = c->sk_ip_len[k] > 16 ? 16 : c->sk_ip_len[k];
    memcpy(ip.own, c->sk_ip[k], ip.n);
    return ip;
}

static int skb_load(orc_proc *p, const uint8_t *pkt, uint32_t L, uint32_t ifindex, const orc_skb_custom *custom) {
    orc_vm *vm = p->vm;
    skb_walk w;
    memset(&w, 0, sizeof w);
    w.pkt = pkt;
    w.L = L;
    w.s4.n = w.d4.n = 4;
    w.s6.n = w.d6.n = 16;
    walk_ethernet(&w, 0, L);
    if (w.err) return ORC_ERR_CTX_LOAD; /* "handling of multiple ... layers not supported" */
    skb_state *s = (skb_state *)calloc(1, sizeof *s);
    sk_state *sk = (sk_state *)calloc(1, sizeof *sk);
    fk_state *fk = (fk_state *)calloc(1, sizeof *fk);
    plain_mem *pm = (plain_mem *)calloc(1, sizeof *pm);
    uint8_t *copy = (uint8_t *)malloc(L ? L : 1);   /* gopacket's copy (NoCopy false) */
    memcpy(copy, pkt, L);
    pm->len = 32 + L + 64;
    pm->b = (uint8_t *)calloc(pm->len, 1);
    pm->big_endian = 1; /* ByteOrder: binary.BigEndian (:116-119) */
    memcpy(pm->b + 32, pkt, L);
    sk->family = w.family;
    sk->src4 = w.s4; sk->dst4 = w.d4; sk->src6 = w.s6; sk->dst6 = w.d6;
    sk->src_port = w.sport;
    sk->dst_port = w.dport;
    sk->state = 7; /* BPF_TCP_CLOSE */
    sk->pkt = copy;
    sk->L = L;
    /* context_sk_buff.go:53-66: a user-given SK replaces the one SKBuffFromBytes made (every
     * field, the addresses included); user-given FlowKeys are the flow keys the program sees */
    if (custom && (custom->flags & ORC_SKB_CUSTOM_SK)) {
        sk->bound_dev_if = custom->sk_bound_dev_if;
        sk->family = custom->sk_family;
        sk->sock_type = custom->sk_type;
        sk->protocol = custom->sk_protocol;
        sk->mark = custom->sk_mark;
        sk->priority = custom->sk_priority;
        sk->src4 = custom_ip(custom, 0);
        sk->dst4 = custom_ip(custom, 1);
        sk->src6 = custom_ip(custom, 2);
        sk->dst6 = custom_ip(custom, 3);
        sk->src_port = custom->sk_src_port;
        sk->dst_port = custom->sk_dst_port;
        sk->state = custom->sk_state;
        sk->rx_queue_mapping = custom->sk_rx_queue_mapping;
    }
    if (custom && (custom->flags & ORC_SKB_CUSTOM_FLOWKEYS)) {
        fk->nhoff = custom->fk_nhoff;
        fk->thoff = custom->fk_thoff;
        fk->addr_proto = custom->fk_addr_proto;
        fk->is_frag = custom->fk_is_frag;
        fk->is_first_frag = custom->fk_is_first_frag;
        fk->is_encap = custom->fk_is_encap;
        fk->ip_proto = custom->fk_ip_proto;
        fk->n_proto = custom->fk_n_proto;
        fk->sport = custom->fk_sport;
        fk->dport = custom->fk_dport;
        fk->flags = custom->fk_flags;
        fk->flow_label = custom->fk_flow_label;
    }
    s->len = L;
    s->protocol = w.protocol;
    s->vlan_proto = w.vlan_proto;
    s->vlan_tci = w.vlan_tci;
    s->vlan_present = w.vlan_present;
    s->tstamp = -62135596800ll; /* time.Time{}.Unix() */
    s->dev_ifindex = ifindex;
    s->sk = sk;
    s->fk = fk;
    s->pkt = pm;
    /* head = 0 + 32, data = 0 + 32, tail = len, end = len (skb_reset_tail_pointer before the reserve) */
    s->head = 32;
    s->data = 32;
    s->tail = L;
    s->end = L;
    /* the reference keeps these objects alive after Cleanup (only the sk_buff entry is deleted) */
    void *objs[] = {sk, fk, pm, pm->b, copy};
    if (vm->nleaks + 5 > vm->cap_leaks) {
        vm->cap_leaks = vm->cap_leaks ? 2 * vm->cap_leaks + 5 : 64;
        vm->leaks = (void **)realloc(vm->leaks, sizeof(void *) * (size_t)vm->cap_leaks);
    }
    for (int k = 0; k < 5; k++) vm->leaks[vm->nleaks++] = objs[k];
    p->skb = s;
    uint32_t sa, ska, fka, pa;
    if (mc_add(vm, s, K_SKB, 192, &sa)) return ORC_ERR_CTX_LOAD;
    if (mc_add(vm, sk, K_SK, 80, &ska)) return ORC_ERR_CTX_LOAD;
    s->sk_addr = ska;
    if (mc_add(vm, fk, K_FK, 40, &fka)) return ORC_ERR_CTX_LOAD;
    s->fk_addr = fka;
    if (mc_add(vm, pm, K_PLAIN, pm->len, &pa)) return ORC_ERR_CTX_LOAD;
    s->head += pa;
    s->data += pa;
    s->tail += pa;
    s->end += pa;
    /* computeDataPointers (:269-281): cb[28:32] = data, cb[32:36] = end, native order */
    for (int k = 0; k < 4; k++) {
        s->cb[28 + k] = (uint8_t)(s->data >> (8 * k));
        s->cb[32 + k] = (uint8_t)(s->end >> (8 * k));
    }
    p->R.r[1] = sa;
    return 0;
}

/* NewProcess(prog, &LinuxContextSKBuff{Packet, Dev}) for single-process stepping (vm.go:198-235,
 * context_sk_buff.go:42-107): NULL (with *status) when the context does not load */
orc_proc *orc_proc_new_skb(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t ifindex, int *status) {
    return orc_proc_new_skb_ctx(vm, prog_id, pkt, L, ifindex, NULL, status);
}

orc_proc *orc_proc_new_skb_ctx(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t ifindex,
                               const void *custom, int *status) {
    if (prog_id < 0 || prog_id >= vm->nprogs) return NULL;
    orc_proc *p = proc_new(vm, prog_id);
    const orc_skb_custom *c = (const orc_skb_custom *)custom;
    const int st = skb_load(p, pkt, L, ifindex, c && c->flags ? c : NULL);
    if (status) *status = st;
    if (st) {
        orc_proc_free(p);
        return NULL;
    }
    return p;
}

int orc_run_skb_batch(orc_vm *vm, int prog_id, const orc_skb_batch *b, orc_results *out) {
    if (prog_id < 0 || prog_id >= vm->nprogs) {
        set_err(vm, "no program with id '%d' is loaded", prog_id);
        return -1;
    }
    uint64_t budget = b->step_budget ? b->step_budget : DEFAULT_BUDGET;
    for (uint32_t i = 0; i < b->n; i++) {
        uint32_t L = b->pkt_len[i];
        uint8_t *mem = b->pkt_data + b->pkt_off[i];
        orc_proc *p = proc_new(vm, prog_id);
        uint32_t steps = 0;
        int32_t epc = -1;
        const orc_skb_custom *cu = b->custom && b->custom[i].flags ? &b->custom[i] : NULL;
        int st = skb_load(p, mem + 32, L, b->ifindex, cu);
        if (!st) {
            const int cpu = b->cpu ? b->cpu[i] : 0;
            if (cpu != -1 && orc_proc_set_cpu(p, cpu)) st = ORC_ERR_NO_CPU;   /* -1: never set */
            else st = run(p, budget, b->ctx_done ? b->ctx_done[i] : 0, b->ctx_done_step ? b->ctx_done_step[i] : 0, &steps, &epc);
        }
        if (out->r0) out->r0[i] = p->R.r[0];
        if (out->status) out->status[i] = (uint8_t)st;
        if (out->steps) out->steps[i] = steps;
        if (out->err_pc) out->err_pc[i] = st == ORC_OK ? -1 : epc;
        if (b->write_back && p->skb) memcpy(mem, p->skb->pkt->b, 32 + L + 64);
        /* Process.Cleanup (vm.go:363-374) + LinuxContextSKBuff.Cleanup (context_sk_buff.go:110-119):
         * the stack and the sk_buff entry only; the sock, flow keys and packet entries stay */
        if (p->skb) {
            mc_del_obj(vm, p->skb);
            free(p->skb);
            p->skb = NULL;
        }
        orc_proc_free(p);
    }
    return 0;
}
