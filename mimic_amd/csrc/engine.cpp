// engine.cpp -- host side of the MI355X batch-eBPF engine: the C ABI of include/mimic_amd.h.
//
// Mirrors the reference's setup-time objects (NewVM / LinuxEmulator.AddMap / VM.AddProgram,
// vm.go:54-139, emulator_linux_.go:67-116, emulator_linux_map_*.go Init) on the host and
// keeps their state on the device:
//  * the static part of the reference MemoryController (maps, programs) as a short segment
//    table -- entries are appended exactly as AddEntry would place them (first fit from
//    0x10000 with a one-byte gap; with no deletions that is "previous end + 1");
//  * every map backing in one device arena;
//  * the loaded programs as one decoded instruction array (DInsn, 16 B per slot).
// The per-packet part (NewProcess/Load/Run/Cleanup) is the kernel in interp.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mimic_amd.h"
#include "blkcache.h"
#include "layout.h"
#include "hashmap.h"
#include "jit.h"
#include "skb.h"

extern "C" int mimic_launch_xdp(const KParams *kp, const KParams *d_kp, hipStream_t st);
extern "C" int mimic_launch_xdp_resume(const KParams *kp, hipStream_t st);

extern "C" int mimic_launch_hash_rebuild(uint8_t *arena, const DMap *m, uint32_t force, hipStream_t st);
extern "C" int mimic_launch_hash_reset(uint8_t *arena, const DMap *m, hipStream_t st);
extern "C" int mimic_launch_hash_normalize(uint8_t *arena, const DMap *m, hipStream_t st);
extern "C" int mimic_launch_hash_compact(uint8_t *arena, const DMap *m, hipStream_t st);
extern "C" int mimic_launch_spread_reduce(const void *part, uint32_t nblocks, uint32_t lanes, uint32_t roww, uint32_t n,
                                          uint8_t *dst, uint64_t stride, hipStream_t st);
extern "C" int mimic_launch_sum_u64(const uint8_t *base, uint64_t stride, uint32_t nvals, uint32_t cpus, uint64_t *out,
                                    hipStream_t st);
extern "C" int mimic_launch_skb_gather(const uint8_t *const *mem, uint32_t n, uint64_t *drv, uint64_t *prefix,
                                       mimic_skb_custom *cust, const uint8_t *has_cust, hipStream_t st);
extern "C" int mimic_launch_skb_prep(const uint8_t *pkt_data, const uint64_t *pkt_off, const uint32_t *pkt_len,
                                     uint32_t n, uint64_t *rec, uint32_t rec_q, uint64_t *prefix, uint64_t *state,
                                     uint64_t init_base, uint32_t use_init, uint32_t rooms, uint32_t sparse,
                                     uint32_t *rooms_state, hipStream_t st);

namespace {

// Host image of one hash map's device index (hashmap.h): bucket records, freelist ring, counters
// and the VM-visible keys backing.  Host map operations (LinuxMap.Update / Lookup / Delete) run
// the sequential form of the device algorithm on this image -- the same hash, probe order and FIFO
// freelist, so every key gets the slot the device (and the reference) would give it -- without a
// device round trip; the image goes to the device in one upload before the device next uses the
// map (flush_host).  valid: the image equals or is newer than the device's (a launch that may
// write the table makes it stale: the next host operation downloads it again); dirty: newer.
//
// After such a launch the image is fetched on demand: the counters at once, bucket
// records and freelist positions a page at a time when an operation first reads them, everything
// left in one copy per region once an operation sequence has faulted MIRROR_BULK pages.  Host
// writes (records, ring positions, keys, values) are staged as arena writes (stage_write) and the
// counters once at flush: a few Updates between two batches move a few pages down and a few
// hundred bytes up, not the whole index both ways.
#define MIRROR_PAGE 8192u   // bytes of records / ring per fetch
#define MIRROR_BULK 32u     // faults after which the rest of the index comes in one copy per region
struct HashMirror {
    bool valid = false, dirty = false;
    std::vector<uint64_t> rec;
    std::vector<int32_t> ring;
    HashCtl ctl{};
    std::vector<uint8_t> rec_pg, ring_pg;   // per page: 1 = on the host
    bool all = true;                        // every page on the host
    uint32_t faults = 0;
};

// mimic_map_share: the VMs whose hash map of one spec is ONE table in the memory of the first
// (the owner); each member's offsets point into it from its own arena
struct ShareGroup {
    struct Member {
        void *vm;              // mimic_vm *
        uint32_t map;
        uint8_t *arena;        // that VM's arena when it joined (an arena that moves would strand the offsets)
    };
    std::vector<Member> members;
    bool owner_gone = false;   // the owner VM was destroyed: the table's memory is gone
};

struct HostMap {
    std::string name;
    uint32_t type, family, key_size, value_size, max_entries, datasec;
    uint32_t obj_addr;      // map object entry
    uint32_t backing_addr;  // cpu-0 backing entry
    uint32_t addr_period;   // per-CPU
    uint32_t ncpu;
    uint64_t dev_off;       // arena offset of the cpu-0 backing
    uint64_t dev_stride;    // arena distance between cpu backings
    // hash families (hashmap.h)
    uint64_t keys_dev_off, ht_dev_off;
    uint32_t keys_addr, ht_cap, rec_q, nlocks, fl_cap;
    // a delete may have left tombstones (hashmap.h): only then can the table need a rebuild
    mutable bool may_tomb = false;
    mutable bool pop_dirty = false;   // a pop-only launch left head / avail to normalise (hashmap.h)
    std::shared_ptr<HashMirror> mir;  // hash families: the host image of the index
    mutable std::shared_ptr<ShareGroup> share;   // mimic_map_share: one table with other VMs' maps
    mutable bool chunk = false;   // the VM's chunk map (layout.h HT_F_CHUNK), picked at the table upload
};

// can the JIT's lane value cache hold a vCPU's row of this map (jit.cpp analyze_vc)?
bool vc_row_ok(uint32_t family, uint32_t max_entries, uint32_t value_size) {
    const uint64_t rb = (uint64_t)max_entries * value_size;
    return family == FAM_PERCPU_ARRAY && rb > 0 && rb <= MIMIC_VC_MAX_ROW && (rb & 7) == 0;
}

struct HostProg {
    std::string name;
    std::vector<DInsn> ins;
    uint32_t addr;
};

// the completion marker of a released process block's last use on the VM's stream (one event may
// cover many blocks: mimic_process_free_many records one for the whole call)
struct HipFence : BlkFence {
    hipEvent_t ev = nullptr;
    hipStream_t st = nullptr;
    void wait() override {
        if (hipEventSynchronize(ev) != hipSuccess) {
            (void)hipGetLastError();
            hipStreamSynchronize(st);
        }
    }
    ~HipFence() override {
        if (ev) hipEventDestroy(ev);
    }
};

}  // namespace

struct mimic_vm {
    mimic_vm_settings s;
    std::string err;
    hipStream_t stream = nullptr;
    uint32_t next_addr = MIMIC_MEM_START;   // first-fit position after the static entries
    std::vector<HostMap> maps;
    std::vector<HostProg> progs;
    std::vector<Seg> segs;
    // device state
    uint8_t *arena = nullptr;
    uint64_t arena_size = 0, arena_cap = 0;
    DInsn *d_insns = nullptr;
    DProg *d_progs = nullptr;
    Seg *d_segs = nullptr;
    DMap *d_maps = nullptr;
    bool tables_dirty = true;
    bool prog_deletes = false;   // some loaded program calls map_delete_elem (helper 3)
    bool prog_updates = false;   // some loaded program calls map_update_elem (helper 2)
    uint8_t *priv = nullptr;
    uint64_t priv_bytes = 0;
    uint32_t priv_lanes = 0;
    uint32_t *d_sched_start = nullptr, *d_sched_pkts = nullptr;
    uint64_t sched_cap_start = 0, sched_cap_pkts = 0;
    uint64_t *d_lane_steps = nullptr;
    uint32_t lane_steps_cap = 0;
    // JIT kernels with deferred slow paths: one DeferRec per lane and the launch's marker word
    // (layout.h); the epoch numbers launches so that no flag is ever cleared
    DeferRec *d_defer = nullptr;
    uint32_t *d_defer_any = nullptr;
    uint32_t defer_cap = 0, defer_epoch = 0;
    uint32_t last_lanes = 0;
    hipStream_t last_stream = nullptr;
    // execution
    int exec_mode = MIMIC_EXEC_JIT;
    std::vector<DInsn> h_all;   // predecoded instruction slots of every program (host copy)
    std::vector<DProg> h_dp;
    hipFunction_t jit_fn[2] = {nullptr, nullptr};   // per CtxKind, generated on first use
    JitInfo jit_info[2]{};
    hipFunction_t jit_fn_cx[2] = {nullptr, nullptr};   // the same with the Run(ctx) check (launches given contexts)
    JitInfo jit_info_cx[2]{};
    // Process.Run tiering (process_advance): a fresh xdp_md process runs on the interpreter's
    // stepping kernel until the VM has made proc_jit_after Runs, then on the program set's
    // single-process JIT form (jit.cpp Gen::proc) -- a compiled program instead of ~0.7 us of
    // interpretation per step.  MIMIC_PROC_JIT=N at VM creation (default 32; 0 at once, -1
    // never).  proc_jit: 0 not built, 1 built and usable, -1 not usable for this program set
    int64_t proc_jit_after = 32;
    uint64_t proc_runs = 0;
    int proc_jit = 0;
    hipFunction_t jit_fn_proc = nullptr;
    JitInfo jit_info_proc{};
    // the spread kernel (jit.cpp analyze_spread, xdp_md only): 0 not built yet, 1 built, -1 the
    // program set does not allow it; spread_bad is the device word a spread launch marks when a
    // generic access reached per-CPU memory (spread_used: some launch could have marked it)
    int spread_state = 0;
    hipFunction_t jit_fn_spread = nullptr;
    JitInfo jit_info_spread{};
    // the owned form of the spread kernel (SpreadReq::own): state as spread_state; its LDS table rows
    int spread_own_state = 0;
    hipFunction_t jit_fn_spread_own = nullptr;
    JitInfo jit_info_spread_own{};
    uint32_t spread_own_rows = 0;
    uint32_t *d_spread_bad = nullptr;
    void *d_spread_part = nullptr;   // spread launches: the blocks' counter tables (mimic_spread_reduce_kernel)
    uint64_t spread_part_cap = 0;
    bool spread_used = false;
    bool comb_used = false;   // a launch ran a kernel with the hash maps' block combiner (HashCtl::comb_fault)
    // host map operations staged for the device (flush_host): value / array writes, deduplicated
    // per arena offset (a later write to the same bytes replaces the earlier one)
    struct PendWrite {
        uint64_t off;
        uint32_t n, at;
    };
    std::vector<PendWrite> pend;
    std::vector<uint8_t> pend_data;
    std::unordered_map<uint64_t, size_t> pend_at;
    bool host_dirty = false;   // some pending write or dirty hash image
    int spread_mode = -1;   // mimic_set_spread: -1 the default policy (env MIMIC_SPREAD), 0 never, 1 whenever allowed
    bool spread_lds = false;   // the spread kernel keeps a block's counters in LDS (else agent-scope atomics)
    int last_exec = 0;          // the kernel the last batch ran on
    // launch parameters of JIT kernels in device memory: a ring of slots written by
    // stream-ordered copies from pinned host memory (a repeated batch reuses its slot)
    static constexpr int KP_SLOTS = 64;
    KParams *d_kp = nullptr, *h_kp = nullptr;
    hipEvent_t kp_ev[KP_SLOTS] = {};
    bool kp_used[KP_SLOTS] = {};
    int kp_next = 0, kp_last = -1;
    hipStream_t kp_last_stream = nullptr;
    // host-resident pipeline (mimic_run_xdp_host): NB rotating device staging slots
    // (packet window, its descriptors, its results); launch parameters are copied on the H2D
    // stream too (kp_copy_stream), so no copy ever queues on the compute stream
    static constexpr int NB = 4;
    struct Slot {
        uint8_t *buf = nullptr;
        uint64_t *off = nullptr;
        uint32_t *len = nullptr;
        uint64_t *r0 = nullptr;
        uint8_t *st = nullptr;
        size_t cap_bytes = 0, cap_n = 0;
        hipEvent_t e_in = nullptr, e_k = nullptr, e_out = nullptr;
        bool used = false;
    } slot[NB];
    hipStream_t s_h2d = nullptr, s_h2d2 = nullptr, s_d2h = nullptr;   // sub-batches alternate H2D streams
    hipStream_t kp_copy_stream = nullptr;
    hipEvent_t kp_copy_ev = nullptr;
    // device-resident batches copy their launch parameters on a side stream: the copy runs while
    // the previous kernel does, so back-to-back batches with different parameters keep no copy
    // (and its completion latency) between their kernels on the compute stream
    hipStream_t s_kp = nullptr;
    hipEvent_t kp_side_ev = nullptr;
    // sk_buff batches (skb.h): per-packet records, their leak prefixes (skb.hip), and
    // the device word pair {next leak address, this batch's leak base}
    SkbRec *d_skb_rec = nullptr;
    uint64_t *d_skb_drv = nullptr;   // the prep kernel's derived record words, SKB_DERIVED_Q per packet
    uint64_t *d_skb_prefix = nullptr, *d_skb_state = nullptr;
    size_t skb_cap = 0;
    // mimic_process_run_many: the gathered descriptors, records, prefixes, custom entries and results
    // of the processes of one launch (one allocation, grown as needed)
    uint8_t *d_many = nullptr;
    size_t many_cap = 0;
    // single processes' memory blocks (proc_alloc): freed blocks are kept per power-of-two size and
    // handed to the next NewProcess, so a process costs no hipMalloc / hipFree once the VM is warm.
    // A block goes back with the fence of its last use on `stream` (null when that use is known to
    // be complete) and is handed out again only once the fence has passed; Cleanup may run on any
    // thread (ProcessPool's Handoff, __del__, a Go finaliser ...).
    // (blkcache.h has the rules; at most 256 MiB of free blocks are kept)
    BlkCache blk{256ull << 20};
    // process operations that enqueue work on `stream` (NewProcess, Run / Step, run_many, Packet)
    // hold run_mu and number their enqueues on seq (blkcache.h SeqClock)
    std::recursive_mutex run_mu;
    SeqClock seq;
    uint32_t proc_gen = 0;   // NewProcess counter: StepState::gen of each process
    bool skb_leaked = false;   // sock / flow-keys / packet entries of earlier sk_buff processes exist
    hipStream_t skb_stream = nullptr;
    bool skb_release_pending = false;   // mimic_skb_release ran: skb_ev marks the end of the released batches
    hipEvent_t skb_ev = nullptr;
    // runs with one context per packet (mimic_run_*_ctx): the packets' context word pointers, and
    // the stream of the last launch that reads them
    const uint32_t **d_cancel_pp = nullptr;
    size_t cancel_pp_cap = 0;
    hipStream_t cancel_pp_stream = nullptr;
};

// context.Context of Run (vm.go:343-360): a word the kernels read before each process's first step
// (runtime.h ctx_done) and the host sets -- on cancel(), or from a timer thread at the deadline.  The
// word is pinned, device-mapped host memory; without a device it is plain host memory (a context
// then works on the host, and no run accepts it).
struct mimic_ctx {
    uint32_t *word = nullptr;     // 0 = not done, 1 = canceled, 2 = deadline exceeded (the first wins)
    uint32_t *dword = nullptr;    // its device address (pinned only)
    bool pinned = false;
    std::mutex mu;
    std::condition_variable cv;
    bool closing = false;
    std::thread timer;
    // launches that read the word: freeing it waits for them (a kernel must never read freed
    // host memory)
    std::vector<hipEvent_t> uses;
};
static void ctx_set(mimic_ctx *c, uint32_t v) {
    uint32_t z = 0;   // Err() keeps the first reason (context.go: cancel of a done context is a no-op)
    __atomic_compare_exchange_n(c->word, &z, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
}
static uint32_t ctx_get(const mimic_ctx *c) { return __atomic_load_n(c->word, __ATOMIC_SEQ_CST); }


static int fail(mimic_vm *vm, int code, const char *fmt, ...) {
    if (vm) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        vm->err = buf;
    }
    return code;
}

#define HIP_OK(vm, call)                                                                        \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) return fail((vm), MIMIC_EDEVICE, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

static int skb_settle(mimic_vm *vm);

// the device copy of kp for a JIT launch on stream st (see mimic_vm::d_kp)
static int kp_slot(mimic_vm *vm, const KParams &kp, hipStream_t st, const KParams **out) {
    if (!vm->d_kp) {
        HIP_OK(vm, hipMalloc(&vm->d_kp, sizeof(KParams) * mimic_vm::KP_SLOTS));
        HIP_OK(vm, hipHostMalloc(&vm->h_kp, sizeof(KParams) * mimic_vm::KP_SLOTS));
        for (auto &e : vm->kp_ev) HIP_OK(vm, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    int slot = vm->kp_last;
    if (slot < 0 || st != vm->kp_last_stream || memcmp(&vm->h_kp[slot], &kp, sizeof kp) != 0) {
        // Every launch from a slot records the slot's event on its own stream right behind the
        // kernel (run_xdp_impl): a slot is reused once that event has passed, whatever stream the
        // caller uses next -- no device-wide wait when the caller changes streams, no reference to
        // a stream the caller may have destroyed.  Only the interpreter and MIMIC_JIT_KARG=0 JIT
        // kernels read their parameters from a slot; the hot JIT kernels take them by value.
        slot = vm->kp_next;
        vm->kp_next = (slot + 1) % mimic_vm::KP_SLOTS;
        if (vm->kp_used[slot]) HIP_OK(vm, hipEventSynchronize(vm->kp_ev[slot]));  // its last kernel is done
        vm->h_kp[slot] = kp;
        if (vm->kp_copy_stream) {   // the host pipeline: behind the sub-batch's own copies
            HIP_OK(vm, hipMemcpyAsync(vm->d_kp + slot, vm->h_kp + slot, sizeof kp, hipMemcpyHostToDevice, vm->kp_copy_stream));
            HIP_OK(vm, hipEventRecord(vm->kp_copy_ev, vm->kp_copy_stream));
            HIP_OK(vm, hipStreamWaitEvent(st, vm->kp_copy_ev, 0));
        } else {
            if (!vm->s_kp) {
                HIP_OK(vm, hipStreamCreateWithFlags(&vm->s_kp, hipStreamNonBlocking));
                HIP_OK(vm, hipEventCreateWithFlags(&vm->kp_side_ev, hipEventDisableTiming));
            }
            // the slot's earlier kernels are done (its event was waited for above)
            HIP_OK(vm, hipMemcpyAsync(vm->d_kp + slot, vm->h_kp + slot, sizeof kp, hipMemcpyHostToDevice, vm->s_kp));
            HIP_OK(vm, hipEventRecord(vm->kp_side_ev, vm->s_kp));
            HIP_OK(vm, hipStreamWaitEvent(st, vm->kp_side_ev, 0));
        }
        vm->kp_last = slot;
        vm->kp_last_stream = st;
    }
    *out = vm->d_kp + slot;
    return slot;
}

static uint32_t stack_size(const mimic_vm *vm) {
    return (uint32_t)(vm->s.stack_frame_size * vm->s.stack_frame_count);
}

// AddEntry for the static part: with no deletions the first fit is "after the last entry"
static uint32_t add_entry(mimic_vm *vm, uint32_t size) {
    uint32_t a = vm->next_addr;
    vm->next_addr = a + size + 1;
    return a;
}

static int arena_reserve(mimic_vm *vm, uint64_t bytes, uint64_t *off) {
    uint64_t need = (vm->arena_size + 255) & ~255ull;
    uint64_t end = need + bytes;
    if (end > vm->arena_cap) {
        uint64_t cap = std::max<uint64_t>(end, vm->arena_cap * 2);
        cap = std::max<uint64_t>(cap, 1 << 20);
        uint8_t *n = nullptr;
        HIP_OK(vm, hipMalloc(&n, cap));
        HIP_OK(vm, hipMemset(n, 0, cap));
        if (vm->arena) {
            HIP_OK(vm, hipMemcpy(n, vm->arena, vm->arena_size, hipMemcpyDeviceToDevice));
            HIP_OK(vm, hipFree(vm->arena));
        }
        vm->arena = n;
        vm->arena_cap = cap;
    }
    *off = need;
    vm->arena_size = end;
    return 0;
}

// Host predecode of one slot into a handler id + uniform facts (see layout.h).  Mirrors the
// effective dispatch table (inst.go:15-78 after inst_gen.go:607-688) and the
// order in which each handler reports errors; anything whose outcome can differ per lane goes
// to H_SLOW or to a fast handler that checks per lane.
static int helper_class(int32_t n) {  // emulator_linux_helpers.go:28-204
    static const int ce[] = {4, 14, 15, 16, 17, 22, 24, 27, 35, 36, 42, 45, 46, 47, 55, 56, 67, 69, 80,
                             112, 113, 114, 115, 119, 120, 122, 123, 128, 129, 141, 148, 151};
    static const int em[] = {1, 2, 3, 5, 7, 8, 9, 12, 25, 38, 65, 87, 88, 89, 125, 160};
    for (int v : ce) if (v == n) return 2;
    for (int v : em) if (v == n) return 1;
    return 0;
}

static uint32_t predecode(const DInsn &x, int64_t i, int64_t n) {
    const uint32_t op = x.w & 0xff, dst = (x.w >> 8) & 0xf, src = (x.w >> 12) & 0xf;
    const int64_t off = (int16_t)(x.w >> 16);
    const int32_t imm32 = (int32_t)(uint32_t)x.k;
    const uint32_t cls = op & 7, hi = op & 0xf0;
    const bool xs = (op & 8) != 0;
    const int64_t tgt = op == 0x85 ? i + (int64_t)imm32 : i + off + 1;  // after Step's PC++
    uint32_t a = 0;
    if (i + 1 < n) a |= AUX_FALL_OK;
    if (tgt >= 0 && tgt < n) a |= AUX_JT_OK;
    if (tgt < 0) a |= AUX_JT_NEG;
    auto err = [&](uint32_t st) { return a | H_ERR | (st << 16); };
    auto sz = [&](uint32_t o) -> uint32_t {
        switch (o & 0x18) { case 0x00: return 4; case 0x08: return 2; case 0x10: return 1; default: return 8; }
    };
    auto jcc_ok = [&](uint32_t jop) {
        switch (jop) {
        case 0x10: case 0x20: case 0x30: case 0x40: case 0x50: case 0x60: case 0x70:
        case 0xa0: case 0xb0: case 0xc0: case 0xd0: return true;
        default: return false;
        }
    };
    if (op == 0x00) return a | H_NOP;
    if (op == 0xff) {  // instJump64JSLEReg (Appendix A)
        if (src > 10 || dst > 10) return err(MIMIC_PANIC_BADREG);
        return a | H_JCC | AUX_X | (0xd0u << 16);
    }
    if (cls == 4 || cls == 7) {
        const bool is64 = cls == 7;
        const uint32_t H = is64 ? H_ALU64 : H_ALU32;
        switch (hi) {
        case 0x00: case 0x10: case 0x20: case 0x40: case 0x50: case 0x60: case 0x70: case 0xa0:
        case 0x30: case 0x90: {
            if (dst > 10 || (xs && src > 10)) return err(MIMIC_PANIC_BADREG);
            const bool div = hi == 0x30 || hi == 0x90;
            if (div && xs) return a | H_SLOW;                                   // per-lane div-by-zero
            if (div && (is64 ? x.k == 0 : (uint32_t)x.k == 0)) return err(MIMIC_PANIC_DIV0);
            if (dst == 10) return err(MIMIC_ERR_R10_WRITE);
            return a | H | (xs ? AUX_X : 0);
        }
        case 0x80:  // NEG
            if (dst > 10) return err(MIMIC_PANIC_BADREG);
            if (dst == 10) return err(MIMIC_ERR_R10_WRITE);
            return a | H;
        case 0xb0:  // MOV
            if ((xs && src > 10) || dst > 10) return err(MIMIC_PANIC_BADREG);
            if (dst == 10) return err(MIMIC_ERR_R10_WRITE);
            return a | H | (xs ? AUX_X : 0);
        case 0xc0:  // ARSH
            if (dst > 10 || (xs && src > 10)) return err(MIMIC_PANIC_BADREG);
            if (!xs && (int64_t)x.k < 0) return err(MIMIC_PANIC_SHIFT);
            if (dst == 10) return err(MIMIC_ERR_R10_WRITE);
            return a | H | (xs ? AUX_X : 0);
        case 0xd0:
            if (is64) return err(MIMIC_ERR_UNSUPPORTED_OP);
            return a | H_SLOW;  // END
        default:
            return err(MIMIC_ERR_UNSUPPORTED_OP);
        }
    }
    if (cls == 5 || cls == 6) {
        const bool j32 = cls == 6;
        if (!j32 && hi == 0x00) return xs ? err(MIMIC_ERR_UNSUPPORTED_OP) : (a | H_JA);
        if (!j32 && hi == 0x90) return xs ? err(MIMIC_ERR_UNSUPPORTED_OP) : (a | H_EXIT);
        if (!j32 && hi == 0x80) {
            if (xs) return err(MIMIC_PANIC_CALLX);
            if (src == 1) return a | H_CALL_LOCAL;
            if (imm32 < 0) return err(MIMIC_PANIC_HELPER_NEG);
            if (imm32 >= 176) return err(MIMIC_ERR_HELPER_UNIMPLEMENTED);
            const int hc = helper_class(imm32);
            if (hc == 0) return err(MIMIC_ERR_HELPER_UNIMPLEMENTED);
            if (hc == 2) return err(MIMIC_ERR_HELPER_CANT_EMULATE);
            switch (imm32) {
            case 1: case 2: case 3: case 8: case 12: case 65: return a | H_CALL;
            default: return err(MIMIC_ERR_ENGINE_HELPER);
            }
        }
        if (jcc_ok(hi)) {
            if (j32 && xs && hi != 0x40) return err(MIMIC_ERR_UNSUPPORTED_OP);  // Q2
            if (dst > 10 || (xs && src > 10)) return err(MIMIC_PANIC_BADREG);
            const bool w32 = j32 || (xs && hi != 0x40);                          // Q1
            return a | H_JCC | (w32 ? AUX_W32 : 0) | (xs ? AUX_X : 0) | (hi << 16);
        }
        return err(MIMIC_ERR_UNSUPPORTED_OP);
    }
    if (cls == 1) {
        if ((op & 0xe0) != 0x60) return err(MIMIC_ERR_UNSUPPORTED_OP);
        if (src > 10) return err(MIMIC_PANIC_BADREG);
        if (dst >= 10) return a | H_SLOW;  // memory errors come before the register error
        return a | H_LDX | (sz(op) << 24);
    }
    if (cls == 2 || cls == 3) {
        if ((op & 0xe0) != 0x60) return err(MIMIC_ERR_UNSUPPORTED_OP);
        if (dst > 10 || (cls == 3 && src > 10)) return err(MIMIC_PANIC_BADREG);
        return a | (cls == 2 ? H_ST : H_STX) | (sz(op) << 24);
    }
    // LD class
    if (op == 0x18) {
        if (dst > 10) return err(MIMIC_PANIC_BADREG);
        if (dst == 10) return err(MIMIC_ERR_R10_WRITE);
        return a | H_LDIMM;
    }
    if ((op & 0xe0) == 0x20 || (op & 0xe0) == 0x40)  // LD_ABS / LD_IND: CustomInstruction
        return a | H_LDABS | ((op & 0x40) ? AUX_X : 0) | (sz(op) << 24);
    return err(MIMIC_ERR_UNSUPPORTED_OP);
}

static DMap to_dmap(const HostMap &m) {
    DMap d{};
    d.family = m.family;
    d.type = m.type;
    d.key_size = m.key_size;
    d.value_size = m.value_size;
    d.max_entries = m.max_entries;
    d.datasec = m.datasec;
    d.obj_addr = m.obj_addr;
    d.backing_addr = m.backing_addr;
    d.addr_period = m.addr_period;
    d.ncpu = m.ncpu;
    d.dev_off = m.dev_off;
    d.dev_stride = m.dev_stride;
    d.keys_dev_off = m.keys_dev_off;
    d.keys_addr = m.keys_addr;
    d.ht_cap = m.ht_cap;
    d.ht_dev_off = m.ht_dev_off;
    d.rec_q = m.rec_q;
    d.nlocks = m.nlocks;
    d.fl_cap = m.fl_cap;
    d.hflags = m.chunk ? HT_F_CHUNK : 0u;
    return d;
}

static bool is_hash(const HostMap &m) { return m.family == FAM_HASH || m.family == FAM_PERCPU_HASH; }

// every program's slots with their predecoded facts, concatenated (interpreter + JIT input)
static void build_host_tables(const std::vector<HostProg> &progs, std::vector<DInsn> &all, std::vector<DProg> &dp) {
    all.clear();
    dp.clear();
    for (size_t pi = 0; pi < progs.size(); pi++) {
        auto &p = progs[pi];
        DProg d{};
        d.base = (uint32_t)all.size();
        d.n = (uint32_t)p.ins.size();
        d.addr = p.addr;
        dp.push_back(d);
        const int64_t n = (int64_t)p.ins.size();
        for (int64_t i = 0; i < n; i++) {
            DInsn x = p.ins[i];
            x.aux = predecode(x, i, n);
            all.push_back(x);
        }
    }
}

static int upload_tables(mimic_vm *vm) {
    if (!vm->tables_dirty) return 0;
    build_host_tables(vm->progs, vm->h_all, vm->h_dp);
    vm->prog_deletes = false;
    vm->prog_updates = false;
    for (auto &x : vm->h_all) {
        if (AUX_H(x.aux) == H_CALL && (uint32_t)x.k == 3) vm->prog_deletes = true;
        if (AUX_H(x.aux) == H_CALL && (uint32_t)x.k == 2) vm->prog_updates = true;
    }
    // map hints of LD_IMM64 constants that are map objects (AUX_MAPHINT): the JIT's inline
    // helpers check the map at run time, so a hint only selects a fast path
    for (auto &x : vm->h_all) {
        if (AUX_H(x.aux) != H_LDIMM || x.k > 0xffffffffull) continue;
        for (size_t m = 0; m < vm->maps.size() && m < 0xfffe; m++) {
            const HostMap &hm = vm->maps[m];
            if (hm.obj_addr == (uint32_t)x.k) {
                x.aux = (x.aux & 0xffffu) | ((uint32_t)(m + 1) << 16);
                break;
            }
        }
    }
    vm->jit_fn[0] = vm->jit_fn[1] = nullptr;
    vm->jit_fn_cx[0] = vm->jit_fn_cx[1] = nullptr;
    vm->jit_fn_proc = nullptr;
    vm->proc_jit = 0;
    vm->jit_fn_spread = nullptr;
    vm->spread_state = 0;
    vm->jit_fn_spread_own = nullptr;
    vm->spread_own_state = 0;
    std::vector<DInsn> all = vm->h_all;
    std::vector<DProg> dp = vm->h_dp;
    all.push_back(DInsn{0, 0, 0});  // keep the array non-empty
    std::vector<DMap> dm;
    // the chunk map (hashmap.h MIMIC_HASH_CHUNK): the first hash map not shared with another VM whose
    // compaction fits one kernel's LDS -- one per VM, so a block never waits for positions of one map
    // while it holds a chunk of another
    bool picked = false;
    for (auto &m : vm->maps) {
        m.chunk = !picked && m.family == FAM_HASH && !m.share && m.max_entries >= 1 && m.max_entries <= HT_CHUNK_MAXE;
        picked |= m.chunk;
    }
    for (auto &m : vm->maps) dm.push_back(to_dmap(m));
    if (dm.empty()) dm.push_back(DMap{});
    if (dp.empty()) dp.push_back(DProg{});
    std::vector<Seg> sg = vm->segs;   // sorted by address: resolve() binary-searches them
    std::sort(sg.begin(), sg.end(), [](const Seg &x, const Seg &y) { return x.lo < y.lo; });
    if (sg.empty()) sg.push_back(Seg{});
    hipFree(vm->d_insns);
    hipFree(vm->d_progs);
    hipFree(vm->d_segs);
    hipFree(vm->d_maps);
    vm->d_insns = nullptr;
    vm->d_progs = nullptr;
    vm->d_segs = nullptr;
    vm->d_maps = nullptr;
    HIP_OK(vm, hipMalloc(&vm->d_insns, all.size() * sizeof(DInsn)));
    HIP_OK(vm, hipMalloc(&vm->d_progs, dp.size() * sizeof(DProg)));
    HIP_OK(vm, hipMalloc(&vm->d_segs, sg.size() * sizeof(Seg)));
    HIP_OK(vm, hipMalloc(&vm->d_maps, dm.size() * sizeof(DMap)));
    HIP_OK(vm, hipMemcpy(vm->d_insns, all.data(), all.size() * sizeof(DInsn), hipMemcpyHostToDevice));
    HIP_OK(vm, hipMemcpy(vm->d_progs, dp.data(), dp.size() * sizeof(DProg), hipMemcpyHostToDevice));
    HIP_OK(vm, hipMemcpy(vm->d_segs, sg.data(), sg.size() * sizeof(Seg), hipMemcpyHostToDevice));
    HIP_OK(vm, hipMemcpy(vm->d_maps, dm.data(), dm.size() * sizeof(DMap), hipMemcpyHostToDevice));
    vm->tables_dirty = false;
    return 0;
}

// host-side MemoryController.GetEntry over the static entries
struct HostRef {
    int kind;          // 0 unresolved, 1 plain (arena), 2 not vmmem, 3 not datasec
    uint64_t dev_off;  // arena offset of region start
    uint32_t off, limit;
};

static HostRef host_resolve(const mimic_vm *vm, uint32_t a) {
    HostRef R{0, 0, 0, 0};
    for (const Seg &g : vm->segs) {
        if (a < g.lo || a > g.hi) continue;
        uint32_t off = a - g.lo;
        switch (g.kind) {
        case SEG_PLAIN: R = {1, g.dev_off, off, g.size}; break;
        case SEG_ARRAY_OBJ: R = {g.datasec ? 1 : 3, g.dev_off, off, g.size}; break;
        case SEG_MAP_OBJ: case SEG_PROG: R = {2, 0, 0, 0}; break;
        case SEG_PERCPU_ARRAY: {
            uint32_t c = off / g.period, r = off - c * g.period;
            uint64_t base = g.dev_off + (uint64_t)c * g.dev_stride;
            if (r <= 8) R = {g.datasec ? 1 : 3, base, r, g.size};
            else R = {1, base, r - 9, g.size};
            break;
        }
        case SEG_PERCPU_VALUES: {
            uint32_t c = off / g.period, r = off - c * g.period;
            R = {1, g.dev_off + (uint64_t)c * g.dev_stride, r, g.size};
            break;
        }
        }
        return R;
    }
    return R;
}

// cilium/ebpf v0.9.0 asm.Instruction.Unmarshal of raw slots + the Nop after LD_IMM64 (vm.go:102-112)
static int decode_program(const uint8_t *raw, uint32_t n_slots, std::vector<DInsn> &out, std::string *err) {
    out.assign(n_slots, DInsn{0, 0, 0});
    for (uint32_t i = 0; i < n_slots; i++) {
        const uint8_t *b = raw + 8ull * i;
        uint32_t op = b[0], dst = b[1] & 0xf, src = b[1] >> 4;
        uint16_t off = (uint16_t)(b[2] | (b[3] << 8));
        int32_t imm;
        memcpy(&imm, b + 4, 4);
        DInsn d{};
        d.w = op | (dst << 8) | (src << 12) | ((uint32_t)off << 16);
        d.k = (uint64_t)(int64_t)imm;
        if (op == 0x18) {
            if (i + 1 >= n_slots) {
                *err = "64bit immediate is missing second half";
                return -1;
            }
            const uint8_t *c = b + 8;
            if (c[0] | c[1] | c[2] | c[3]) {
                *err = "64bit immediate has non-zero fields";
                return -1;
            }
            uint32_t hi;
            memcpy(&hi, c + 4, 4);
            d.k = ((uint64_t)hi << 32) | (uint32_t)imm;
            out[i] = d;
            out[++i] = DInsn{0, 0, 0};
            continue;
        }
        out[i] = d;
    }
    return 0;
}

extern "C" {

int mimic_abi_version(void) { return MIMIC_ABI_VERSION; }

const char *mimic_last_error(const mimic_vm *vm) { return vm ? vm->err.c_str() : "null vm"; }

int mimic_vm_create(const mimic_vm_settings *settings, mimic_vm **out) {
    if (!settings || !out) return MIMIC_EINVAL;
    if (settings->vcpus <= 0) return MIMIC_EINVAL;
    mimic_vm *vm = new mimic_vm();
    vm->s = *settings;
    if (vm->s.stack_frame_size <= 0) vm->s.stack_frame_size = 256;
    if (vm->s.stack_frame_count <= 0) vm->s.stack_frame_count = 8;
    if (vm->s.vcpu_count <= 0) {
        vm->s.vcpu_begin = 0;
        vm->s.vcpu_count = vm->s.vcpus;
    }
    if (vm->s.vcpu_begin < 0 || vm->s.vcpu_begin + vm->s.vcpu_count > vm->s.vcpus) {
        delete vm;
        return MIMIC_EINVAL;
    }
    if (stack_size(vm) % 8 != 0 || stack_size(vm) > (1u << 20)) {
        delete vm;
        return MIMIC_EINVAL;
    }
    vm->exec_mode = settings->exec_mode;
    if (vm->exec_mode == MIMIC_EXEC_DEFAULT) {
        const char *e = getenv("MIMIC_EXEC");
        vm->exec_mode = (e && !strcmp(e, "interp")) ? MIMIC_EXEC_INTERP : MIMIC_EXEC_JIT;
    }
    if (const char *pj = getenv("MIMIC_PROC_JIT")) vm->proc_jit_after = *pj ? atoll(pj) : 32;
    if (vm->exec_mode != MIMIC_EXEC_INTERP && vm->exec_mode != MIMIC_EXEC_JIT) {
        delete vm;
        return MIMIC_EINVAL;
    }
    if (hipSetDevice(vm->s.device) != hipSuccess || hipStreamCreateWithFlags(&vm->stream, hipStreamNonBlocking) != hipSuccess) {
        delete vm;
        return MIMIC_EDEVICE;
    }
    *out = vm;
    return 0;
}

void mimic_vm_destroy(mimic_vm *vm) {
    if (!vm) return;
    hipSetDevice(vm->s.device);
    // everything this VM enqueued, on any stream (its own, side streams, callers' streams), ends
    // before its memory -- device blocks, pinned process state, the arena -- is released
    hipDeviceSynchronize();
    for (auto &m : vm->maps) {   // leave the shared tables (an owner takes its table's memory along)
        if (!m.share) continue;
        auto &mem = m.share->members;
        if (!mem.empty() && mem[0].vm == vm) m.share->owner_gone = true;
        for (size_t k = 0; k < mem.size(); k++)
            if (mem[k].vm == vm) {
                if (k == 0) hipDeviceSynchronize();   // the members' launches on the owner's table end first
                mem.erase(mem.begin() + (long)k);
                break;
            }
        m.share.reset();
    }
    vm->blk.drain([](Blk &b) {
        hipFree(b.dev);
        if (b.host) hipHostFree(b.host);
    });
    hipFree(vm->arena);
    hipFree(vm->d_insns);
    hipFree(vm->d_progs);
    hipFree(vm->d_segs);
    hipFree(vm->d_maps);
    hipFree(vm->priv);
    hipFree(vm->d_sched_start);
    hipFree(vm->d_sched_pkts);
    hipFree(vm->d_lane_steps);
    hipFree(vm->d_spread_bad);
    hipFree(vm->d_spread_part);
    hipFree(vm->d_cancel_pp);
    hipFree(vm->d_defer);
    hipFree(vm->d_defer_any);
    hipFree(vm->d_kp);
    if (vm->h_kp) hipHostFree(vm->h_kp);
    for (auto &sl : vm->slot) {
        hipFree(sl.buf);
        hipFree(sl.off);
        hipFree(sl.len);
        hipFree(sl.r0);
        hipFree(sl.st);
        for (hipEvent_t e : {sl.e_in, sl.e_k, sl.e_out})
            if (e) hipEventDestroy(e);
    }
    if (vm->kp_copy_ev) hipEventDestroy(vm->kp_copy_ev);
    if (vm->kp_side_ev) hipEventDestroy(vm->kp_side_ev);
    if (vm->s_kp) hipStreamDestroy(vm->s_kp);
    hipFree(vm->d_skb_rec);
    hipFree(vm->d_skb_drv);
    hipFree(vm->d_skb_prefix);
    hipFree(vm->d_many);
    hipFree(vm->d_skb_state);
    if (vm->s_h2d) hipStreamDestroy(vm->s_h2d);
    if (vm->s_h2d2) hipStreamDestroy(vm->s_h2d2);
    if (vm->s_d2h) hipStreamDestroy(vm->s_d2h);
    for (auto &e : vm->kp_ev)
        if (e) hipEventDestroy(e);
    if (vm->skb_ev) hipEventDestroy(vm->skb_ev);
    if (vm->stream) hipStreamDestroy(vm->stream);
    delete vm;
}

static void mirror_fresh(const HostMap &m);
static_assert(sizeof(mimic_skb_custom) == 136, "mimic_skb_custom: the layout _lib.SKB_CUSTOM_DTYPE and the oracle use");

// MapSpecToLinuxMap (emulator_linux_map.go:57-113) + Init + AddMap
int mimic_map_create(mimic_vm *vm, const mimic_map_spec *spec, uint32_t *map_id) {
    if (!vm || !spec || !map_id) return MIMIC_EINVAL;
    if (vm->skb_leaked)   // first fit would now place it in the freed stack / sk_buff hole or after the leaks
        return fail(vm, MIMIC_ENOTSUP, "adding maps after sk_buff batches is not supported (mimic_skb_release first)");
    hipSetDevice(vm->s.device);
    if (int rc = skb_settle(vm)) return rc;
    std::string name = spec->name ? spec->name : "";
    for (auto &m : vm->maps)
        if (m.name == name) return fail(vm, MIMIC_EINVAL, "map with name '%s' already exists in emulator", name.c_str());
    HostMap m{};
    m.name = name;
    m.type = spec->type;
    m.key_size = spec->key_size;
    m.value_size = spec->value_size;
    m.max_entries = spec->max_entries;
    m.datasec = (spec->flags & MIMIC_MAP_F_DATASEC) ? 1 : 0;
    const uint32_t id = (uint32_t)vm->maps.size();
    const uint64_t vbytes = (uint64_t)spec->max_entries * spec->value_size;
    if (vbytes > 0xffffffffull) return fail(vm, MIMIC_EINVAL, "map too large");
    const uint32_t ES = (uint32_t)vbytes;
    switch (spec->type) {
    case 2: case 3: case 12: case 14: case 15: case 16: case 17: case 8: case 20: {
        // LinuxArrayMap.Init, emulator_linux_map_array.go:30-54
        m.family = FAM_ARRAY;
        int rc = arena_reserve(vm, ES, &m.dev_off);
        if (rc) return rc;
        m.obj_addr = add_entry(vm, 8);
        m.backing_addr = add_entry(vm, ES);
        m.ncpu = 1;
        Seg o{};
        o.lo = m.obj_addr;
        o.hi = m.obj_addr + 8;
        o.kind = SEG_ARRAY_OBJ;
        o.id = id;
        o.dev_off = m.dev_off;
        o.size = ES;
        o.datasec = m.datasec;
        vm->segs.push_back(o);
        Seg b{};
        b.lo = m.backing_addr;
        b.hi = m.backing_addr + ES;
        b.kind = SEG_PLAIN;
        b.id = id;
        b.dev_off = m.dev_off;
        b.size = ES;
        vm->segs.push_back(b);
        break;
    }
    case 6: {
        // LinuxPerCPUArrayMap.Init, emulator_linux_map_array.go:185-215
        m.family = FAM_PERCPU_ARRAY;
        const uint32_t V = (uint32_t)vm->s.vcpus;
        int rc = arena_reserve(vm, (uint64_t)ES * V, &m.dev_off);
        if (rc) return rc;
        m.dev_stride = ES;
        m.obj_addr = add_entry(vm, 8);
        Seg o{};
        o.lo = m.obj_addr;
        o.hi = m.obj_addr + 8;
        o.kind = SEG_MAP_OBJ;
        o.id = id;
        vm->segs.push_back(o);
        const uint32_t first = vm->next_addr;
        const uint64_t period = (uint64_t)ES + 10;
        if ((uint64_t)first + period * V > 0xffffffffull) return fail(vm, MIMIC_ENOMEM, "out of memory (32-bit address space)");
        vm->next_addr = (uint32_t)(first + period * V);
        m.backing_addr = first + 9;
        m.addr_period = (uint32_t)period;
        m.ncpu = V;
        Seg g{};
        g.lo = first;
        g.hi = (uint32_t)(first + period * (V - 1) + 9 + ES);
        g.kind = SEG_PERCPU_ARRAY;
        g.id = id;
        g.dev_off = m.dev_off;
        g.size = ES;
        g.period = (uint32_t)period;
        g.count = V;
        g.datasec = m.datasec;
        g.dev_stride = ES;
        vm->segs.push_back(g);
        break;
    }
    case 1: case 13: case 18: case 19: case 24: case 25: case 26: case 28: case 29:
    case 5: case 21: {
        // LinuxHashMap.Init (emulator_linux_map_hash.go:43-97) / LinuxPerCPUHashMap.Init (:439-500)
        const bool percpu = spec->type == 5 || spec->type == 21;
        m.family = percpu ? FAM_PERCPU_HASH : FAM_HASH;
        const uint64_t kbytes = (uint64_t)spec->max_entries * spec->key_size;
        if (kbytes > 0xffffffffull) return fail(vm, MIMIC_EINVAL, "map too large");
        const uint32_t EK = (uint32_t)kbytes;
        const uint32_t V = percpu ? (uint32_t)vm->s.vcpus : 1u;
        m.ncpu = V;
        m.dev_stride = ES;
        int rc = arena_reserve(vm, (uint64_t)ES * V, &m.dev_off);
        if (!rc) rc = arena_reserve(vm, EK, &m.keys_dev_off);
        // device index: capacity for E live keys at load <= 1/2
        m.ht_cap = 16;
        while (m.ht_cap < 2ull * spec->max_entries + 2) m.ht_cap <<= 1;
        m.rec_q = 1 + (spec->key_size + 7) / 8;
        // stripe locks: 4 per bucket (up to 2^22).  A lane's lock is picked by its key's hash, so
        // lanes inserting one key serialise and other keys collide only by chance.  The cfg-4
        // inserting launch (E = 131 072, 2^19 buckets): 2^12 locks 2.0 ms, 2^16 0.53 ms, 2^19
        // 0.44 ms, 2^21 0.41 ms (tools/run_insert_knobs.sh; MIMIC_HASH_LOCKS_LOG2 = v sets 2^v)
        static const int lk_log2 = [] {
            const char *e = getenv("MIMIC_HASH_LOCKS_LOG2");
            const int v = e ? atoi(e) : 0;
            return v >= 4 && v <= 26 ? v : 0;
        }();
        m.nlocks = lk_log2 ? 1u << lk_log2 : (uint32_t)std::min<uint64_t>(4ull * m.ht_cap, 1ull << 22);
        m.fl_cap = 16;
        while (m.fl_cap < 2ull * spec->max_entries + 2) m.fl_cap <<= 1;
        // index region (hashmap.h h_table): records | rebuild copy | locks | freelist ring | HashCtl
        const uint64_t rec_bytes = (uint64_t)m.ht_cap * m.rec_q * 8;
        const uint64_t lock_off = 2 * rec_bytes, fl_off = lock_off + (uint64_t)m.nlocks * 4,
                       ctl_off = (fl_off + (uint64_t)m.fl_cap * 4 + 127) & ~127ull;   // hashmap.h h_ctl
        // (+ the chunked reservations' slot bits, slot buckets and handed-back remainders)
        if (!rc) rc = arena_reserve(vm, ctl_off + sizeof(HashCtl) + ht_ext_bytes(spec->max_entries), &m.ht_dev_off);
        if (rc) return rc;
        HIP_OK(vm, hipMemset(vm->arena + m.ht_dev_off, 0xff, rec_bytes));
        HIP_OK(vm, hipMemset(vm->arena + m.ht_dev_off + ctl_off + sizeof(HashCtl), 0, ht_ext_bytes(spec->max_entries)));
        std::vector<int32_t> fl(m.fl_cap, -1);
        for (uint32_t i = 0; i < spec->max_entries; i++) fl[i] = (int32_t)i;  // freelist <- 0..E-1 (:61-64)
        HIP_OK(vm, hipMemcpy(vm->arena + m.ht_dev_off + fl_off, fl.data(), fl.size() * 4, hipMemcpyHostToDevice));
        HashCtl c{};
        c.head = 0;
        c.tail = spec->max_entries;
        c.avail = (int32_t)spec->max_entries;
        HIP_OK(vm, hipMemcpy(vm->arena + m.ht_dev_off + ctl_off, &c, sizeof c, hipMemcpyHostToDevice));
        m.mir = std::make_shared<HashMirror>();
        mirror_fresh(m);
        auto plain = [&](uint32_t lo, uint32_t size, uint64_t dev_off) {
            Seg b{};
            b.lo = lo;
            b.hi = lo + size;
            b.kind = SEG_PLAIN;
            b.id = id;
            b.dev_off = dev_off;
            b.size = size;
            vm->segs.push_back(b);
        };
        auto obj = [&]() {
            m.obj_addr = add_entry(vm, 8);
            Seg o{};
            o.lo = m.obj_addr;
            o.hi = m.obj_addr + 8;
            o.kind = SEG_MAP_OBJ;
            o.id = id;
            vm->segs.push_back(o);
        };
        if (percpu) {  // values per cpu first, then the map object, then the keys
            const uint32_t first = vm->next_addr;
            const uint64_t period = (uint64_t)ES + 1;
            if ((uint64_t)first + period * V > 0xffffffffull) return fail(vm, MIMIC_ENOMEM, "out of memory (32-bit address space)");
            vm->next_addr = (uint32_t)(first + period * V);
            m.backing_addr = first;
            m.addr_period = (uint32_t)period;
            Seg g{};
            g.lo = first;
            g.hi = (uint32_t)(first + period * (V - 1) + ES);
            g.kind = SEG_PERCPU_VALUES;
            g.id = id;
            g.dev_off = m.dev_off;
            g.size = ES;
            g.period = (uint32_t)period;
            g.count = V;
            g.dev_stride = ES;
            vm->segs.push_back(g);
            obj();
            m.keys_addr = add_entry(vm, EK);
            plain(m.keys_addr, EK, m.keys_dev_off);
        } else {       // map object, keys, values
            obj();
            m.keys_addr = add_entry(vm, EK);
            plain(m.keys_addr, EK, m.keys_dev_off);
            m.backing_addr = add_entry(vm, ES);
            plain(m.backing_addr, ES, m.dev_off);
        }
        break;
    }
    default:
        return fail(vm, MIMIC_ENOTSUP, "unsupported map type '%u'", spec->type);
    }
    vm->maps.push_back(m);
    vm->tables_dirty = true;
    *map_id = id;
    return 0;
}

static int map_check(mimic_vm *vm, uint32_t id) {
    if (!vm) return MIMIC_EINVAL;
    if (id >= vm->maps.size()) return fail(vm, MIMIC_ENOENT, "no map %u", id);
    hipSetDevice(vm->s.device);
    return 0;
}

// cpu-resolved backing offset (array / per-CPU array / hash values / per-CPU hash values);
// returns <0 on error (fatal in the reference)
static int array_cpu(mimic_vm *vm, const HostMap &m, int32_t cpu, uint64_t *base) {
    if (m.family == FAM_PERCPU_ARRAY || m.family == FAM_PERCPU_HASH) {
        if (cpu < 0 || (uint32_t)cpu >= m.ncpu) return fail(vm, MIMIC_EINVAL, "invalid CPU ID");
        *base = m.dev_off + (uint64_t)cpu * m.dev_stride;
    } else {
        *base = m.dev_off;
    }
    return 0;
}

// wait for the last batch before touching map state from the host
static int settle(mimic_vm *vm) {
    if (int rc = skb_settle(vm)) return rc;
    if (vm->last_stream) HIP_OK(vm, hipStreamSynchronize(vm->last_stream));
    return 0;
}

// ---------------------------------------------------------------------------------------------
// host map operations (HashMirror): the index region's layout (hashmap.h h_table)
// ---------------------------------------------------------------------------------------------
static void ht_offsets(const HostMap &m, uint64_t *rec_bytes, uint64_t *fl_off, uint64_t *ctl_off) {
    *rec_bytes = (uint64_t)m.ht_cap * m.rec_q * 8;
    *fl_off = 2 * *rec_bytes + (uint64_t)m.nlocks * 4;
    *ctl_off = (*fl_off + (uint64_t)m.fl_cap * 4 + 127) & ~127ull;
}

// a freshly created table: every bucket EMPTY, the freelist 0..E-1 (emulator_linux_map_hash.go:56-64)
static void mirror_fresh(const HostMap &m) {
    HashMirror &x = *m.mir;
    x.rec.assign((size_t)m.ht_cap * m.rec_q, ~0ull);
    x.ring.assign(m.fl_cap, -1);
    for (uint32_t i = 0; i < m.max_entries; i++) x.ring[i] = (int32_t)i;
    x.ctl = HashCtl{};
    x.ctl.head = 0;
    x.ctl.tail = m.max_entries;
    x.ctl.avail = (int32_t)m.max_entries;
    x.rec_pg.assign(((size_t)m.ht_cap * m.rec_q * 8 + MIRROR_PAGE - 1) / MIRROR_PAGE, 1);
    x.ring_pg.assign(((size_t)m.fl_cap * 4 + MIRROR_PAGE - 1) / MIRROR_PAGE, 1);
    x.all = true;
    x.faults = 0;
    x.valid = true;
    x.dirty = false;
}

// the device's table as the image's source (after the last batch): the counters now, head / avail
// normalised as mimic_hash_normalize_kernel would (a pop-only launch may leave head past tail);
// records and ring pages when first read (mirror_page)
static int mirror_ensure(mimic_vm *vm, const HostMap &m) {
    HashMirror &x = *m.mir;
    if (x.valid) return 0;
    int rc = settle(vm);
    if (rc) return rc;
    uint64_t rb, fo, co;
    ht_offsets(m, &rb, &fo, &co);
    x.rec.resize((size_t)m.ht_cap * m.rec_q);
    x.ring.resize(m.fl_cap);
    x.rec_pg.assign((rb + MIRROR_PAGE - 1) / MIRROR_PAGE, 0);
    x.ring_pg.assign(((size_t)m.fl_cap * 4 + MIRROR_PAGE - 1) / MIRROR_PAGE, 0);
    x.all = false;
    x.faults = 0;
    HIP_OK(vm, hipMemcpy(&x.ctl, vm->arena + m.ht_dev_off + co, sizeof(HashCtl), hipMemcpyDeviceToHost));
    if (x.ctl.head > x.ctl.tail) x.ctl.head = x.ctl.tail;
    x.ctl.avail = (int32_t)(x.ctl.tail - x.ctl.head);
    x.valid = true;
    x.dirty = false;
    return 0;
}

// byte range [lo, hi) of a region (records at 0, ring at fo) on the host: the missing pages of it
// come down (all of both regions once the operations have faulted MIRROR_BULK times)
static int mirror_pages(mimic_vm *vm, const HostMap &m, bool ring, uint64_t lo, uint64_t hi) {
    HashMirror &x = *m.mir;
    if (x.all) return 0;
    uint64_t rb, fo, co;
    ht_offsets(m, &rb, &fo, &co);
    const uint8_t *base = vm->arena + m.ht_dev_off;
    std::vector<uint8_t> &pg = ring ? x.ring_pg : x.rec_pg;
    const uint64_t size = ring ? (uint64_t)m.fl_cap * 4 : rb;
    uint8_t *host = ring ? (uint8_t *)x.ring.data() : (uint8_t *)x.rec.data();
    for (uint64_t q = lo / MIRROR_PAGE; q * MIRROR_PAGE < hi; q++) {
        if (pg[q]) continue;
        if (++x.faults > MIRROR_BULK) {   // the rest of both regions at once
            for (int reg = 0; reg < 2; reg++) {
                std::vector<uint8_t> &pp = reg ? x.ring_pg : x.rec_pg;
                uint8_t *h = reg ? (uint8_t *)x.ring.data() : (uint8_t *)x.rec.data();
                const uint64_t sz = reg ? (uint64_t)m.fl_cap * 4 : rb, off = reg ? fo : 0;
                for (size_t a = 0; a < pp.size();) {   // runs of absent pages
                    if (pp[a]) { a++; continue; }
                    size_t b = a;
                    while (b < pp.size() && !pp[b]) b++;
                    const uint64_t s0 = (uint64_t)a * MIRROR_PAGE, s1 = std::min<uint64_t>((uint64_t)b * MIRROR_PAGE, sz);
                    HIP_OK(vm, hipMemcpy(h + s0, base + off + s0, s1 - s0, hipMemcpyDeviceToHost));
                    for (size_t c = a; c < b; c++) pp[c] = 1;
                    a = b;
                }
            }
            x.all = true;
            return 0;
        }
        const uint64_t s0 = q * MIRROR_PAGE, s1 = std::min<uint64_t>(s0 + MIRROR_PAGE, size);
        HIP_OK(vm, hipMemcpy(host + s0, base + (ring ? fo : 0) + s0, s1 - s0, hipMemcpyDeviceToHost));
        pg[q] = 1;
    }
    return 0;
}
// bucket record p / ring position at, on the host
static int mirror_rec(mimic_vm *vm, const HostMap &m, uint32_t p) {
    const uint64_t b = (uint64_t)p * m.rec_q * 8;
    return mirror_pages(vm, m, false, b, b + (uint64_t)m.rec_q * 8);
}
static int mirror_ring(mimic_vm *vm, const HostMap &m, uint64_t at) {
    const uint64_t b = (at & (m.fl_cap - 1)) * 4;
    return mirror_pages(vm, m, true, b, b + 4);
}

// a host write of n bytes at arena offset off, applied before the device next reads the arena.
// The writes of one flush land in parallel (one scatter launch): a later write of the same offset
// and size replaces the earlier one; callers never stage two writes of different sizes that overlap.
static void stage_write(mimic_vm *vm, uint64_t off, const void *src, uint32_t n) {
    if (!n) return;
    auto it = vm->pend_at.find(off);
    if (it != vm->pend_at.end() && vm->pend[it->second].n == n) {
        memcpy(vm->pend_data.data() + vm->pend[it->second].at, src, n);
    } else {
        vm->pend_at[off] = vm->pend.size();
        vm->pend.push_back({off, n, (uint32_t)vm->pend_data.size()});
        vm->pend_data.insert(vm->pend_data.end(), (const uint8_t *)src, (const uint8_t *)src + n);
    }
    vm->host_dirty = true;
}

extern "C" int mimic_launch_scatter(uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *at,
                                    const uint8_t *data, uint32_t n, hipStream_t st);

// Everything host map operations staged goes to the device (after the last batch): dirty hash
// images in one copy per region, pending writes as one scatter launch (a few: plain copies).
static int flush_host(mimic_vm *vm) {
    if (!vm->host_dirty) return 0;
    int rc = settle(vm);
    if (rc) return rc;
    for (auto &m : vm->maps) {   // the records, ring positions and keys went out as staged writes
        if (!m.mir || !m.mir->dirty) continue;
        HashMirror &x = *m.mir;
        uint64_t rb, fo, co;
        ht_offsets(m, &rb, &fo, &co);
        stage_write(vm, m.ht_dev_off + co, &x.ctl, sizeof(HashCtl));
        x.dirty = false;
        m.pop_dirty = false;   // the uploaded counters are normalised
    }
    const size_t n = vm->pend.size();
    if (n && n <= 8) {
        for (auto &w : vm->pend) HIP_OK(vm, hipMemcpy(vm->arena + w.off, vm->pend_data.data() + w.at, w.n, hipMemcpyHostToDevice));
    } else if (n) {
        std::vector<uint64_t> offs(n);
        std::vector<uint32_t> lens(n), at(n);
        for (size_t k = 0; k < n; k++) {
            offs[k] = vm->pend[k].off;
            lens[k] = vm->pend[k].n;
            at[k] = vm->pend[k].at;
        }
        const size_t bytes = n * 16 + vm->pend_data.size() + 16;
        uint8_t *d = nullptr;
        HIP_OK(vm, hipMalloc(&d, bytes));
        uint64_t *doffs = (uint64_t *)d;
        uint32_t *dlens = (uint32_t *)(d + n * 8), *dat = dlens + n;
        uint8_t *ddata = d + n * 16;
        hipError_t e = hipMemcpy(doffs, offs.data(), n * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(dlens, lens.data(), n * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(dat, at.data(), n * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(ddata, vm->pend_data.data(), vm->pend_data.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess && mimic_launch_scatter(vm->arena, doffs, dlens, dat, ddata, (uint32_t)n, vm->stream))
            e = hipErrorLaunchFailure;
        if (e == hipSuccess) e = hipStreamSynchronize(vm->stream);
        hipFree(d);
        if (e != hipSuccess) return fail(vm, MIMIC_EDEVICE, "map writes: %s", hipGetErrorString(e));
    }
    vm->pend.clear();
    vm->pend_data.clear();
    vm->pend_at.clear();
    vm->host_dirty = false;
    return 0;
}

// ---- shared tables (mimic_map_share) ----------------------------------------------------------
// every member's host image of a shared table is stale (a launch or host write of any member)
static void share_stale(const HostMap &m) {
    if (!m.share) return;
    for (auto &mb : m.share->members) {
        const HostMap &x = ((mimic_vm *)mb.vm)->maps[mb.map];
        if (x.mir) x.mir->valid = false;
    }
}
// a shared table can be used by this VM: its owner alive, no member's arena moved, no member's
// programs delete (every launch on it is pop-only: hashmap.h h_insert_nolock)
static int share_check(mimic_vm *vm, const HostMap &m) {
    if (!m.share) return 0;
    if (m.share->owner_gone) return fail(vm, MIMIC_ENOTSUP, "map '%s': the VM that owns the shared table was destroyed", m.name.c_str());
    for (auto &mb : m.share->members) {
        const mimic_vm *o = (const mimic_vm *)mb.vm;
        if (o->arena != mb.arena)
            return fail(vm, MIMIC_ENOTSUP, "map '%s': a VM sharing it created maps after the share (its arena moved)", m.name.c_str());
        if (o->prog_deletes)
            return fail(vm, MIMIC_ENOTSUP, "map '%s': shared tables take programs that never delete (map_delete_elem)", m.name.c_str());
    }
    return 0;
}
// before a host operation on a shared table: every member's staged writes and launches have
// reached the device (a device-wide wait: the other VMs run on their own streams), and this VM's
// image is fetched again
static int share_pre(mimic_vm *vm, const HostMap &m) {
    if (!m.share) return 0;
    int rc = share_check(vm, m);
    if (rc) return rc;
    for (auto &mb : m.share->members) {
        mimic_vm *o = (mimic_vm *)mb.vm;
        if (o != vm && o->host_dirty && (rc = flush_host(o))) return fail(vm, rc, "shared map: %s", o->err.c_str());
    }
    HIP_OK(vm, hipDeviceSynchronize());
    if (m.mir) m.mir->valid = false;
    return 0;
}
// after a host write on a shared table: on the device at once, the members' images stale
static int share_post(mimic_vm *vm, const HostMap &m, int rc) {
    if (!m.share || rc < 0) return rc;
    const int fr = flush_host(vm);
    share_stale(m);
    return fr ? fr : rc;
}

// the sequential hash algorithm on the image (hashmap.h h_find / h_probe_held / h_place_held /
// h_fl_pop / h_fl_push with one thread): slot of the key or -1; *pos = its bucket, *freep = the
// first reusable bucket on its probe path
// (MH_FAULT: a page could not be fetched; the error is the VM's)
#define MH_FAULT (-2)
static int32_t mh_probe(mimic_vm *vm, const HostMap &m, const KeyBytes &ks, uint64_t h, uint32_t *pos, uint32_t *freep) {
    const HashMirror &x = *m.mir;
    const uint32_t mask = m.ht_cap - 1, tag = (uint32_t)(h >> 32), nq = (m.key_size + 7) >> 3;
    uint32_t p = (uint32_t)h & mask;
    *freep = HT_EMPTY;
    for (uint32_t n = 0; n < m.ht_cap; n++, p = (p + 1) & mask) {
        if (mirror_rec(vm, m, p)) return MH_FAULT;
        const uint64_t *r = &x.rec[(size_t)p * m.rec_q];
        const uint32_t st = (uint32_t)r[0];
        if (st == HT_EMPTY) {
            if (*freep == HT_EMPTY) *freep = p;
            return -1;
        }
        if (st == HT_TOMB) {
            if (*freep == HT_EMPTY) *freep = p;
            continue;
        }
        if (st < HT_BUSY && (uint32_t)(r[0] >> 32) == tag) {
            bool eq = true;
            for (uint32_t q = 0; q < nq && eq; q++) eq = r[1 + q] == ks.word(q);
            if (eq) {
                *pos = p;
                return (int32_t)st;
            }
        }
    }
    return -1;
}

// LinuxHashMap.Update :158-203 / LinuxPerCPUHashMap.Update :564-612 on the image: 0 or E2BIG
static int mh_update(mimic_vm *vm, const HostMap &m, const void *key, const void *value, int32_t cpu) {
    HashMirror &x = *m.mir;
    const KeyBytes ks{(const uint8_t *)key, m.key_size};
    const uint64_t h = h_hash(ks, m.key_size);
    uint32_t pos = 0, freep = HT_EMPTY;
    int32_t idx = mh_probe(vm, m, ks, h, &pos, &freep);
    if (idx == MH_FAULT) return MIMIC_EDEVICE;
    if (idx < 0) {
        if (x.ctl.avail <= 0) return 7;   // the freelist is empty: syscall.E2BIG
        const uint64_t at = x.ctl.head;
        if (mirror_ring(vm, m, at) || mirror_rec(vm, m, freep)) return MIMIC_EDEVICE;
        x.ctl.avail--;
        x.ctl.head++;
        int32_t &f = x.ring[at & (m.fl_cap - 1)];
        idx = f;
        f = -1;
        uint64_t rb, fo, co;
        ht_offsets(m, &rb, &fo, &co);
        stage_write(vm, m.ht_dev_off + fo + (at & (m.fl_cap - 1)) * 4, &f, 4);
        uint64_t *r = &x.rec[(size_t)freep * m.rec_q];
        if ((uint32_t)r[0] == HT_EMPTY) x.ctl.used0++;
        for (uint32_t q = 0; q * 8 < m.key_size; q++) r[1 + q] = ks.word(q);
        r[0] = ((uint64_t)(uint32_t)(h >> 32) << 32) | (uint32_t)idx;
        stage_write(vm, m.ht_dev_off + (uint64_t)freep * m.rec_q * 8, r, m.rec_q * 8);
        stage_write(vm, m.keys_dev_off + (uint64_t)idx * m.key_size, key, m.key_size);   // keys.Write (:188-192)
        x.dirty = true;
        vm->host_dirty = true;
    }
    // values[cpu].Write(idx * S, value) (:193-200)
    stage_write(vm, m.dev_off + (m.family == FAM_PERCPU_HASH ? (uint64_t)cpu * m.dev_stride : 0) + (uint64_t)idx * m.value_size,
                value, m.value_size);
    return 0;
}

// LinuxHashMap.Delete :225-255 on the image (an absent key is no error)
static int mh_delete(mimic_vm *vm, const HostMap &m, const void *key) {
    HashMirror &x = *m.mir;
    const KeyBytes ks{(const uint8_t *)key, m.key_size};
    const uint64_t h = h_hash(ks, m.key_size);
    uint32_t pos = 0, freep;
    const int32_t idx = mh_probe(vm, m, ks, h, &pos, &freep);
    if (idx == MH_FAULT) return MIMIC_EDEVICE;
    if (idx < 0) return 0;
    const uint64_t at = x.ctl.tail;
    if (mirror_ring(vm, m, at)) return MIMIC_EDEVICE;
    uint64_t &w = x.rec[(size_t)pos * m.rec_q];
    w = (w & ~0xffffffffull) | HT_TOMB;
    x.ctl.tail++;
    x.ring[at & (m.fl_cap - 1)] = idx;   // the freelist's tail (:244-250)
    uint64_t rb, fo, co;
    ht_offsets(m, &rb, &fo, &co);
    // (the whole record, as inserts stage it: stage_write merges writes of one offset and size only)
    stage_write(vm, m.ht_dev_off + (uint64_t)pos * m.rec_q * 8, &w, m.rec_q * 8);
    stage_write(vm, m.ht_dev_off + fo + (at & (m.fl_cap - 1)) * 4, &idx, 4);
    x.ctl.avail++;
    x.dirty = true;
    vm->host_dirty = true;
    m.may_tomb = true;
    return 0;
}

// LinuxArrayMap.Update / LinuxPerCPUArrayMap.Update (emulator_linux_map_array.go:97-113, 244-250),
// LinuxHashMap.Update / LinuxPerCPUHashMap.Update (emulator_linux_map_hash.go:158-203, 564-612)
int mimic_map_update(mimic_vm *vm, uint32_t id, const void *key, const void *value, uint32_t flags, int32_t cpu) {
    (void)flags;  // Q10: flags are ignored
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    uint64_t base;
    if (is_hash(m)) {
        if (m.family == FAM_HASH) cpu = 0;  // LinuxHashMap ignores cpuid
        else if ((rc = array_cpu(vm, m, cpu, &base))) return rc;
        if ((rc = share_pre(vm, m)) || (rc = mirror_ensure(vm, m))) return rc;
        return share_post(vm, m, mh_update(vm, m, key, value, cpu));
    }
    if ((rc = array_cpu(vm, m, cpu, &base))) return rc;
    if (m.key_size != 4) return fail(vm, MIMIC_EINVAL, "invalid key length, must be 4 bytes for array maps");
    uint32_t k;
    memcpy(&k, key, 4);
    if (k >= m.max_entries) return 7;  // syscall.E2BIG
    stage_write(vm, base + (uint64_t)k * m.value_size, value, m.value_size);   // applied before the device reads the map
    return 0;
}

// n LinuxMap.Update calls in one (keys packed K bytes apart, values S bytes apart): rc_out[i] =
// what the i-th call returns (0 or a positive errno); returns 0 or the first fatal error
int mimic_map_update_batch(mimic_vm *vm, uint32_t id, const void *keys, const void *values, uint32_t n, uint32_t flags,
                           int32_t cpu, int32_t *rc_out) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    for (uint32_t i = 0; i < n; i++) {
        rc = mimic_map_update(vm, id, (const uint8_t *)keys + (size_t)i * m.key_size,
                              (const uint8_t *)values + (size_t)i * m.value_size, flags, cpu);
        if (rc < 0) return rc;
        if (rc_out) rc_out[i] = rc;
    }
    return 0;
}

// LinuxMap.Lookup: the value's virtual address, 0 when absent (emulator_linux_map_array.go:78-94,
// 235-241; emulator_linux_map_hash.go:134-155, 537-561)
int mimic_map_lookup(mimic_vm *vm, uint32_t id, const void *key, int32_t cpu, uint32_t *addr_out) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    uint64_t base;
    if (is_hash(m)) {
        uint32_t b = m.backing_addr;
        if (m.family == FAM_PERCPU_HASH) {
            if ((rc = array_cpu(vm, m, cpu, &base))) return rc;
            b += (uint32_t)cpu * m.addr_period;
        }
        if ((rc = share_pre(vm, m)) || (rc = mirror_ensure(vm, m))) return rc;
        const KeyBytes ks{(const uint8_t *)key, m.key_size};
        uint32_t pos = 0, freep;
        const int32_t slot = mh_probe(vm, m, ks, h_hash(ks, m.key_size), &pos, &freep);
        if (slot == MH_FAULT) return MIMIC_EDEVICE;
        *addr_out = slot < 0 ? 0 : b + (uint32_t)slot * m.value_size;
        return 0;
    }
    if ((rc = array_cpu(vm, m, cpu, &base))) return rc;
    if (m.key_size != 4) return fail(vm, MIMIC_EINVAL, "invalid key length, must be 4 bytes for array maps");
    uint32_t k;
    memcpy(&k, key, 4);
    uint32_t b = m.backing_addr + (m.family == FAM_PERCPU_ARRAY ? (uint32_t)cpu * m.addr_period : 0u);
    *addr_out = k >= m.max_entries ? 0 : b + k * m.value_size;
    return 0;
}

// LinuxMapDeleter.Delete (emulator_linux_map_hash.go:225-255, 634-664); arrays are not deleters
int mimic_map_delete(mimic_vm *vm, uint32_t id, const void *key) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    if (!is_hash(m)) return fail(vm, MIMIC_EINVAL, "can't delete from given LinuxMap");
    if ((rc = share_pre(vm, m)) || (rc = mirror_ensure(vm, m))) return rc;
    return share_post(vm, m, mh_delete(vm, m, key));
}

// live (key, slot) pairs of a hash map in table order
static int hash_entries(mimic_vm *vm, const HostMap &m, uint8_t *keys, int32_t *slots, size_t cap_entries,
                        uint32_t *n_out) {
    int rc = share_pre(vm, m);
    if (!rc) rc = mirror_ensure(vm, m);
    if (!rc) rc = mirror_pages(vm, m, false, 0, (uint64_t)m.ht_cap * m.rec_q * 8);   // every record
    if (rc) return rc;
    const std::vector<uint64_t> &rec = m.mir->rec;
    uint32_t n = 0;
    for (uint32_t p = 0; p < m.ht_cap; p++) {
        const uint64_t *r = &rec[(size_t)p * m.rec_q];
        if ((uint32_t)r[0] >= m.max_entries) continue;
        if (n >= cap_entries) return fail(vm, MIMIC_EINVAL, "buffer too small");
        if (keys) memcpy(keys + (size_t)n * m.key_size, r + 1, m.key_size);
        if (slots) slots[n] = (int32_t)(uint32_t)r[0];
        n++;
    }
    *n_out = n;
    return 0;
}

// LinuxMap.Keys (emulator_linux_map_hash.go:113-131): the live keys, packed, in table order
// (the reference returns Go map order, which is unspecified)
int mimic_map_keys(mimic_vm *vm, uint32_t id, void *out, size_t cap, uint32_t *n_out) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    if (!n_out) return MIMIC_EINVAL;
    if (!is_hash(m)) {  // array family: keys 0..E-1 (emulator_linux_map_array.go:64-75)
        if (cap < (uint64_t)m.max_entries * 4) return fail(vm, MIMIC_EINVAL, "buffer too small");
        for (uint32_t k = 0; k < m.max_entries; k++) memcpy((uint8_t *)out + 4ull * k, &k, 4);
        *n_out = m.max_entries;
        return 0;
    }
    return hash_entries(vm, m, (uint8_t *)out, nullptr, m.key_size ? cap / m.key_size : m.max_entries, n_out);
}

// KeyToIndex as (key, slot) pairs: where each live key's value sits in the values backing(s)
int mimic_map_entries(mimic_vm *vm, uint32_t id, void *keys_out, int32_t *slots_out, size_t cap_entries,
                      uint32_t *n_out) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    if (!n_out) return MIMIC_EINVAL;
    if (!is_hash(m)) return fail(vm, MIMIC_EINVAL, "not a hash map");
    return hash_entries(vm, m, (uint8_t *)keys_out, slots_out, cap_entries, n_out);
}

int mimic_map_read_values(mimic_vm *vm, uint32_t id, int32_t cpu, void *out, size_t cap) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    uint64_t base;
    if ((rc = array_cpu(vm, m, cpu, &base))) return rc;
    uint64_t n = (uint64_t)m.max_entries * m.value_size;
    if (cap < n) return fail(vm, MIMIC_EINVAL, "buffer too small");
    if ((rc = share_pre(vm, m)) || (rc = flush_host(vm)) || (rc = settle(vm))) return rc;
    HIP_OK(vm, hipMemcpy(out, vm->arena + base, n, hipMemcpyDeviceToHost));
    return (int)n;
}

// mimic_map_share: vm's map `id` becomes the owner VM's map `owner_id` -- ONE table for both (the
// reference's LinuxHashMap shared by every process of a pool, emulator_linux_map_hash.go:21-255):
// every insert, E2BIG and lookup of either VM's launches and host operations sees the other's.
int mimic_map_share(mimic_vm *vm, uint32_t id, mimic_vm *owner, uint32_t owner_id) {
    if (!vm || !owner || vm == owner) return MIMIC_EINVAL;
    int rc = map_check(vm, id);
    if (rc) return rc;
    if (owner_id >= owner->maps.size()) return fail(vm, MIMIC_ENOENT, "owner has no map %u", owner_id);
    HostMap &m = vm->maps[id];
    const HostMap &o = owner->maps[owner_id];
    if (vm->s.device != owner->s.device)
        return fail(vm, MIMIC_ENOTSUP, "shared tables live on one device (peer tables over xGMI are not built)");
    if (!is_hash(m) || m.family != o.family || m.key_size != o.key_size || m.value_size != o.value_size ||
        m.max_entries != o.max_entries || m.ncpu != o.ncpu || m.dev_stride != o.dev_stride || m.ht_cap != o.ht_cap ||
        m.rec_q != o.rec_q || m.nlocks != o.nlocks || m.fl_cap != o.fl_cap)
        return fail(vm, MIMIC_EINVAL, "map '%s': only a hash map of the same spec can share a table", m.name.c_str());
    if (m.share) return fail(vm, MIMIC_EINVAL, "map '%s' already shares a table", m.name.c_str());
    if ((rc = flush_host(vm)) || (rc = flush_host(owner)) || (rc = settle(vm)) || (rc = settle(owner))) return rc;
    if (!o.share) {
        o.share = std::make_shared<ShareGroup>();
        o.share->members.push_back({owner, owner_id, owner->arena});
    }
    // this map's offsets now lead from this VM's arena into the owner's table (64-bit wraparound)
    const uint64_t a = (uint64_t)(uintptr_t)vm->arena, b = (uint64_t)(uintptr_t)owner->arena;
    m.dev_off = b + o.dev_off - a;
    m.keys_dev_off = b + o.keys_dev_off - a;
    m.ht_dev_off = b + o.ht_dev_off - a;
    m.share = o.share;
    m.share->members.push_back({vm, id, vm->arena});
    m.pop_dirty = o.pop_dirty;
    m.may_tomb = o.may_tomb;
    share_stale(m);
    vm->tables_dirty = true;   // the device map table carries the new offsets
    owner->tables_dirty = true;   // (and the owner's map is no longer its chunk map)
    return share_check(vm, m);
}

int mimic_map_reset(mimic_vm *vm, uint32_t id, void *hip_stream) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    if (m.type == 3) return fail(vm, MIMIC_ENOTSUP, "program arrays are not reset");   // ebpf.ProgramArray
    hipSetDevice(vm->s.device);
    if ((rc = share_pre(vm, m)) || (rc = skb_settle(vm)) || (rc = flush_host(vm))) return rc;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : vm->stream;
    if (vm->last_stream && vm->last_stream != st) HIP_OK(vm, hipStreamSynchronize(vm->last_stream));
    if (is_hash(m)) {   // one kernel: values, keys, index (interp.hip mimic_hash_reset_kernel)
        m.pop_dirty = false;
        const DMap dm = to_dmap(m);
        if (mimic_launch_hash_reset(vm->arena, &dm, st))
            return fail(vm, MIMIC_EDEVICE, "reset: %s", hipGetErrorString(hipGetLastError()));
        share_stale(m);
        mirror_fresh(m);   // the image of the table the reset leaves
    } else {
        HIP_OK(vm, hipMemsetAsync(vm->arena + m.dev_off, 0, (size_t)m.dev_stride * m.ncpu, st));
    }
    vm->last_stream = st;
    return 0;
}

int mimic_map_read_values_range(mimic_vm *vm, uint32_t id, int32_t cpu_begin, int32_t cpu_end, void *out, size_t cap) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    uint32_t c0 = 0, c1 = 1;
    if (m.family == FAM_PERCPU_ARRAY || m.family == FAM_PERCPU_HASH) {
        if (cpu_begin < 0 || cpu_end > (int32_t)m.ncpu || cpu_begin >= cpu_end) return fail(vm, MIMIC_EINVAL, "bad cpu range");
        c0 = (uint32_t)cpu_begin;
        c1 = (uint32_t)cpu_end;
    } else if (cpu_begin != 0 || cpu_end != 1) {
        return fail(vm, MIMIC_EINVAL, "bad cpu range");
    }
    const uint64_t row = (uint64_t)m.max_entries * m.value_size, n = row * (c1 - c0);
    if (cap < n) return fail(vm, MIMIC_EINVAL, "buffer too small");
    if (n == 0) return 0;
    if ((rc = share_pre(vm, m)) || (rc = flush_host(vm)) || (rc = settle(vm))) return rc;
    if (m.dev_stride == row || c1 - c0 == 1)
        HIP_OK(vm, hipMemcpy(out, vm->arena + m.dev_off + (uint64_t)c0 * m.dev_stride, n, hipMemcpyDeviceToHost));
    else
        HIP_OK(vm, hipMemcpy2D(out, row, vm->arena + m.dev_off + (uint64_t)c0 * m.dev_stride, m.dev_stride, row,
                               c1 - c0, hipMemcpyDeviceToHost));
    return 0;
}

int mimic_map_sum_u64(mimic_vm *vm, uint32_t id, int32_t cpu_begin, int32_t cpu_end, uint64_t *out, size_t cap) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    const HostMap &m = vm->maps[id];
    if (m.value_size != 8) return fail(vm, MIMIC_EINVAL, "value size must be 8");
    if (cap < m.max_entries) return fail(vm, MIMIC_EINVAL, "buffer too small");
    uint32_t c0 = 0, c1 = 1;
    if (m.family == FAM_PERCPU_ARRAY || m.family == FAM_PERCPU_HASH) {
        if (cpu_begin < 0 || cpu_end > (int32_t)m.ncpu || cpu_begin >= cpu_end) return fail(vm, MIMIC_EINVAL, "bad cpu range");
        c0 = (uint32_t)cpu_begin;
        c1 = (uint32_t)cpu_end;
    }
    if (m.max_entries == 0) return 0;
    if ((rc = share_pre(vm, m)) || (rc = flush_host(vm))) return rc;
    uint64_t *d = nullptr;
    HIP_OK(vm, hipMalloc(&d, m.max_entries * sizeof(uint64_t)));
    hipStream_t st = vm->last_stream ? vm->last_stream : vm->stream;
    hipError_t e = hipSuccess;
    if (mimic_launch_sum_u64(vm->arena + m.dev_off + (uint64_t)c0 * m.dev_stride, m.dev_stride, m.max_entries, c1 - c0,
                             d, st))
        e = hipErrorLaunchFailure;
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, m.max_entries * sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipFree(d);
    if (e != hipSuccess) return fail(vm, MIMIC_EDEVICE, "sum: %s", hipGetErrorString(e));
    return 0;
}

int mimic_map_addr(mimic_vm *vm, uint32_t id, uint32_t *addr_out) {
    int rc = map_check(vm, id);
    if (rc) return rc;
    *addr_out = vm->maps[id].obj_addr;
    return 0;
}

// VM.AddProgram (vm.go:98-139) + LinuxEmulator.RewriteProgram (emulator_linux_.go:292-339)
int mimic_program_load(mimic_vm *vm, const char *name, const void *insns, uint32_t n_slots,
                       const mimic_reloc *relocs, uint32_t n_relocs, uint32_t *prog_id) {
    if (!vm || (!insns && n_slots) || !prog_id) return MIMIC_EINVAL;
    if (vm->skb_leaked)
        return fail(vm, MIMIC_ENOTSUP, "adding programs after sk_buff batches is not supported (mimic_skb_release first)");
    if (int rc = skb_settle(vm)) return rc;
    uint64_t total = n_slots;
    for (auto &q : vm->progs) total += q.ins.size();
    if (n_slots >= (1u << MIMIC_PC_BITS) || total >= 0x7fffffffull) return fail(vm, MIMIC_EINVAL, "program too long");
    if (vm->progs.size() >= 65535) return fail(vm, MIMIC_EINVAL, "too many programs");
    hipSetDevice(vm->s.device);
    HostProg p;
    p.name = name ? name : "";
    std::string derr;
    if (decode_program((const uint8_t *)insns, n_slots, p.ins, &derr)) return fail(vm, MIMIC_EINVAL, "%s", derr.c_str());
    for (uint32_t r = 0; r < n_relocs; r++) {
        uint32_t s = relocs[r].slot;
        if (s >= n_slots) return fail(vm, MIMIC_EINVAL, "relocation slot %u out of range", s);
        DInsn &d = p.ins[s];
        uint32_t op = d.w & 0xff, src = (d.w >> 12) & 0xf;
        if (!(op == 0x18 && (src == 1 || src == 2))) continue;  // !IsLoadFromMap
        if (relocs[r].map_id >= vm->maps.size())
            return fail(vm, MIMIC_EINVAL, "program references a map that does not exist in the emulator");
        uint32_t a = vm->maps[relocs[r].map_id].obj_addr;
        if (src == 1) d.k = a;                                        // PseudoMapFD
        else d.k = (uint64_t)((int64_t)a + (int64_t)(int16_t)(d.w >> 16));  // PseudoMapValue (Q16)
    }
    p.addr = add_entry(vm, 8);
    Seg g{};
    g.lo = p.addr;
    g.hi = p.addr + 8;
    g.kind = SEG_PROG;
    g.id = (uint32_t)vm->progs.size();
    vm->segs.push_back(g);
    vm->progs.push_back(std::move(p));
    vm->tables_dirty = true;
    *prog_id = g.id;
    return 0;
}

int mimic_program_addr(mimic_vm *vm, uint32_t prog_id, uint32_t *addr_out) {
    if (!vm || prog_id >= vm->progs.size()) return MIMIC_EINVAL;
    *addr_out = vm->progs[prog_id].addr;
    return 0;
}

int mimic_stack_addr(mimic_vm *vm, uint32_t *addr_out) {
    if (!vm) return MIMIC_EINVAL;
    *addr_out = vm->next_addr;
    return 0;
}

int mimic_mem_read(mimic_vm *vm, uint32_t addr, void *buf, uint32_t len) {
    if (!vm) return MIMIC_EINVAL;
    hipSetDevice(vm->s.device);
    HostRef R = host_resolve(vm, addr);
    if (R.kind == 0) return fail(vm, MIMIC_EFAULT, "memory controller can't resolve address 0x%x", addr);
    if (R.kind == 2) return fail(vm, MIMIC_EFAULT, "not vm memory 0x%x", addr);
    if (R.kind == 3) return fail(vm, MIMIC_EFAULT, "Can't access non-data-section array map directly");
    if ((uint64_t)R.off + len > R.limit) return fail(vm, MIMIC_EFAULT, "out of bounds");
    if (int rc = flush_host(vm)) return rc;
    if (vm->last_stream) HIP_OK(vm, hipStreamSynchronize(vm->last_stream));
    HIP_OK(vm, hipMemcpy(buf, vm->arena + R.dev_off + R.off, len, hipMemcpyDeviceToHost));
    return 0;
}

int mimic_mem_load(mimic_vm *vm, uint32_t addr, int32_t size, uint64_t *out) {
    if (size != 1 && size != 2 && size != 4 && size != 8) return MIMIC_EINVAL;
    uint64_t v = 0;
    int rc = mimic_mem_read(vm, addr, &v, (uint32_t)size);
    if (rc) return rc;
    *out = v;
    return 0;
}

// the batch form of NewProcess / SetCPUID / Run / Cleanup.  shift: for an INTERLEAVED
// sub-batch, the index of its first packet in the whole batch (vCPU of packet k = (shift+k) % V)
struct SkbRun {     // the sk_buff part of a batch (mimic_run_skb)
    uint32_t ifindex;
    const mimic_skb_custom *custom;   // device, [n] or null
    // processes whose Load ran at NewProcess (mimic_process_run_many): their derived record words,
    // absolute leak addresses (+ flags) and a zero base, gathered -- no prep kernel for this batch
    const uint64_t *pre_drv = nullptr, *pre_prefix = nullptr, *pre_base = nullptr;
    uint32_t *rooms_state = nullptr;   // the batch's rooms-clean word (mimic_skb_batch.rooms_state) or null
};
struct StepRun {    // a stepped single process (mimic_process_*): its state, private memory and budget
    StepState *state;
    uint8_t *priv;
    uint64_t priv_bytes;
    uint64_t budget;
    // an sk_buff process: its own record, leak prefix and leak base (made once, at NewProcess)
    SkbRec *skb_rec = nullptr;
    const uint64_t *skb_prefix = nullptr, *skb_base = nullptr;
    const mimic_skb_custom *skb_custom = nullptr;   // its user-given sock / flow keys (device, one entry) or null
    uint32_t gen = 0;   // the generation its state carries (StepState::gen)
    // its first launch: the NewProcess image (device-visible host address), its device block, bytes
    const uint8_t *img = nullptr;
    uint8_t *img_dst = nullptr;
    uint32_t img_n = 0;
    // Process.Run of a fresh xdp_md process on the single-process JIT form (vm->jit_fn_proc) on
    // vCPU `cpu` (this engine's): a one-lane batch whose exit writes the state
    bool jit = false;
    int32_t cpu = 0;
};

struct CtxRun {      // Run(ctx) of a batch: one context for every packet, or one per packet (host array)
    mimic_ctx *all;
    mimic_ctx *const *per_packet;
    // per_packet's context words already on the device (the host pipeline uploads the whole batch's
    // array once; a sub-batch points into it): no per-launch upload
    const uint32_t *const *dev_pp = nullptr;
};
// mimic_run_xdp_many: the batches of one launch (b[0] is the one run_xdp_impl is given); `used` is
// set when the launch ran all of them (an owned spread kernel), else it ran b[0] only
struct ManyRun {
    const mimic_xdp_batch *b;
    const mimic_xdp_results *r;
    uint32_t k;
    bool used;
};
static int run_xdp_impl(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *b, const mimic_xdp_results *res,
                        hipStream_t st_in, uint64_t shift, const SkbRun *skb = nullptr, const StepRun *step = nullptr,
                        const CtxRun *cx = nullptr, ManyRun *mr = nullptr);

int mimic_run_xdp(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *b, const mimic_xdp_results *res,
                  void *hip_stream) {
    return run_xdp_impl(vm, prog_id, b, res, (hipStream_t)hip_stream, 0);
}

// k batches of one program as few launches as possible: groups of up to MIMIC_MANY_MAX batches run as
// ONE launch of the owned spread kernel when the programs and the batches allow it (every thread runs
// its packets of each batch in turn: a vCPU's packets keep batch order, as processPool draining a
// backlog of batches would), else one launch per batch.  Not in the reference API.
int mimic_run_xdp_many(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *b, const mimic_xdp_results *res, uint32_t k,
                       void *hip_stream) {
    if (!vm || (k && (!b || !res))) return MIMIC_EINVAL;
    hipStream_t st = (hipStream_t)hip_stream;
    // batches that can share a launch: same size, schedule and scalar fields, no per-packet arrays
    auto same = [&](const mimic_xdp_batch &x, const mimic_xdp_batch &y) {
        return x.n == y.n && x.schedule == y.schedule && x.schedule != MIMIC_SCHED_EXPLICIT && !x.headroom && !y.headroom &&
               !x.tailroom && !y.tailroom && !x.ingress_ifindex && !y.ingress_ifindex && !x.rx_queue_index &&
               !y.rx_queue_index && !x.egress_ifindex && !y.egress_ifindex && x.headroom_all == y.headroom_all &&
               x.tailroom_all == y.tailroom_all && x.ingress_all == y.ingress_all && x.rxq_all == y.rxq_all &&
               x.egress_all == y.egress_all && x.step_budget == y.step_budget;
    };
    for (uint32_t a = 0; a < k;) {
        uint32_t e = a + 1;
        while (e < k && e - a < MIMIC_MANY_MAX && same(b[a], b[e])) e++;
        ManyRun mr{b + a, res + a, e - a, false};
        int rc = run_xdp_impl(vm, prog_id, b + a, res + a, st, 0, nullptr, nullptr, nullptr, e - a > 1 ? &mr : nullptr);
        if (rc) return rc;
        if (!mr.used)   // one launch per batch
            for (uint32_t q = a + 1; q < e; q++)
                if ((rc = run_xdp_impl(vm, prog_id, b + q, res + q, st, 0))) return rc;
        a = e;
    }
    return 0;
}

int mimic_run_xdp_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *b, const mimic_xdp_results *res,
                      void *hip_stream, mimic_ctx *ctx, mimic_ctx *const *ctx_per_packet) {
    const CtxRun cx{ctx, ctx_per_packet};
    return run_xdp_impl(vm, prog_id, b, res, (hipStream_t)hip_stream, 0, nullptr, nullptr, &cx);
}

static int run_skb_impl(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *sb, const mimic_xdp_results *res,
                        void *hip_stream, const CtxRun *cx);

// Batch form of NewProcess(prog, &LinuxContextSKBuff{Packet, Dev}) + SetCPUID + Run + Cleanup
int mimic_run_skb(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *sb, const mimic_xdp_results *res,
                  void *hip_stream) {
    return run_skb_impl(vm, prog_id, sb, res, hip_stream, nullptr);
}

int mimic_run_skb_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *sb, const mimic_xdp_results *res,
                      void *hip_stream, mimic_ctx *ctx, mimic_ctx *const *ctx_per_packet) {
    const CtxRun cx{ctx, ctx_per_packet};
    return run_skb_impl(vm, prog_id, sb, res, hip_stream, &cx);
}

static int run_skb_impl(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *sb, const mimic_xdp_results *res,
                        void *hip_stream, const CtxRun *cx) {
    if (!vm || !sb || !res) return MIMIC_EINVAL;
    mimic_xdp_batch b{};
    b.n = sb->n;
    b.schedule = sb->schedule;
    b.pkt_data = sb->pkt_data;
    b.pkt_off = sb->pkt_off;
    b.pkt_len = sb->pkt_len;
    b.cpu = sb->cpu;
    b.step_budget = sb->step_budget;
    SkbRun r{sb->ifindex, sb->custom};
    r.rooms_state = sb->rooms_state;
    return run_xdp_impl(vm, prog_id, &b, res, (hipStream_t)hip_stream, 0, &r, nullptr, cx);
}

int mimic_skb_release(mimic_vm *vm) {
    if (!vm) return MIMIC_EINVAL;
    hipSetDevice(vm->s.device);
    // No host wait here: the next sk_buff batch on the same stream is ordered behind the last one
    // anyway (a wait would leave the GPU idle for a host round trip per batch); anything else that
    // needs the sk_buff work finished calls skb_settle() first.
    // an engine-owned event behind the released batches: the caller may destroy its stream after this
    if (vm->skb_stream) {
        if (!vm->skb_ev) HIP_OK(vm, hipEventCreateWithFlags(&vm->skb_ev, hipEventDisableTiming));
        HIP_OK(vm, hipEventRecord(vm->skb_ev, vm->skb_stream));
        vm->skb_stream = nullptr;
        vm->skb_release_pending = true;
    }
    vm->skb_leaked = false;
    return 0;
}

// wait for the sk_buff batches mimic_skb_release let go of (map / program loads, xdp_md batches)
static int skb_settle(mimic_vm *vm) {
    if (vm->skb_release_pending) HIP_OK(vm, hipEventSynchronize(vm->skb_ev));
    vm->skb_release_pending = false;
    return 0;
}

// the sk_buff records and leak addresses of a batch (skb.hip), on stream st; `into`
// (a stepped process's own arrays, one packet) instead of the VM's batch arrays
struct SkbInto {
    SkbRec *rec;
    uint64_t *prefix;   // 2 words (skb.h skb_leak_pre)
};
static int skb_ensure(mimic_vm *vm, uint32_t n, hipStream_t st);
static int skb_prepare(mimic_vm *vm, const mimic_xdp_batch *b, hipStream_t st, const SkbInto *into = nullptr,
                       bool records = true, bool sparse = false, uint32_t *rooms_state = nullptr) {
    const uint32_t n = b->n;
    if (vm->skb_stream && vm->skb_stream != st) HIP_OK(vm, hipStreamSynchronize(vm->skb_stream));
    // batches released on a stream the caller may have destroyed since: ordered through their event
    if (vm->skb_release_pending) HIP_OK(vm, hipStreamWaitEvent(st, vm->skb_ev, 0));
    int rc0 = skb_ensure(vm, n, st);
    if (rc0) return rc0;
    // the first leak follows the stack and sk_buff entries: St + S + 1 + 193
    const uint64_t init = (uint64_t)vm->next_addr + stack_size(vm) + 1 + SKB_STRUCT_SIZE + 1;
    // a batch's derived words go to the compact array (read by skb_load*), a process's into its record
    uint64_t *out = into ? (uint64_t *)into->rec : records ? vm->d_skb_drv : nullptr;
    const uint32_t out_q = into ? (uint32_t)(sizeof(SkbRec) / 8) : SKB_DERIVED_Q;
    // MIMIC_SKB_ROOMS_CHAIN=1 (measurement, JIT batches only): the chain kernel reads the rooms itself
    static const bool rooms_chain = getenv("MIMIC_SKB_ROOMS_CHAIN") && getenv("MIMIC_SKB_ROOMS_CHAIN")[0] == '1';
    // MIMIC_SKB_ROOMS_ZERO=1: the prep zeroes every loaded packet's rooms without reading them
    static const bool rooms_zero = getenv("MIMIC_SKB_ROOMS_ZERO") && getenv("MIMIC_SKB_ROOMS_ZERO")[0] == '1';
    if (mimic_launch_skb_prep(b->pkt_data, b->pkt_off, b->pkt_len, n, out, out_q, into ? into->prefix : vm->d_skb_prefix,
                              vm->d_skb_state, init, vm->skb_leaked ? 0u : 1u, (rooms_chain && !into) ? 0u : rooms_zero ? 2u : 1u,
                              (sparse && !into) ? 1u : 0u, into ? nullptr : rooms_state, st))
        return fail(vm, MIMIC_EDEVICE, "sk_buff prep: %s", hipGetErrorString(hipGetLastError()));
    if (n) vm->skb_leaked = true;
    vm->skb_stream = st;
    return 0;
}

// the VM's sk_buff batch arrays for n packets (records, derived words, prefixes) and its leak state
static int skb_ensure(mimic_vm *vm, uint32_t n, hipStream_t st) {
    if (n > vm->skb_cap || !vm->d_skb_state) {
        HIP_OK(vm, hipStreamSynchronize(st));
        hipFree(vm->d_skb_rec);
        hipFree(vm->d_skb_drv);
        hipFree(vm->d_skb_prefix);
        vm->d_skb_rec = nullptr;
        vm->d_skb_drv = nullptr;
        vm->d_skb_prefix = nullptr;
        const size_t cap = std::max<size_t>(n, 1024);
        HIP_OK(vm, hipMalloc(&vm->d_skb_rec, cap * sizeof(SkbRec)));
        HIP_OK(vm, hipMalloc(&vm->d_skb_drv, cap * 8 * SKB_DERIVED_Q));
        // within-block prefixes, then the blocks' offsets (skb.hip)
        HIP_OK(vm, hipMalloc(&vm->d_skb_prefix, (cap + (cap >> SKB_PREP_LOG2) + 1) * 8));
        if (!vm->d_skb_state) {   // leak cursor, batch base, the prep kernel's block counter (zero)
            HIP_OK(vm, hipMalloc(&vm->d_skb_state, 32));
            HIP_OK(vm, hipMemset(vm->d_skb_state, 0, 32));
        }
        vm->skb_cap = cap;
    }
    return 0;
}

// the private-memory plan of a VM: qwords per lane and the qword offsets of its areas
struct PrivPlan {
    uint32_t xdp_q, frame_q, key_q, q_per_lane;
};
static PrivPlan priv_plan(const mimic_vm *vm) {
    PrivPlan p;
    const uint32_t stack_q = stack_size(vm) / 8;   // stack | xdp_md overlay | saved frames | hash key
    p.xdp_q = stack_q;
    p.frame_q = p.xdp_q + 3;
    p.key_q = p.frame_q + MIMIC_MAX_FRAMES * MIMIC_FRAME_QWORDS;
    uint32_t key_words = 0;  // hash helpers copy the key here once (derefMapKey)
    for (auto &m : vm->maps)
        if (is_hash(m)) key_words = std::max(key_words, (m.key_size + 7) / 8);
    p.q_per_lane = p.key_q + key_words;
    return p;
}

// The spread kernel of the VM's xdp_md programs (jit.cpp analyze_spread), built once per program
// set: the VM's per-CPU arrays whose values the arena keeps 8-byte aligned are the candidates; the
// analysis names the one map the programs count into, and the kernel is then generated with an
// LDS counter table when a block's rows fit 32 KiB.
// packets per spread block (MIMIC_SPREAD_PPB, measurement: a multiple of 256; default 1024)
static uint32_t spread_ppb() {
    static const uint32_t v = [] {
        const char *e = getenv("MIMIC_SPREAD_PPB");
        const uint32_t x = e ? (uint32_t)atoi(e) : 0u;
        return x >= 256 && x % 256 == 0 ? x : 1024u;
    }();
    return v;
}
static int spread_build(mimic_vm *vm) {
    if (vm->spread_state) return 0;
    vm->spread_state = -1;
    SpreadReq req;
    req.ppb = spread_ppb();
    for (size_t s = 0; s < vm->h_all.size(); s++) {
        const DInsn &x = vm->h_all[s];
        const uint32_t mh = AUX_MAPHINT(x.aux);
        if (AUX_H(x.aux) != H_LDIMM || !mh || mh > vm->maps.size()) continue;
        const HostMap &hm = vm->maps[mh - 1];
        const DMap dm = to_dmap(hm);
        if (hm.family != FAM_PERCPU_ARRAY || (dm.dev_off & 7) || (dm.dev_stride & 7)) continue;
        req.slot_map[(uint32_t)s] = mh - 1;
        req.shape[mh - 1] = {hm.max_entries * hm.value_size, hm.value_size};
    }
    if (req.slot_map.empty()) return 0;
    JitInfo info{};
    std::string src = mimic_jit_source(vm->h_dp, vm->h_all, CTX_XDP, &info, nullptr, false, &req);
    if (!info.spread) return 0;
    // the counted map and its row: an LDS table of min(ppb, V) rows when that fits 32 KiB
    uint32_t row = 0;
    for (auto &kv : req.shape) row = std::max(row, kv.second.first);
    const uint64_t rows = std::min<uint64_t>(req.ppb, (uint64_t)vm->s.vcpu_count);
    if (rows * row <= 32768) {
        req.lds_rows = (uint32_t)rows;
        src = mimic_jit_source(vm->h_dp, vm->h_all, CTX_XDP, &info, nullptr, false, &req);
    }
    vm->spread_lds = req.lds_rows > 0;
    std::string log;
    if (mimic_jit_compile(vm->s.device, src, &vm->jit_fn_spread, &log))
        return fail(vm, MIMIC_EDEVICE, "JIT build failed (spread kernel): %s", log.c_str());
    vm->jit_info_spread = info;
    vm->spread_state = 1;
    return 0;
}

// lanes the one-lane JIT kernel holds resident at its 4-wave budget: CUs x 4 SIMDs x 4 waves x 64
static uint32_t chip_lanes(mimic_vm *vm) {
    static int cus = 0;
    if (!cus) {
        hipDeviceProp_t pr;
        cus = hipGetDeviceProperties(&pr, vm->s.device) == hipSuccess && pr.multiProcessorCount > 0 ? pr.multiProcessorCount : 256;
    }
    return (uint32_t)cus * 4u * 4u * 64u;
}

// The owned form (jit.cpp, SpreadReq::own): built once per program set when the programs allow a
// spread kernel; its LDS table holds up to 256 rows of the counted map's row (32 KiB at most), so a
// batch with P packets per vCPU can use it when 256 / P rows fit.
static int spread_build_own(mimic_vm *vm) {
    if (vm->spread_own_state) return 0;
    vm->spread_own_state = -1;
    SpreadReq req;
    req.own = true;
    for (size_t s = 0; s < vm->h_all.size(); s++) {
        const DInsn &x = vm->h_all[s];
        const uint32_t mh = AUX_MAPHINT(x.aux);
        if (AUX_H(x.aux) != H_LDIMM || !mh || mh > vm->maps.size()) continue;
        const HostMap &hm = vm->maps[mh - 1];
        const DMap dm = to_dmap(hm);
        if (hm.family != FAM_PERCPU_ARRAY || (dm.dev_off & 7) || (dm.dev_stride & 7)) continue;
        req.slot_map[(uint32_t)s] = mh - 1;
        req.shape[mh - 1] = {hm.max_entries * hm.value_size, hm.value_size};
    }
    if (req.slot_map.empty()) return 0;
    uint32_t row = 0;
    for (auto &kv : req.shape) row = std::max(row, kv.second.first);
    if (!row) return 0;
    req.lds_rows = std::min<uint32_t>(256u, 32768u / row);
    if (req.lds_rows < 2) return 0;
    JitInfo info{};
    const std::string src = mimic_jit_source(vm->h_dp, vm->h_all, CTX_XDP, &info, nullptr, false, &req);
    if (!info.spread || !info.spread_own) return 0;
    std::string log;
    if (mimic_jit_compile(vm->s.device, src, &vm->jit_fn_spread_own, &log))
        return fail(vm, MIMIC_EDEVICE, "JIT build failed (owned spread kernel): %s", log.c_str());
    vm->jit_info_spread_own = info;
    vm->spread_own_rows = req.lds_rows;
    vm->spread_own_state = 1;
    return 0;
}

// The VM's private memory for `lanes` lanes of q_per_lane qwords, qword-interleaved with stride
// vm->priv_lanes >= lanes (a launch with fewer lanes uses the larger stride as it is)
static int priv_ensure(mimic_vm *vm, uint32_t q_per_lane, uint32_t lanes, hipStream_t st) {
    const uint32_t stride = std::max(lanes, vm->priv_lanes);
    const uint64_t need = (uint64_t)q_per_lane * stride * 8;
    if (vm->priv && need <= vm->priv_bytes) return 0;
    hipStreamSynchronize(st);
    hipFree(vm->priv);
    vm->priv = nullptr;
    HIP_OK(vm, hipMalloc(&vm->priv, std::max<uint64_t>(need, 8)));
    vm->priv_bytes = std::max<uint64_t>(need, 8);
    vm->priv_lanes = stride;
    return 0;
}

// a spread launch marked per-CPU memory touched outside fused increments (an internal assertion:
// jit.cpp analyze_spread's base provenance keeps such program sets off spread kernels): its
// results may not be the reference's, which is reported as an engine error (stream synchronized)
static int spread_check(mimic_vm *vm) {
    // a block combiner that gave up waiting (hashmap.h h_comb_reserve): its lanes got no position
    if (vm->comb_used) {
        for (const HostMap &m : vm->maps) {
            if (!is_hash(m)) continue;
            uint64_t rb, fo, co;
            ht_offsets(m, &rb, &fo, &co);
            uint32_t f = 0;
            HIP_OK(vm, hipMemcpy(&f, vm->arena + m.ht_dev_off + co + offsetof(HashCtl, comb_fault), 4, hipMemcpyDeviceToHost));
            if (f) return fail(vm, MIMIC_EDEVICE, "map '%s': a block combiner or chunk refill of freelist reservations gave up (engine fault)",
                               m.name.c_str());
        }
    }
    if (!vm->spread_used || !vm->d_spread_bad) return 0;
    uint32_t f = 0;
    HIP_OK(vm, hipMemcpy(&f, vm->d_spread_bad, 4, hipMemcpyDeviceToHost));
    if (f) return fail(vm, MIMIC_EDEVICE, "a spread launch reached per-CPU map memory outside a fused increment");
    return 0;
}

// LD_IMM64 slots naming a per-CPU array whose row the lane value cache can hold, with its E * S
static std::vector<std::pair<uint32_t, uint32_t>> vc_slots_of(const mimic_vm *vm) {
    std::vector<std::pair<uint32_t, uint32_t>> vc;
    for (size_t s = 0; s < vm->h_all.size(); s++) {
        const DInsn &x = vm->h_all[s];
        const uint32_t mh = AUX_MAPHINT(x.aux);
        if (AUX_H(x.aux) != H_LDIMM || !mh || mh > vm->maps.size()) continue;
        const HostMap &hm = vm->maps[mh - 1];
        if (vc_row_ok(hm.family, hm.max_entries, hm.value_size)) vc.push_back({(uint32_t)s, hm.max_entries * hm.value_size});
    }
    return vc;
}

static int run_xdp_impl(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *b, const mimic_xdp_results *res,
                        hipStream_t st_in, uint64_t first_index, const SkbRun *skb, const StepRun *step,
                        const CtxRun *cx, ManyRun *mr) {
    if (!vm || !b || !res) return MIMIC_EINVAL;
    if (prog_id >= vm->progs.size()) return fail(vm, MIMIC_EINVAL, "no program with id '%u' is loaded", prog_id);
    if (b->n > 0 && (!b->pkt_data || !b->pkt_off || !b->pkt_len)) return fail(vm, MIMIC_EINVAL, "missing packet arrays");
    if (cx && cx->all && cx->per_packet) return fail(vm, MIMIC_EINVAL, "one context for the batch or one per packet, not both");
    if (cx && cx->all && !cx->all->pinned) return fail(vm, MIMIC_EDEVICE, "the context was made without a device");
    if (cx && cx->per_packet)
        for (uint32_t i = 0; i < b->n; i++)
            if (cx->per_packet[i] && !cx->per_packet[i]->pinned)
                return fail(vm, MIMIC_EDEVICE, "packet %u: the context was made without a device", i);
    if (!skb) {
        const int rc = skb_settle(vm);
        if (rc) return rc;
    }
    if (!skb && vm->skb_leaked)   // the xdp entries would land in the freed hole or after the leaks
        return fail(vm, MIMIC_ENOTSUP, "xdp_md batches after sk_buff batches are not supported (mimic_skb_release first)");
    const uint32_t ctx = skb ? CTX_SKB : CTX_XDP;
    hipSetDevice(vm->s.device);
    int rc = upload_tables(vm);
    if (!rc) rc = flush_host(vm);   // host map operations before this batch
    if (rc) return rc;
    hipStream_t st = st_in ? st_in : vm->stream;
    const uint32_t cpu_lanes = step ? 1u : (uint32_t)vm->s.vcpu_count;
    const bool proc_jit = step && step->jit;
    // EXPLICIT batches may hold processes whose CPU ID is unset (-1) or V: two extra lanes
    bool extra = false;
    if (!step && b->schedule == MIMIC_SCHED_EXPLICIT && b->cpu)
        for (uint32_t i = 0; i < b->n && !extra; i++) extra = b->cpu[i] == -1 || b->cpu[i] == vm->s.vcpus;
    const uint32_t lanes = cpu_lanes + (extra ? 2u : 0u);
    const uint32_t S = stack_size(vm);
    // private memory: stack | xdp_md overlay | saved frames | hash key, qword-interleaved over lanes
    const PrivPlan pp = priv_plan(vm);
    const uint32_t xdp_q = pp.xdp_q, frame_q = pp.frame_q, key_q = pp.key_q, q_per_lane = pp.q_per_lane;
    const uint32_t plan = (lanes + 255) & ~255u;
    if (step) {
        if (step->priv_bytes < (uint64_t)q_per_lane * 8) return fail(vm, MIMIC_EINVAL, "process private memory too small");
    } else {
        rc = priv_ensure(vm, q_per_lane, plan, st);
        if (rc) return rc;
    }
    if (lanes > vm->lane_steps_cap) {
        hipStreamSynchronize(st);
        hipFree(vm->d_lane_steps);
        vm->d_lane_steps = nullptr;
        HIP_OK(vm, hipMalloc(&vm->d_lane_steps, (uint64_t)plan * sizeof(uint64_t)));
        vm->lane_steps_cap = plan;
    }
    KParams kp{};
    kp.insns = vm->d_insns;
    kp.progs = vm->d_progs;
    kp.segs = vm->d_segs;
    kp.maps = vm->d_maps;
    kp.arena = vm->arena;
    kp.nprogs = (uint32_t)vm->progs.size();
    kp.nsegs = (uint32_t)vm->segs.size();
    kp.nmaps = (uint32_t)vm->maps.size();
    kp.entry_prog = prog_id;
    kp.static_next = vm->next_addr;
    kp.stack_size = S;
    kp.frame_size = (uint32_t)vm->s.stack_frame_size;
    uint32_t shift = 3;  // lazy-zero granule above the first 512 stack bytes
    while (S > 512 && ((S - 512 + (1u << shift) - 1) >> shift) > 64) shift++;
    kp.chunk_shift = shift;
    kp.max_tail_calls = (uint32_t)std::max(0, vm->s.max_tail_calls);
    kp.total_vcpus = (uint32_t)vm->s.vcpus;
    kp.vcpu_begin = proc_jit ? (uint32_t)step->cpu : (uint32_t)vm->s.vcpu_begin;   // (lane 0 = the process's vCPU)
    kp.lanes = lanes;
    kp.cpu_lanes = cpu_lanes;
    kp.priv_lanes = step ? 1u : vm->priv_lanes;
    kp.priv = step ? step->priv : vm->priv;
    kp.priv_xdp_q = xdp_q;
    kp.priv_frame_q = frame_q;
    kp.priv_key_q = key_q;
    kp.budget = step ? step->budget : (b->step_budget ? b->step_budget : MIMIC_DEFAULT_BUDGET);
    kp.step = step ? step->state : nullptr;
    kp.step_gen = step ? step->gen : 0u;
    if (step) {
        kp.step_img = step->img;
        kp.step_dst = step->img_dst;
        kp.step_img_n = step->img_n;
        kp.step_ins_n = (uint32_t)std::min<size_t>(vm->h_all.size(), 2048);   // 32 KiB of LDS
    }
    kp.n = b->n;
    kp.sched = b->schedule;
    kp.pkt_data = b->pkt_data;
    kp.pkt_off = b->pkt_off;
    kp.pkt_len = b->pkt_len;
    kp.headroom_arr = b->headroom;
    kp.tailroom_arr = b->tailroom;
    kp.ingress_arr = b->ingress_ifindex;
    kp.rxq_arr = b->rx_queue_index;
    kp.egress_arr = b->egress_ifindex;
    kp.headroom = b->headroom_all;
    kp.tailroom = b->tailroom_all;
    kp.ingress = b->ingress_all;
    kp.rxq = b->rxq_all;
    kp.egress = b->egress_all;
    kp.r0 = res->r0;
    kp.status = res->status;
    kp.steps = res->steps;
    kp.err_pc = res->err_pc;
    kp.lane_steps = vm->d_lane_steps;
    if (cx && cx->all) {
        kp.cancel = cx->all->dword;
        kp.cancel_any = 1;
    } else if (cx && cx->dev_pp && b->n) {
        kp.cancel_pp = cx->dev_pp;
        kp.cancel_any = 1;
    } else if (cx && cx->per_packet && b->n) {
        std::vector<const uint32_t *> w(b->n);
        bool any = false;
        for (uint32_t i = 0; i < b->n; i++) {
            w[i] = cx->per_packet[i] ? cx->per_packet[i]->dword : nullptr;
            any |= w[i] != nullptr;
        }
        if (any) {
            // an earlier launch may still read the pointer array
            if (vm->cancel_pp_stream) hipStreamSynchronize(vm->cancel_pp_stream);
            hipStreamSynchronize(st);
            vm->cancel_pp_stream = st;
            if (b->n > vm->cancel_pp_cap) {
                hipFree(vm->d_cancel_pp);
                vm->d_cancel_pp = nullptr;
                HIP_OK(vm, hipMalloc(&vm->d_cancel_pp, (size_t)b->n * sizeof(void *)));
                vm->cancel_pp_cap = b->n;
            }
            HIP_OK(vm, hipMemcpy(vm->d_cancel_pp, w.data(), (size_t)b->n * sizeof(void *), hipMemcpyHostToDevice));
            kp.cancel_pp = vm->d_cancel_pp;
            kp.cancel_any = 1;
        }
    }
    switch (b->schedule) {
    case MIMIC_SCHED_CHUNKED:
        kp.per_lane = lanes ? (uint32_t)(((uint64_t)b->n + lanes - 1) / lanes) : 0;
        break;
    case MIMIC_SCHED_INTERLEAVED:
        kp.sched_shift = lanes ? (uint32_t)(first_index % lanes) : 0;
        kp.per_lane = lanes ? (uint32_t)(((uint64_t)b->n + kp.sched_shift + lanes - 1) / lanes) : 0;
        break;
    case MIMIC_SCHED_EXPLICIT: {
        if (!b->cpu && b->n) return fail(vm, MIMIC_EINVAL, "explicit schedule needs cpu[]");
        // stable counting sort of packets by vCPU (each vCPU runs its packets in order)
        std::vector<uint32_t> start(lanes + 1, 0), pk(b->n);
        std::vector<uint32_t> lane_of(b->n);
        for (uint32_t i = 0; i < b->n; i++) {
            const int32_t id = b->cpu[i];
            int64_t c = (int64_t)id - vm->s.vcpu_begin;
            if (id == -1) c = cpu_lanes;                       // SetCPUID never called (vm.go:214)
            else if (id == vm->s.vcpus) c = cpu_lanes + 1;     // accepted by SetCPUID (vm.go:273)
            else if (c < 0 || c >= (int64_t)cpu_lanes)
                return fail(vm, MIMIC_EINVAL, "packet %u: cpu %d not on this engine", i, id);
            lane_of[i] = (uint32_t)c;
            start[c + 1]++;
        }
        uint32_t mx = 0;
        for (uint32_t c = 0; c < lanes; c++) {
            mx = std::max(mx, start[c + 1]);
            start[c + 1] += start[c];
        }
        std::vector<uint32_t> fill(start.begin(), start.end() - 1);
        for (uint32_t i = 0; i < b->n; i++) pk[fill[lane_of[i]]++] = i;
        hipStreamSynchronize(st);
        if (start.size() > vm->sched_cap_start) {
            hipFree(vm->d_sched_start);
            vm->d_sched_start = nullptr;
            HIP_OK(vm, hipMalloc(&vm->d_sched_start, start.size() * 4));
            vm->sched_cap_start = start.size();
        }
        if (pk.size() > vm->sched_cap_pkts || !vm->d_sched_pkts) {
            hipFree(vm->d_sched_pkts);
            vm->d_sched_pkts = nullptr;
            HIP_OK(vm, hipMalloc(&vm->d_sched_pkts, std::max<size_t>(pk.size(), 1) * 4));
            vm->sched_cap_pkts = std::max<size_t>(pk.size(), 1);
        }
        HIP_OK(vm, hipMemcpy(vm->d_sched_start, start.data(), start.size() * 4, hipMemcpyHostToDevice));
        if (!pk.empty()) HIP_OK(vm, hipMemcpy(vm->d_sched_pkts, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
        kp.sched_start = vm->d_sched_start;
        kp.sched_pkts = vm->d_sched_pkts;
        kp.per_lane = mx;
        break;
    }
    default:
        return fail(vm, MIMIC_EINVAL, "unknown schedule %u", b->schedule);
    }
    // stepping runs on the interpreter; a Run the engine chose for the single-process JIT form
    // (process_advance) on that form
    bool jit = vm->exec_mode == MIMIC_EXEC_JIT && (!step || proc_jit);
    if (jit && !proc_jit && !vm->jit_fn[ctx]) {
        std::string log;
        const std::vector<std::pair<uint32_t, uint32_t>> vc = vc_slots_of(vm);
        if (mimic_jit_compile(vm->s.device, mimic_jit_source(vm->h_dp, vm->h_all, ctx, &vm->jit_info[ctx], &vc),
                              &vm->jit_fn[ctx], &log))
            return fail(vm, MIMIC_EDEVICE, "JIT build failed: %s", log.c_str());
        // A small kernel is built for 4 waves per SIMD (jit.cpp); when that spills, the form
        // without early packet loads (whose values are what stays live) may not: keep the one
        // with less scratch.  cfg 4: 0.136 -> 0.128 ms per launch.
        const JitInfo &j0 = vm->jit_info[ctx];
        int ls0 = 0;
        if (j0.early_loads && j0.cold_inline &&
            hipFuncGetAttribute(&ls0, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, vm->jit_fn[ctx]) == hipSuccess && ls0 > 0) {
            JitInfo j1;
            hipFunction_t f1 = nullptr;
            int ls1 = 0;
            if (!mimic_jit_compile(vm->s.device, mimic_jit_source(vm->h_dp, vm->h_all, ctx, &j1, &vc, true), &f1, &log) &&
                hipFuncGetAttribute(&ls1, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, f1) == hipSuccess && ls1 < ls0) {
                vm->jit_fn[ctx] = f1;
                vm->jit_info[ctx] = j1;
            }
        }
    }
    if (jit && !proc_jit) {  // a loop-free kernel has no budget checks: tiny budgets run on the interpreter
        const uint64_t bound = mimic_jit_step_bound(vm->jit_info[ctx], kp.max_tail_calls);
        if (bound && kp.budget < bound) jit = false;
    }
    // Spread launch (jit.cpp analyze_spread): a vCPU's packets on many lanes, for batches where
    // every vCPU has many packets (the one-lane-per-vCPU kernel would run them as one serial chain
    // per lane, e.g. V = runtime.NumCPU(), vm.go:64).  MIMIC_SPREAD=0: never; =1: whenever the
    // program set allows it; default: when n >= 8 V.
    bool spread = false, own = false;
    if (jit && !step && !skb && b->n > 0 && (b->schedule == MIMIC_SCHED_CHUNKED || b->schedule == MIMIC_SCHED_INTERLEAVED)) {
        const char *sv = getenv("MIMIC_SPREAD");
        const int knob = vm->spread_mode >= 0 ? vm->spread_mode : sv && *sv ? atoi(sv) : -1;
        // the owned form, for batches of 2..256 packets per vCPU (Q packets per thread, below): by
        // default whenever the programs and the table allow it -- classifier at V = 262 144 (cfg 2)
        // 25.0 vs 25.7 us, parse5 at V = 262 144 (cfg 3) 0.74 vs 1.03 ms, V = 16 384 with 64 packets
        // per vCPU 2x the table spread (profiles/r05/).  MIMIC_SPREAD_OWN=0: never.
        const char *ov = getenv("MIMIC_SPREAD_OWN");
        const bool own_pref = !(ov && ov[0] == '0');
        if (knob != 0 && own_pref && kp.per_lane >= 2 && kp.per_lane <= 256) {
            rc = spread_build_own(vm);
            if (rc) return rc;
            // Q packets per thread: enough threads to fill the chip about once (fewer, longer threads
            // measured faster: V = 131 072, P = 4: 17.6 us at Q = 1, 15.5 at Q = 2), a divisor of P
            // whose 256 Q / P rows fit the table (MIMIC_SPREAD_OWN_Q: a fixed Q, measurement)
            const uint32_t P = kp.per_lane, cl = chip_lanes(vm);
            const char *qv = getenv("MIMIC_SPREAD_OWN_Q");
            uint32_t q = qv && *qv ? (uint32_t)atoi(qv) : (uint32_t)std::max<uint64_t>(1, ((uint64_t)b->n + cl - 1) / cl);
            q = std::max<uint32_t>(1, std::min(q, P));
            while (q > 1 && (P % q || 256u * q / P > vm->spread_own_rows)) q--;
            kp.own_q = q;
            own = vm->spread_own_state > 0 && P % q == 0 && 256u * q / P <= vm->spread_own_rows && 256u * q / P >= 1u &&
                  mimic_jit_step_bound(vm->jit_info_spread_own, kp.max_tail_calls) <= kp.budget;
            spread = own;
        }
        if (!own && (knob == 1 || (knob != 0 && (uint64_t)b->n >= 8ull * cpu_lanes))) {
            rc = spread_build(vm);
            if (rc) return rc;
            spread = vm->spread_state > 0 && mimic_jit_step_bound(vm->jit_info_spread, kp.max_tail_calls) <= kp.budget;
            // without the LDS table every increment is a scattered agent-scope atomic: worth it only
            // when the one-lane-per-vCPU kernel has few lanes
            if (knob != 1 && !vm->spread_lds && cpu_lanes > 16384) spread = false;
        }
    }
    // a launch given contexts runs the variant with the per-packet Run(ctx) check, one lane per vCPU
    const bool cxk = jit && kp.cancel_any;
    if (cxk) {
        spread = own = false;
        if (!vm->jit_fn_cx[ctx]) {
            const std::vector<std::pair<uint32_t, uint32_t>> vc = vc_slots_of(vm);
            std::string log;
            // with or without early packet loads as the VM's own kernel (the spill choice above)
            if (mimic_jit_compile(vm->s.device,
                                  mimic_jit_source(vm->h_dp, vm->h_all, ctx, &vm->jit_info_cx[ctx], &vc,
                                                   !vm->jit_info[ctx].early_loads, nullptr, true),
                                  &vm->jit_fn_cx[ctx], &log))
                return fail(vm, MIMIC_EDEVICE, "JIT build failed: %s", log.c_str());
        }
    }
    const JitInfo &ji = proc_jit ? vm->jit_info_proc : own ? vm->jit_info_spread_own : spread ? vm->jit_info_spread
                        : cxk ? vm->jit_info_cx[ctx] : vm->jit_info[ctx];
    hipFunction_t jfn = proc_jit ? vm->jit_fn_proc : own ? vm->jit_fn_spread_own : spread ? vm->jit_fn_spread
                        : cxk ? vm->jit_fn_cx[ctx] : vm->jit_fn[ctx];
    if (proc_jit && (!jfn || !ji.proc_ok || !ji.karg)) return fail(vm, MIMIC_EDEVICE, "process: no single-process JIT kernel (engine)");
    uint32_t run_lanes = lanes;
    if (spread) {
        // owned: 256 / P vCPU lanes per block
        const uint32_t orows = own ? 256u / (kp.per_lane / kp.own_q) : 1u;
        const uint32_t blocks = own ? (cpu_lanes + orows - 1) / orows
                                    : (uint32_t)(((uint64_t)b->n + spread_ppb() - 1) / spread_ppb());
        run_lanes = blocks * 256u;
        rc = priv_ensure(vm, q_per_lane, run_lanes, st);   // private memory (stack ...) per spread lane
        if (rc) return rc;
        if (run_lanes > vm->lane_steps_cap) {
            hipStreamSynchronize(st);
            hipFree(vm->d_lane_steps);
            vm->d_lane_steps = nullptr;
            HIP_OK(vm, hipMalloc(&vm->d_lane_steps, (uint64_t)run_lanes * sizeof(uint64_t)));
            vm->lane_steps_cap = run_lanes;
        }
        if (!vm->d_spread_bad) {
            HIP_OK(vm, hipMalloc(&vm->d_spread_bad, 64));
            HIP_OK(vm, hipMemset(vm->d_spread_bad, 0, 64));
        }
        kp.lanes = run_lanes;
        kp.priv = vm->priv;
        kp.priv_lanes = vm->priv_lanes;
        kp.lane_steps = vm->d_lane_steps;
        kp.spread_bad = vm->d_spread_bad;
        vm->spread_used = true;
        // an LDS table that covers every lane and has no more counters than a block has packets
        // (dense): the blocks' tables go to a buffer and one reduce kernel adds them into the map
        // (jit.cpp spread flush).  Sparser tables keep one agent-scope add per non-zero counter.
        kp.spread_part = nullptr;
        if (!own && ji.spread_rows && ji.spread_rows == cpu_lanes && ji.spread_n &&
            (uint64_t)cpu_lanes * ji.spread_roww <= spread_ppb()) {
            const uint64_t need = (uint64_t)blocks * ji.spread_rows * ji.spread_roww * ji.spread_n;
            if (need > vm->spread_part_cap) {
                HIP_OK(vm, hipStreamSynchronize(st));
                hipFree(vm->d_spread_part);
                vm->d_spread_part = nullptr;
                HIP_OK(vm, hipMalloc(&vm->d_spread_part, need));
                vm->spread_part_cap = need;
            }
            kp.spread_part = vm->d_spread_part;
        }
    }
    kp.skb_rec_built = 1;
    if (skb && step && step->skb_rec) {   // a stepped sk_buff process: Load ran at NewProcess
        kp.ctx_kind = CTX_SKB;
        kp.skb_ifindex = skb->ifindex;
        kp.skb_rec = step->skb_rec;
        kp.skb_prefix = step->skb_prefix;
        kp.skb_base = step->skb_base;
        kp.skb_custom = step->skb_custom;
    } else if (skb && skb->pre_drv) {   // processes loaded at NewProcess (mimic_process_run_many)
        rc = skb_ensure(vm, b->n, st);   // kp.skb_rec: where deferred lanes and the interpreter keep records
        if (rc) return rc;
        kp.ctx_kind = CTX_SKB;
        kp.skb_ifindex = skb->ifindex;
        kp.skb_rec = vm->d_skb_rec;
        kp.skb_drv = skb->pre_drv;
        kp.skb_prefix = skb->pre_prefix;
        kp.skb_base = skb->pre_base;
        kp.skb_custom = skb->custom;
        vm->skb_stream = st;
    } else if (skb) {
        // a JIT kernel that walks the headers itself needs the footprints only; one that derives the
        // common frames' records itself (skb_load_fast): exception records only
        const bool own_recs = jit && ji.skb_walk, sparse = jit && ji.skb_fast;
        rc = skb_prepare(vm, b, st, nullptr, !own_recs, sparse, skb->rooms_state);
        if (rc) return rc;
        kp.skb_rooms_state = skb->rooms_state;
        kp.skb_rec_built = own_recs ? 0u : sparse ? 2u : 1u;
        kp.ctx_kind = CTX_SKB;
        kp.skb_ifindex = skb->ifindex;
        kp.skb_rec = vm->d_skb_rec;
        kp.skb_drv = own_recs ? nullptr : vm->d_skb_drv;
        kp.skb_prefix = vm->d_skb_prefix;
        kp.skb_base = vm->d_skb_state + 1;
        kp.skb_custom = skb->custom;
    }
    // compact hash tables whose buckets are mostly tombstones (device-side check, no host sync)
    // (skipped while no delete can have run on the map: without tombstones live entries stay
    // below half of the table, so the check would always decline -- and a kernel between the
    // batches costs a launch gap)
    // A launch whose programs never delete pops the freelists without the `avail` semaphore
    // (hashmap.h h_insert_wave pop_only); one that may delete first normalises maps left so.
    kp.hash_pop_only = vm->prog_deletes ? 0u : 1u;
    // no program can write a hash map: during the launch every table is read-only
    kp.hash_ro = (vm->prog_deletes || vm->prog_updates) ? 0u : 1u;
    for (auto &m : vm->maps) {
        if (!is_hash(m)) continue;
        if (m.share) {   // one table with other VMs' maps: their staged host writes first
            if ((rc = share_check(vm, m))) return rc;
            for (auto &mb : m.share->members) {
                mimic_vm *o = (mimic_vm *)mb.vm;
                if (o != vm && o->host_dirty && (rc = flush_host(o))) return fail(vm, rc, "shared map: %s", o->err.c_str());
            }
            share_stale(m);   // this launch may write the table: every member's image
        }
        const DMap dm = to_dmap(m);
        if (vm->prog_deletes && m.pop_dirty) {
            if (mimic_launch_hash_normalize(vm->arena, &dm, st))
                return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
            m.pop_dirty = false;
        }
        if (!vm->prog_deletes) m.pop_dirty = true;
        if (vm->prog_deletes) m.may_tomb = true;
        // the launch may change the table (or the rebuild below may): the host image is stale
        if (m.mir && (vm->prog_updates || vm->prog_deletes || m.may_tomb)) m.mir->valid = false;
        if (!m.may_tomb) continue;
        if (mimic_launch_hash_rebuild(vm->arena, &dm, 0, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
    }
    vm->last_exec = jit ? (own ? MIMIC_EXEC_SPREAD_OWN : spread ? MIMIC_EXEC_SPREAD : MIMIC_EXEC_JIT) : MIMIC_EXEC_INTERP;
    if (jit && ji.defer) {   // the lanes' suspended processes (DeferRec) and the launch's marker
        if (lanes > vm->defer_cap || !vm->d_defer_any) {
            hipStreamSynchronize(st);
            hipFree(vm->d_defer);
            vm->d_defer = nullptr;
            HIP_OK(vm, hipMalloc(&vm->d_defer, (uint64_t)plan * sizeof(DeferRec)));
            HIP_OK(vm, hipMemset(vm->d_defer, 0, (uint64_t)plan * sizeof(DeferRec)));
            vm->defer_cap = plan;
            if (!vm->d_defer_any) {
                HIP_OK(vm, hipMalloc(&vm->d_defer_any, 64));
                HIP_OK(vm, hipMemset(vm->d_defer_any, 0, 64));
            }
        }
        if (++vm->defer_epoch == 0) vm->defer_epoch = 1;   // 0 is what the buffers start as
        kp.defer = vm->d_defer;
        kp.defer_any = vm->d_defer_any;
        kp.defer_epoch = vm->defer_epoch;
    }
    if (jit && ji.hash_combine) vm->comb_used = true;
    if (mr) {   // every batch of a multi-batch launch in this one (the owned form only: jit.cpp)
        mr->used = jit && own && !ji.defer && mr->k >= 1 && mr->k <= MIMIC_MANY_MAX;
        if (mr->used) {
            kp.many_n = mr->k;
            for (uint32_t q = 0; q < mr->k; q++)
                kp.many[q] = BatchRef{mr->b[q].pkt_data, mr->b[q].pkt_off, mr->b[q].pkt_len, mr->r[q].r0, mr->r[q].status,
                                      mr->r[q].steps, mr->r[q].err_pc, 0};
        }
    }
    if (jit && ji.karg) {  // launch parameters by value: the runtime copies them into the kernarg segment
        if (mimic_jit_launch(jfn, ji, &kp, nullptr, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
        // the interpreter finishes what the kernel deferred (a wave without a deferred lane returns at once)
        if (ji.defer && mimic_launch_xdp_resume(&kp, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
    } else if (step) {   // the stepping kernel takes its parameters by value: no slot, no copy
        if (mimic_launch_xdp(&kp, nullptr, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
    } else {  // launch parameters are read from a device copy
        const KParams *dkp = nullptr;
        const int slot = kp_slot(vm, kp, st, &dkp);
        if (slot < 0) return slot;
        if (jit ? mimic_jit_launch(jfn, ji, &kp, dkp, st) : mimic_launch_xdp(&kp, dkp, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
        if (jit && ji.defer && mimic_launch_xdp_resume(&kp, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
        HIP_OK(vm, hipEventRecord(vm->kp_ev[slot], st));   // the slot is free again once this passes
        vm->kp_used[slot] = true;
    }
    if (jit && ji.hash_chunk) {   // the chunk map's holes filled (interp.hip mimic_hash_compact_kernel)
        for (const HostMap &m : vm->maps) {
            if (!m.chunk) continue;
            const DMap dm = to_dmap(m);
            if (mimic_launch_hash_compact(vm->arena, &dm, st))
                return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
        }
    }
    if (jit && kp.spread_part) {   // a spread launch's block counter tables into the map
        const DMap dm = to_dmap(vm->maps[ji.spread_map]);
        if (mimic_launch_spread_reduce(kp.spread_part, kp.lanes / 256u, kp.cpu_lanes, ji.spread_roww, ji.spread_n,
                                       vm->arena + dm.dev_off + (uint64_t)kp.vcpu_begin * dm.dev_stride, dm.dev_stride, st))
            return fail(vm, MIMIC_EDEVICE, "launch: %s", hipGetErrorString(hipGetLastError()));
    }
    if (kp.cancel_any) {   // the contexts' words are read until these launches end (mimic_ctx_free waits)
        auto mark = [&](mimic_ctx *c) -> int {
            std::lock_guard<std::mutex> lk(c->mu);
            std::vector<hipEvent_t> keep;   // finished uses are dropped
            for (hipEvent_t e : c->uses) {
                if (hipEventQuery(e) == hipSuccess) hipEventDestroy(e);
                else keep.push_back(e);
            }
            c->uses.swap(keep);
            hipEvent_t ev = nullptr;
            HIP_OK(vm, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_OK(vm, hipEventRecord(ev, st));
            c->uses.push_back(ev);
            return 0;
        };
        if (cx->all) {
            if ((rc = mark(cx->all))) return rc;
        } else {
            std::vector<mimic_ctx *> u;
            for (uint32_t i = 0; i < b->n; i++)
                if (cx->per_packet[i]) u.push_back(cx->per_packet[i]);
            std::sort(u.begin(), u.end());
            u.erase(std::unique(u.begin(), u.end()), u.end());
            for (mimic_ctx *c : u)
                if ((rc = mark(c))) return rc;
        }
    }
    vm->last_lanes = run_lanes;
    vm->last_stream = st;
    return 0;
}

}  // extern "C"

// A single process's memory (NewProcess, vm.go:198-235).  Its device block holds
//   descriptor (pkt_off = 0, pkt_len) | sk_buff memory @PD_SKB: SkbRec | prefix (2 words) | base |
//   mimic_skb_custom | packet memory @PD_PKT (headroom + len + tailroom)
// and the pinned, device-mapped host half of the same block holds
//   StepState @0 | one-packet results @PH_RES: r0 | status | steps | err_pc | a read-back word |
//   the device block's upload image @PH_IMG.
// The stepping kernel reads and writes the StepState and the results in place, so a Run / Step is
// one launch and one host sync, and NewProcess is one asynchronous copy of the image (no sync).
namespace {
constexpr size_t PD_LEN = 8, PD_SKB = 64;
constexpr size_t PD_PKT = (PD_SKB + sizeof(SkbRec) + 24 + sizeof(mimic_skb_custom) + 63) & ~(size_t)63;
constexpr size_t PH_RES = (sizeof(StepState) + 63) & ~(size_t)63;
constexpr size_t PH_R0 = PH_RES, PH_ST = PH_RES + 8, PH_STEPS = PH_RES + 16, PH_EPC = PH_RES + 20, PH_WORD = PH_RES + 24;
constexpr size_t PH_IMG = PH_RES + 64;
}  // namespace

struct mimic_process {
    mimic_vm *vm = nullptr;
    uint32_t prog = 0;
    uint32_t H = 0, T = 0, len = 0;
    int32_t ingress = 0, rxq = 0, egress = 0;
    uint8_t *d_pkt = nullptr;         // packet memory H + len + T (device)
    uint8_t *d_skbmem = nullptr;      // SkbRec | prefix (2 words) | base | mimic_skb_custom (device)
    StepState *hs = nullptr;          // the state in the pinned host half ...
    StepState *hs_dev = nullptr;      // ... and its device-visible address
    uint8_t *hres = nullptr, *hres_dev = nullptr;   // the one-packet results, likewise
    uint64_t priv_bytes = 0;
    StepState h;                      // host copy after the last launch
    int32_t cpu = -1;
    uint32_t gen = 0;                 // NewProcess number: the StepState generation its launches expect
    uint32_t static_next = 0;         // the VM's static layout the saved state's addresses assume
    uint8_t *arena = nullptr;
    // LinuxContextSKBuff processes (context_sk_buff.go): the record, leak prefix (0) and leak base
    // of the process's Load, made at NewProcess like the reference's
    bool skb = false;
    bool skb_custom = false;          // a user-given sock / flow keys after the base word
    uint32_t ifindex = 0;
    Blk mem;                          // the block above
    Blk priv;                         // private memory (stack, frames, ...): device only
    uint64_t last_seq = 0;            // vm->seq number of the last work enqueued that touches mem / priv
    bool uploaded = false;            // the device block holds the NewProcess image (else only the host half)
    size_t img_n = 0;                 // the image's bytes (the device block's [0, img_n))
};

// blocks of single processes, from the VM's cache (one hipMalloc / hipHostMalloc per size class ever)
static bool proc_alloc(mimic_vm *vm, size_t n, bool host, Blk *out) {
    if (vm->blk.take(n, host, out)) return true;
    out->cls = BlkCache::size_class(n);
    if (hipMalloc(&out->dev, out->cls) != hipSuccess) {
        (void)hipGetLastError();
        *out = Blk{};
        return false;
    }
    if (host) {
        void *h = nullptr, *d = nullptr;
        if (hipHostMalloc(&h, out->cls, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            hipFree(out->dev);
            *out = Blk{};
            return false;
        }
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            (void)hipGetLastError();
            d = h;
        }
        out->host = (uint8_t *)h;
        out->hdev = (uint8_t *)d;
    }
    return true;
}
// run_mu held: work touching p's memory was just enqueued on vm->stream
static void proc_enq(mimic_process *p) { p->last_seq = p->vm->seq.next(); }
// run_mu held: the host sync of a process operation
static hipError_t proc_sync(mimic_vm *vm) {
    const uint64_t upto = vm->seq.issued();
    const hipError_t e = hipStreamSynchronize(vm->stream);
    if (e == hipSuccess) vm->seq.complete(upto);
    return e;
}
// the fence a block released now must carry: null when its last enqueue `seq` is known complete,
// else an event behind everything enqueued on vm->stream so far
static std::shared_ptr<BlkFence> proc_fence(mimic_vm *vm, uint64_t seq) {
    if (vm->seq.idle(seq)) return nullptr;
    auto f = std::make_shared<HipFence>();
    f->st = vm->stream;
    if (hipEventCreateWithFlags(&f->ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(f->ev, vm->stream) == hipSuccess)
        return f;
    (void)hipGetLastError();
    hipStreamSynchronize(vm->stream);   // no event: wait for the stream instead
    return nullptr;
}
static void proc_release_blk(mimic_vm *vm, Blk &b, const std::shared_ptr<BlkFence> &fence) {
    if (b.dev && !vm->blk.give(b, fence)) {   // the cache is full
        if (fence) fence->wait();
        hipFree(b.dev);
        if (b.host) hipHostFree(b.host);
    }
    b = Blk{};
}
static void process_release(mimic_process *p, const std::shared_ptr<BlkFence> &fence) {
    proc_release_blk(p->vm, p->mem, fence);
    proc_release_blk(p->vm, p->priv, fence);
}

static void process_regs(const mimic_process *p, mimic_process_regs *out) {
    if (!out) return;
    memset(out, 0, sizeof *out);
    for (int q = 0; q < 11; q++) out->r[q] = p->h.r[q];
    out->pc = p->h.pc;
    out->prog_id = p->h.started ? p->h.prog : p->prog;
    out->steps = p->h.steps;
    out->status = p->h.finished ? p->h.status : MIMIC_OK;
    out->exited = p->h.finished;
}

// one launch: run the process until `budget` total steps (or exit / error), then one host sync.
// The kernel restores the state from the pinned host half and saves it there (interp.hip MODE_STEP);
// nothing else of the process is in flight then (every operation on it ends with a sync, and its
// NewProcess upload precedes this launch on the same stream).
// Process.Run tiering (mimic_vm::proc_jit_after): the program set's single-process JIT form, built
// once per program set; false when it is not usable (then Runs stay on the interpreter)
static bool proc_jit_ready(mimic_vm *vm) {
    if (vm->proc_jit == 0) {
        vm->proc_jit = -1;
        const std::vector<std::pair<uint32_t, uint32_t>> vc = vc_slots_of(vm);
        std::string log;
        JitInfo ji{};
        hipFunction_t fn = nullptr;
        const std::string src = mimic_jit_source(vm->h_dp, vm->h_all, CTX_XDP, &ji, &vc, false, nullptr, false, true);
        if (ji.proc_ok && ji.karg && !mimic_jit_compile(vm->s.device, src, &fn, &log)) {
            vm->jit_fn_proc = fn;
            vm->jit_info_proc = ji;
            vm->proc_jit = 1;
        }
    }
    return vm->proc_jit > 0;
}
// a Run (not a Step) of a process that has not started, on one of this engine's vCPUs, with a
// budget the loop-free form cannot exceed, once the VM has made enough Runs
static bool proc_jit_use(mimic_process *p, uint64_t budget) {
    mimic_vm *vm = p->vm;
    if (vm->exec_mode != MIMIC_EXEC_JIT || vm->proc_jit_after < 0 || p->skb || p->h.started) return false;
    if (p->cpu < vm->s.vcpu_begin || p->cpu >= vm->s.vcpu_begin + vm->s.vcpu_count) return false;
    if (vm->proc_runs++ < (uint64_t)vm->proc_jit_after || !proc_jit_ready(vm)) return false;
    const uint64_t bound = mimic_jit_step_bound(vm->jit_info_proc, (uint32_t)std::max(0, vm->s.max_tail_calls));
    return bound && bound <= budget;
}

static int process_advance(mimic_process *p, uint64_t budget, bool run = false) {
    mimic_vm *vm = p->vm;
    std::lock_guard<std::recursive_mutex> lk(vm->run_mu);
    hipSetDevice(vm->s.device);
    // the VM may have grown (maps / programs) since the process was made: its private plan too
    const PrivPlan pp = priv_plan(vm);
    // a started process's saved registers, stack / packet pointers and translation cache hold
    // addresses of the layout it started in: a map or program loaded since moved its entries
    // (the reference's entries would have stayed put) and may have moved the arena
    if (p->h.started && (vm->next_addr != p->static_next || vm->arena != p->arena))
        return fail(vm, MIMIC_ENOTSUP, "a map or program was loaded after the process started; its layout changed");
    if ((uint64_t)pp.q_per_lane * 8 > p->priv_bytes && p->h.started)
        return fail(vm, MIMIC_ENOTSUP, "the VM's process layout changed under a started process");
    p->static_next = vm->next_addr;
    p->arena = vm->arena;
    if ((uint64_t)pp.q_per_lane * 8 > p->priv_bytes) {
        proc_release_blk(vm, p->priv, proc_fence(vm, p->last_seq));
        p->priv_bytes = (uint64_t)pp.q_per_lane * 8;
        if (!proc_alloc(vm, p->priv_bytes, false, &p->priv)) return fail(vm, MIMIC_ENOMEM, "process private memory");
    }
    StepState *S = p->hs;
    *S = p->h;
    S->cpu = p->cpu;
    S->gen = p->gen;
    p->hres[PH_ST - PH_RES] = 0xff;
    mimic_xdp_batch b{};
    b.n = 1;
    b.schedule = MIMIC_SCHED_CHUNKED;
    b.pkt_data = p->d_pkt;
    b.pkt_off = (const uint64_t *)p->mem.dev;
    b.pkt_len = (const uint32_t *)(p->mem.dev + PD_LEN);
    b.headroom_all = p->H;
    b.tailroom_all = p->T;
    b.ingress_all = p->ingress;
    b.rxq_all = p->rxq;
    b.egress_all = p->egress;
    mimic_xdp_results r{};
    r.r0 = (uint64_t *)(p->hres_dev + (PH_R0 - PH_RES));
    r.status = p->hres_dev + (PH_ST - PH_RES);
    r.steps = (uint32_t *)(p->hres_dev + (PH_STEPS - PH_RES));
    r.err_pc = (int32_t *)(p->hres_dev + (PH_EPC - PH_RES));
    StepRun sr{p->hs_dev, p->priv.dev, p->priv_bytes, budget};
    sr.gen = p->gen;
    if (run && !upload_tables(vm) && proc_jit_use(p, budget)) {   // (the tables the form is built from first)
        // the compiled program on lane 0 = the process's vCPU; a process whose image is still only
        // in the pinned half runs on it there (its packet bytes read and written over the bus, no
        // upload copy ahead of the launch: mimic_process_packet reads that half while !uploaded)
        sr.jit = true;
        sr.cpu = p->cpu;
        if (!p->uploaded) {
            uint8_t *img = p->mem.hdev + PH_IMG;
            b.pkt_data = img + PD_PKT;
            b.pkt_off = (const uint64_t *)img;
            b.pkt_len = (const uint32_t *)(img + PD_LEN);
        }
    } else if (!p->uploaded) {   // the kernel copies the image in before the process's first step
        sr.img = p->mem.hdev + PH_IMG;
        sr.img_dst = p->mem.dev;
        sr.img_n = (uint32_t)p->img_n;
    }
    SkbRun skr{p->ifindex};
    if (p->skb) {
        sr.skb_rec = (SkbRec *)p->d_skbmem;
        sr.skb_prefix = (const uint64_t *)(p->d_skbmem + sizeof(SkbRec));
        sr.skb_base = (const uint64_t *)(p->d_skbmem + sizeof(SkbRec) + 16);
        if (p->skb_custom) sr.skb_custom = (const mimic_skb_custom *)(p->d_skbmem + sizeof(SkbRec) + 24);
    }
    const int rc = run_xdp_impl(vm, p->prog, &b, &r, vm->stream, 0, p->skb ? &skr : nullptr, &sr);
    proc_enq(p);
    const hipError_t e = proc_sync(vm);   // the one host sync of Run / Step
    if (rc) return rc;
    if (!sr.jit) p->uploaded = true;
    if (e != hipSuccess) return fail(vm, MIMIC_EDEVICE, "process: %s", hipGetErrorString(e));
    if (p->hres[PH_ST - PH_RES] == MIMIC_ERR_ENGINE_STATE || S->gen != p->gen)
        return fail(vm, MIMIC_EDEVICE, "process: the stepping launch found another process's state (engine assertion)");
    p->h = *S;
    return 0;
}

extern "C" {

// NewProcess: the process's block, its upload image written in the pinned half and copied to the
// device with one asynchronous copy on vm->stream (run_mu held)
static int process_make(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t headroom,
                        uint32_t tailroom, int32_t ingress_ifindex, int32_t rx_queue_index, int32_t egress_ifindex,
                        const mimic_skb_custom *custom, bool upload, mimic_process **out) {
    hipSetDevice(vm->s.device);
    const uint64_t M = (uint64_t)headroom + len + tailroom;
    const size_t total = PD_PKT + (size_t)std::max<uint64_t>(M, 1);
    mimic_process *p = new mimic_process();
    p->vm = vm;
    p->prog = prog_id;
    p->H = headroom;
    p->T = tailroom;
    p->len = len;
    p->ingress = ingress_ifindex;
    p->rxq = rx_queue_index;
    p->egress = egress_ifindex;
    if (!proc_alloc(vm, PH_IMG + total, true, &p->mem)) {
        delete p;
        return fail(vm, MIMIC_ENOMEM, "process memory");
    }
    p->gen = ++vm->proc_gen;
    memset(&p->h, 0, sizeof p->h);
    p->h.gen = p->gen;
    uint8_t *hb = p->mem.host, *db = p->mem.dev;
    p->hs = (StepState *)hb;
    p->hs_dev = (StepState *)p->mem.hdev;
    p->hres = hb + PH_RES;
    p->hres_dev = p->mem.hdev + PH_RES;
    p->d_skbmem = db + PD_SKB;
    p->d_pkt = db + PD_PKT;
    // the image: descriptor (off 0, len), zeroed sk_buff memory and rooms, the packet at +headroom,
    // a user-given sock / flow keys after the record's base word
    uint8_t *img = hb + PH_IMG;
    memset(img, 0, PD_PKT + headroom);
    memcpy(img + PD_LEN, &len, 4);
    if (custom) memcpy(img + PD_SKB + sizeof(SkbRec) + 24, custom, sizeof *custom);
    if (len) memcpy(img + PD_PKT + headroom, packet, len);
    memset(img + PD_PKT + headroom + len, 0, total - (PD_PKT + headroom + len));
    p->img_n = total;
    // an xdp_md process's first launch copies the image itself (interp.hip MODE_STEP); an sk_buff
    // process's Load runs now and needs it on the device
    const hipError_t e = upload ? hipMemcpyAsync(db, img, total, hipMemcpyHostToDevice, vm->stream) : hipSuccess;
    if (upload) {
        proc_enq(p);
        p->uploaded = true;
    }
    if (e != hipSuccess) {
        process_release(p, proc_fence(vm, p->last_seq));
        delete p;
        return fail(vm, MIMIC_EDEVICE, "process: %s", hipGetErrorString(e));
    }
    *out = p;
    return 0;
}

int mimic_process_new(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t headroom,
                      uint32_t tailroom, int32_t ingress_ifindex, int32_t rx_queue_index, int32_t egress_ifindex,
                      mimic_process **out) {
    if (!vm || !out || (len && !packet)) return MIMIC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(vm->run_mu);
    if (prog_id >= vm->progs.size()) return fail(vm, MIMIC_EINVAL, "no program with id '%u' is loaded", prog_id);
    if (vm->skb_leaked) return fail(vm, MIMIC_ENOTSUP, "xdp_md processes after sk_buff batches are not supported");
    return process_make(vm, prog_id, packet, len, headroom, tailroom, ingress_ifindex, rx_queue_index, egress_ifindex,
                        nullptr, false, out);
}

int mimic_process_new_skb(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t ifindex,
                          mimic_process **out) {
    return mimic_process_new_skb_ctx(vm, prog_id, packet, len, ifindex, nullptr, out);
}

int mimic_process_new_skb_ctx(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t ifindex,
                              const mimic_skb_custom *custom, mimic_process **out) {
    if (!vm || !out || (len && !packet)) return MIMIC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(vm->run_mu);
    if (prog_id >= vm->progs.size()) return fail(vm, MIMIC_EINVAL, "no program with id '%u' is loaded", prog_id);
    // the packet memory is SKB_HEADROOM + len + SKB_TAILROOM with the frame at +SKB_HEADROOM
    // (context_sk_buff.go:42-107), run by the interpreter's stepping kernel as a one-packet batch
    const bool cust = custom && custom->flags;
    int rc = process_make(vm, prog_id, packet, len, SKB_HEADROOM, SKB_TAILROOM, 0, 0, 0, cust ? custom : nullptr, true, out);
    if (rc) return rc;
    mimic_process *p = *out;
    p->skb = true;
    p->ifindex = ifindex;
    p->skb_custom = cust;
    auto drop = [&](int code, const char *what) {
        mimic_process_free(p);
        *out = nullptr;
        return code == MIMIC_EDEVICE && what ? fail(vm, code, "process: %s", what) : code;
    };
    // LinuxContextSKBuff.Load now, as NewProcess does in the reference: the record and the leak
    // addresses (the VM's leak cursor moves past this process's sock / flow keys / packet)
    if ((rc = upload_tables(vm))) return drop(rc, nullptr);
    mimic_xdp_batch b{};
    b.n = 1;
    b.pkt_data = p->d_pkt;
    b.pkt_off = (const uint64_t *)p->mem.dev;
    b.pkt_len = (const uint32_t *)(p->mem.dev + PD_LEN);
    // d_skbmem: the record | its 2 prefix words | the batch base
    const SkbInto into{(SkbRec *)p->d_skbmem, (uint64_t *)(p->d_skbmem + sizeof(SkbRec))};
    if ((rc = skb_prepare(vm, &b, vm->stream, &into))) return drop(rc, nullptr);
    hipError_t e = hipMemcpyAsync(p->d_skbmem + sizeof(SkbRec) + 16, vm->d_skb_state + 1, 8, hipMemcpyDeviceToDevice,
                                  vm->stream);
    uint32_t *lw = (uint32_t *)(p->hres + (PH_WORD - PH_RES));   // SkbRec.len, read back into the pinned half
    if (e == hipSuccess) e = hipMemcpyAsync(lw, p->d_skbmem, 4, hipMemcpyDeviceToHost, vm->stream);
    proc_enq(p);
    const hipError_t es = proc_sync(vm);
    if (e == hipSuccess) e = es;
    if (e != hipSuccess) return drop(MIMIC_EDEVICE, hipGetErrorString(e));
    if (*lw & SKB_LOAD_FAILED) {   // NewProcess returns the context's Load error (vm.go:226-229); nothing leaked
        mimic_process_free(p);
        *out = nullptr;
        return fail(vm, MIMIC_EINVAL, "load context: the sk_buff context did not decode (ERR_CTX_LOAD)");
    }
    return 0;
}

int mimic_process_set_cpu(mimic_process *p, int32_t id) {
    if (!p) return MIMIC_EINVAL;
    if (id < 0) return fail(p->vm, MIMIC_EINVAL, "not a valid CPU ID");
    if (id > p->vm->s.vcpus)
        return fail(p->vm, MIMIC_EINVAL, "vm only has %d vCPUs, max CPU ID is %d", p->vm->s.vcpus, p->vm->s.vcpus - 1);
    p->cpu = id;
    return 0;
}

int mimic_process_step(mimic_process *p, uint32_t n, mimic_process_regs *out) {
    if (!p) return MIMIC_EINVAL;
    if (p->h.finished) {
        process_regs(p, out);
        // a clean exit leaves PC on the exit instruction: stepping it again exits again
        return p->h.status == MIMIC_OK ? 0 : fail(p->vm, MIMIC_EINVAL, "process has been terminated");
    }
    if (n) {
        const int rc = process_advance(p, (uint64_t)p->h.steps + n);
        if (rc) return rc;
    }
    process_regs(p, out);
    return 0;
}

int mimic_process_run(mimic_process *p, uint64_t budget, mimic_process_regs *out) {
    if (!p) return MIMIC_EINVAL;
    if (p->h.finished) return mimic_process_step(p, 0, out);
    const int rc = process_advance(p, (uint64_t)p->h.steps + (budget ? budget : MIMIC_DEFAULT_BUDGET), true);
    if (rc) return rc;
    process_regs(p, out);
    return 0;
}

// ---- context.Context (Run(ctx), vm.go:343-360) ------------------------------------------------
int mimic_ctx_new(uint64_t timeout_ns, mimic_ctx **out) {
    if (!out) return MIMIC_EINVAL;
    mimic_ctx *c = new mimic_ctx();
    void *w = nullptr;
    if (hipHostMalloc(&w, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
        void *d = nullptr;
        if (hipHostGetDevicePointer(&d, w, 0) != hipSuccess) d = w;
        c->word = (uint32_t *)w;
        c->dword = (uint32_t *)d;
        c->pinned = true;
    } else {
        (void)hipGetLastError();
        c->word = (uint32_t *)calloc(1, 64);
        if (!c->word) {
            delete c;
            return MIMIC_ENOMEM;
        }
    }
    *c->word = 0;
    if (timeout_ns) {   // context.WithTimeout: a timer sets DeadlineExceeded unless freed first
        const auto until = std::chrono::steady_clock::now() + std::chrono::nanoseconds(timeout_ns);
        c->timer = std::thread([c, until] {
            std::unique_lock<std::mutex> lk(c->mu);
            if (!c->cv.wait_until(lk, until, [c] { return c->closing; })) ctx_set(c, 2);
        });
    }
    *out = c;
    return 0;
}

void mimic_ctx_cancel(mimic_ctx *c) {
    if (c) ctx_set(c, 1);
}

int mimic_ctx_err(const mimic_ctx *c) { return c ? (int)ctx_get(c) : MIMIC_EINVAL; }

int mimic_ctx_pinned(const mimic_ctx *c) { return c ? (int)c->pinned : MIMIC_EINVAL; }

void mimic_ctx_free(mimic_ctx *c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        c->closing = true;
    }
    c->cv.notify_all();
    if (c->timer.joinable()) c->timer.join();
    for (hipEvent_t e : c->uses) {
        hipEventSynchronize(e);
        hipEventDestroy(e);
    }
    if (c->pinned) hipHostFree(c->word);
    else free(c->word);
    delete c;
}

// Process.Run(ctx): the process advances in launches of a growing number of steps and the context
// is checked before each (the reference checks before every step, vm.go:344-349: here a cancel is
// seen within one launch).  Done: MIMIC_ECANCELED / MIMIC_EDEADLINE (ctx.Err()) with the process
// suspended where it stopped -- Run or Step continue it.  budget 0 with a context: no step budget
// (the context bounds the run, as in the reference; the step counter is 32 bits).
int mimic_process_run_ctx(mimic_process *p, uint64_t budget, mimic_ctx *ctx, mimic_process_regs *out) {
    if (!p) return MIMIC_EINVAL;
    if (!ctx) return mimic_process_run(p, budget, out);
    if (p->h.finished) return mimic_process_step(p, 0, out);
    const uint64_t end = budget ? (uint64_t)p->h.steps + budget : 0xffffffffull;
    uint64_t slice = 4096;
    for (;;) {
        const uint32_t d = ctx_get(ctx);
        if (d) {
            process_regs(p, out);
            return fail(p->vm, d == 1 ? MIMIC_ECANCELED : MIMIC_EDEADLINE,
                        d == 1 ? "context canceled" : "context deadline exceeded");
        }
        const uint64_t to = std::min<uint64_t>(end, (uint64_t)p->h.steps + slice);
        const int rc = process_advance(p, to);
        if (rc) return rc;
        if (p->h.finished || (uint64_t)p->h.steps >= end || (uint64_t)p->h.steps < to) break;
        if (slice < (1ull << 20)) slice <<= 1;
    }
    process_regs(p, out);
    return 0;
}

// n x Process.Run(ctx) of fresh sk_buff processes of one VM, program and ifindex as ONE launch
// (processPool's workers, vm.go:548-573): each process keeps the addresses its Load reserved at
// NewProcess (gathered from its own record, mimic_launch_skb_gather) and runs on vCPU p->cpu in
// array order; a vCPU's processes run in that order.  No step budget (Run(ctx) with ctxs, or
// Background).  Afterwards each process is finished: R0, status, steps in out[i] (and its host
// state); registers R1-R10 and the PC are not kept by a batch lane (out[i].r[1..10] = 0, pc = the
// failing instruction or -1).  Packet memory is the process's own (mimic_process_packet).
int mimic_process_run_many(mimic_process *const *ps, uint32_t n, const int32_t *cpus, mimic_ctx *const *ctxs,
                           mimic_process_regs *out) {
    if (!ps || !n) return n ? MIMIC_EINVAL : 0;
    mimic_vm *vm = ps[0] ? ps[0]->vm : nullptr;
    if (!vm) return MIMIC_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(vm->run_mu);
    const uint32_t prog = ps[0]->prog, ifindex = ps[0]->ifindex;
    uint8_t *lo = nullptr;
    bool any_cust = false;
    // every process is checked before any is changed (a refused call leaves them as they were)
    for (uint32_t i = 0; i < n; i++) {
        mimic_process *p = ps[i];
        if (!p || p->vm != vm) return fail(vm, MIMIC_EINVAL, "process %u: not a process of this VM", i);
        if (cpus && (cpus[i] < 0 || cpus[i] > vm->s.vcpus)) return fail(vm, MIMIC_EINVAL, "process %u: not a valid CPU ID", i);
        if (!p->skb) return fail(vm, MIMIC_ENOTSUP, "process %u: not an sk_buff process", i);
        if (p->prog != prog || p->ifindex != ifindex)
            return fail(vm, MIMIC_EINVAL, "process %u: one program and one interface per launch", i);
        if (p->h.started) return fail(vm, MIMIC_EINVAL, "process %u: already started (Run / Step it instead)", i);
        if (!lo || p->d_pkt < lo) lo = p->d_pkt;
        any_cust |= p->skb_custom;
    }
    if (cpus)   // SetCPUID (vm.go:268-283) of each process first
        for (uint32_t i = 0; i < n; i++) ps[i]->cpu = cpus[i];
    hipSetDevice(vm->s.device);
    hipStream_t st = vm->stream;
    const uint64_t seq = vm->seq.next();   // the launch below touches every process's memory
    for (uint32_t i = 0; i < n; i++) ps[i]->last_seq = seq;
    const uint32_t nb = (n + 255) / 256;
    // one device block: pkt_off | pkt_len | mem pointers | drv | prefix | base | has_cust | custom | results
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_off = 0, o_len = o_off + al((size_t)n * 8), o_mem = o_len + al((size_t)n * 4),
                 o_drv = o_mem + al((size_t)n * 8), o_pre = o_drv + al((size_t)n * 8 * SKB_DERIVED_Q),
                 o_base = o_pre + al(((size_t)n + nb) * 8), o_hc = o_base + 256, o_cu = o_hc + al(n),
                 o_r0 = o_cu + (any_cust ? al((size_t)n * sizeof(mimic_skb_custom)) : 0), o_st = o_r0 + al((size_t)n * 8),
                 o_steps = o_st + al(n), o_epc = o_steps + al((size_t)n * 4), total = o_epc + al((size_t)n * 4);
    if (total > vm->many_cap) {
        HIP_OK(vm, hipStreamSynchronize(st));
        hipFree(vm->d_many);
        vm->d_many = nullptr;
        HIP_OK(vm, hipMalloc(&vm->d_many, total));
        vm->many_cap = total;
    }
    uint8_t *D = vm->d_many;
    std::vector<uint8_t> host(o_drv);   // the host-made part: offsets, lengths, record pointers
    std::vector<int32_t> cpu(n);
    std::vector<uint8_t> hc(n);
    for (uint32_t i = 0; i < n; i++) {
        const mimic_process *p = ps[i];
        const uint64_t off = (uint64_t)(p->d_pkt - lo);
        const uint32_t len = p->len;
        const uint8_t *m = p->d_skbmem;
        memcpy(host.data() + o_off + 8 * (size_t)i, &off, 8);
        memcpy(host.data() + o_len + 4 * (size_t)i, &len, 4);
        memcpy(host.data() + o_mem + 8 * (size_t)i, &m, 8);
        cpu[i] = p->cpu;
        hc[i] = p->skb_custom ? 1 : 0;
    }
    HIP_OK(vm, hipMemcpyAsync(D, host.data(), o_drv, hipMemcpyHostToDevice, st));
    HIP_OK(vm, hipMemsetAsync(D + o_base, 0, 8, st));
    if (any_cust) HIP_OK(vm, hipMemcpyAsync(D + o_hc, hc.data(), n, hipMemcpyHostToDevice, st));
    if (mimic_launch_skb_gather((const uint8_t *const *)(D + o_mem), n, (uint64_t *)(D + o_drv), (uint64_t *)(D + o_pre),
                                any_cust ? (mimic_skb_custom *)(D + o_cu) : nullptr, D + o_hc, st))
        return fail(vm, MIMIC_EDEVICE, "gather: %s", hipGetErrorString(hipGetLastError()));
    mimic_xdp_batch b{};
    b.n = n;
    b.schedule = MIMIC_SCHED_EXPLICIT;
    b.pkt_data = lo;
    b.pkt_off = (const uint64_t *)(D + o_off);
    b.pkt_len = (const uint32_t *)(D + o_len);
    b.cpu = cpu.data();
    b.step_budget = ~0ull >> 1;   // Run(ctx): no budget
    mimic_xdp_results r{};
    r.r0 = (uint64_t *)(D + o_r0);
    r.status = D + o_st;
    r.steps = (uint32_t *)(D + o_steps);
    r.err_pc = (int32_t *)(D + o_epc);
    SkbRun skr{ifindex, any_cust ? (const mimic_skb_custom *)(D + o_cu) : nullptr};
    skr.pre_drv = (const uint64_t *)(D + o_drv);
    skr.pre_prefix = (const uint64_t *)(D + o_pre);
    skr.pre_base = (const uint64_t *)(D + o_base);
    CtxRun cx{nullptr, ctxs};
    int rc = run_xdp_impl(vm, prog, &b, &r, st, 0, &skr, nullptr, ctxs ? &cx : nullptr);
    if (rc) return rc;
    std::vector<uint8_t> res(total - o_r0);
    HIP_OK(vm, hipMemcpyAsync(res.data(), D + o_r0, res.size(), hipMemcpyDeviceToHost, st));
    HIP_OK(vm, proc_sync(vm));
    for (uint32_t i = 0; i < n; i++) {
        mimic_process *p = ps[i];
        uint64_t r0;
        uint32_t steps;
        int32_t epc;
        memcpy(&r0, res.data() + 8 * (size_t)i, 8);
        memcpy(&steps, res.data() + (o_steps - o_r0) + 4 * (size_t)i, 4);
        memcpy(&epc, res.data() + (o_epc - o_r0) + 4 * (size_t)i, 4);
        const uint8_t status = res[(o_st - o_r0) + i];
        memset(p->h.r, 0, sizeof p->h.r);
        p->h.r[0] = r0;
        p->h.pc = status ? epc : -1;
        p->h.prog = prog;
        p->h.steps = steps;
        p->h.status = status;
        p->h.started = 1;
        p->h.finished = 1;
        p->static_next = vm->next_addr;
        p->arena = vm->arena;
        process_regs(p, out ? out + i : nullptr);
    }
    return 0;
}

int mimic_process_packet(mimic_process *p, void *buf, size_t cap) {
    if (!p || !buf) return MIMIC_EINVAL;
    const uint64_t M = (uint64_t)p->H + p->len + p->T;
    if (cap < M) return fail(p->vm, MIMIC_EINVAL, "buffer too small");
    mimic_vm *vm = p->vm;
    std::lock_guard<std::recursive_mutex> lk(vm->run_mu);
    if (!p->uploaded) {   // never launched: the packet memory is the NewProcess image
        memcpy(buf, p->mem.host + PH_IMG + PD_PKT, M);
        return (int)M;
    }
    hipSetDevice(vm->s.device);
    // on the process's stream: behind its NewProcess upload and its launches
    const hipError_t e = hipMemcpyAsync(buf, p->d_pkt, M, hipMemcpyDeviceToHost, vm->stream);
    proc_enq(p);
    const hipError_t es = proc_sync(vm);
    if (e != hipSuccess || es != hipSuccess) return fail(vm, MIMIC_EDEVICE, "packet: %s", hipGetErrorString(e != hipSuccess ? e : es));
    return (int)M;
}

// Process.Cleanup (vm.go:363-374): no host wait -- the blocks go back to the VM's cache with the
// fence of their last use (none when that use is known complete, as after Run / Step)
void mimic_process_free(mimic_process *p) {
    if (!p) return;
    hipSetDevice(p->vm->s.device);
    process_release(p, proc_fence(p->vm, p->last_seq));
    delete p;
}

void mimic_process_free_many(mimic_process *const *ps, uint32_t n) {
    mimic_vm *last = nullptr;
    std::shared_ptr<BlkFence> f;
    bool have = false;   // f is the fence of `last`'s stream for this call
    for (uint32_t i = 0; i < n; i++) {
        mimic_process *p = ps[i];
        if (!p) continue;
        if (p->vm != last) {
            last = p->vm;
            hipSetDevice(last->s.device);
            have = false;
            f.reset();
        }
        const bool busy = !last->seq.idle(p->last_seq);
        if (busy && !have) {   // one event for the call's blocks still in use
            f = proc_fence(last, p->last_seq);
            have = true;
        }
        process_release(p, busy ? f : nullptr);
        delete p;
    }
}

int mimic_sync(mimic_vm *vm, void *hip_stream) {
    if (!vm) return MIMIC_EINVAL;
    hipSetDevice(vm->s.device);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : vm->stream;
    HIP_OK(vm, hipStreamSynchronize(st));
    return spread_check(vm);
}

int mimic_last_steps(mimic_vm *vm, uint64_t *steps_out) {
    if (!vm || !steps_out) return MIMIC_EINVAL;
    hipSetDevice(vm->s.device);
    *steps_out = 0;
    if (!vm->last_lanes) return 0;
    if (vm->last_stream) HIP_OK(vm, hipStreamSynchronize(vm->last_stream));
    std::vector<uint64_t> h(vm->last_lanes);
    HIP_OK(vm, hipMemcpy(h.data(), vm->d_lane_steps, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t = 0;
    for (uint64_t v : h) t += v;
    *steps_out = t;
    return spread_check(vm);
}

int mimic_exec_mode(const mimic_vm *vm) { return vm ? vm->exec_mode : MIMIC_EINVAL; }
int mimic_set_spread(mimic_vm *vm, int32_t mode) {
    if (!vm || mode < -1 || mode > 1) return MIMIC_EINVAL;
    vm->spread_mode = mode;
    return 0;
}
int mimic_last_exec(const mimic_vm *vm) { return vm ? vm->last_exec : MIMIC_EINVAL; }

// The JIT kernel source for a set of raw programs (slots as mimic_program_load takes them; map
// relocations do not change the code shape).  Returns the source length; copies it if it fits.
// Host only: no device needed.
long mimic_jit_source_for(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, char *buf, size_t cap) {
    return mimic_jit_source_for_ctx(progs, n_slots, n_progs, MIMIC_CTX_XDP, buf, cap);
}

long mimic_jit_source_for_ctx(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind,
                              char *buf, size_t cap) {
    return mimic_jit_source_vc(progs, n_slots, n_progs, ctx_kind, nullptr, 0, buf, cap);
}

long mimic_jit_source_vc(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind,
                         const uint32_t *vc_slots, uint32_t n_vc, char *buf, size_t cap) {
    // (ctx_kind | 0x100: the single-process form of an xdp_md set, what Process.Run tiers up to)
    const bool proc = (ctx_kind & 0x100) != 0;
    ctx_kind &= 0xff;
    if (ctx_kind != MIMIC_CTX_XDP && ctx_kind != MIMIC_CTX_SKB) return MIMIC_EINVAL;
    if (proc && ctx_kind != MIMIC_CTX_XDP) return MIMIC_EINVAL;
    std::vector<HostProg> hp(n_progs);
    for (uint32_t p = 0; p < n_progs; p++) {
        std::string err;
        if (decode_program((const uint8_t *)progs[p], n_slots[p], hp[p].ins, &err)) return MIMIC_EINVAL;
    }
    std::vector<DInsn> all;
    std::vector<DProg> dp;
    build_host_tables(hp, all, dp);
    std::vector<std::pair<uint32_t, uint32_t>> vc;
    for (uint32_t q = 0; q < n_vc; q++) {
        const uint32_t p = vc_slots[3 * q], s = vc_slots[3 * q + 1], rb = vc_slots[3 * q + 2];
        if (p >= dp.size() || s >= dp[p].n) return MIMIC_EINVAL;
        vc.push_back({dp[p].base + s, rb});
    }
    const std::string src = mimic_jit_source(dp, all, (uint32_t)ctx_kind, nullptr, &vc, false, nullptr, false, proc);
    if (buf && cap > src.size()) memcpy(buf, src.c_str(), src.size() + 1);
    return (long)src.size();
}

// The spread kernel's source for raw programs (host only): pc = (program, slot, map id) triples of
// the LD_IMM64 slots naming a per-CPU array's object, shapes = (map id, E * S, S) triples, lds_rows
// as spread_build() picks it.  *spread_out = 1 when the programs allow a spread kernel (else the
// returned source is the plain one).
long mimic_jit_source_spread(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, const uint32_t *pc,
                             uint32_t n_pc, const uint32_t *shapes, uint32_t n_shapes, uint32_t lds_rows,
                             int32_t *spread_out, char *buf, size_t cap) {
    std::vector<HostProg> hp(n_progs);
    for (uint32_t p = 0; p < n_progs; p++) {
        std::string err;
        if (decode_program((const uint8_t *)progs[p], n_slots[p], hp[p].ins, &err)) return MIMIC_EINVAL;
    }
    std::vector<DInsn> all;
    std::vector<DProg> dp;
    build_host_tables(hp, all, dp);
    SpreadReq req;
    for (uint32_t q = 0; q < n_pc; q++) {
        const uint32_t p = pc[3 * q], sl = pc[3 * q + 1];
        if (p >= dp.size() || sl >= dp[p].n) return MIMIC_EINVAL;
        req.slot_map[dp[p].base + sl] = pc[3 * q + 2];
    }
    for (uint32_t q = 0; q < n_shapes; q++) req.shape[shapes[3 * q]] = {shapes[3 * q + 1], shapes[3 * q + 2]};
    req.lds_rows = lds_rows & 0x7fffffffu;
    req.own = (lds_rows >> 31) != 0;   // bit 31: the owned form (spread_build_own)
    JitInfo info{};
    const std::string src = mimic_jit_source(dp, all, MIMIC_CTX_XDP, &info, nullptr, false, &req);
    if (spread_out) *spread_out = info.spread ? 1 : 0;
    if (buf && cap > src.size()) memcpy(buf, src.c_str(), src.size() + 1);
    return (long)src.size();
}

// Build the JIT kernel for raw programs into the MIMIC_JIT_CACHE directory (host only): a
// later process that loads the same programs finds the code object there.
int mimic_jit_prebuild(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs) {
    return mimic_jit_prebuild_ctx(progs, n_slots, n_progs, MIMIC_CTX_XDP);
}

int mimic_jit_prebuild_ctx(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind) {
    if (ctx_kind != MIMIC_CTX_XDP && ctx_kind != MIMIC_CTX_SKB) return MIMIC_EINVAL;
    std::vector<HostProg> hp(n_progs);
    for (uint32_t p = 0; p < n_progs; p++) {
        std::string err;
        if (decode_program((const uint8_t *)progs[p], n_slots[p], hp[p].ins, &err)) return MIMIC_EINVAL;
    }
    std::vector<DInsn> all;
    std::vector<DProg> dp;
    build_host_tables(hp, all, dp);
    std::string log;
    return mimic_jit_prebuild_source(mimic_jit_source(dp, all, (uint32_t)ctx_kind, nullptr), &log) ? MIMIC_EINVAL : 0;
}

// hipRTC-compile a JIT source for gfx950 without loading it (host only).  0 = ok; the compiler
// log is copied to log (if given).
int mimic_jit_check(const char *src, char *log, size_t cap, size_t *code_size) {
    std::string lg;
    const int rc = mimic_jit_check_source(src ? src : "", &lg, code_size);
    if (log && cap) {
        const size_t n = std::min(cap - 1, lg.size());
        memcpy(log, lg.data(), n);
        log[n] = 0;
    }
    return rc ? MIMIC_EINVAL : 0;
}

int mimic_jit_cache_source(const char *src) {
    if (!src) return MIMIC_EINVAL;
    std::string log;
    return mimic_jit_prebuild_source(src, &log) ? MIMIC_EINVAL : 0;
}

int mimic_jit_code(const char *src, void *code, size_t cap, size_t *code_size) {
    if (!src || !code_size) return MIMIC_EINVAL;
    std::vector<char> co;
    std::string log;
    if (mimic_jit_build_code(src, co, &log)) return MIMIC_EINVAL;
    *code_size = co.size();
    if (code && cap >= co.size()) memcpy(code, co.data(), co.size());
    return 0;
}

int mimic_host_register(void *p, size_t bytes) {
    if (!p || !bytes) return MIMIC_EINVAL;
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? 0 : MIMIC_EDEVICE;
}

int mimic_host_unregister(void *p) {
    if (!p) return MIMIC_EINVAL;
    return hipHostUnregister(p) == hipSuccess ? 0 : MIMIC_EDEVICE;
}

// Sub-batch c: its host byte window [lo, hi) (packets need not be in order) and whether its
// packets are ascending and non-overlapping (pkt_out copies the window back as one block).
struct HostWindow {
    uint64_t lo = ~0ull, hi = 0;
    bool ascending = true;
};
// branch-free loops the compiler vectorises (AVX2 is on every host this runs on: Zen 4/5 EPYC)
__attribute__((target("avx2"))) static HostWindow host_window(const mimic_xdp_host_batch *hb, uint32_t a, uint32_t m,
                                                             uint64_t room) {
    const uint64_t *off = hb->pkt_off + a;
    const uint32_t *len = hb->pkt_len + a;
    uint64_t lo = ~0ull, hi = 0, bad = 0;
    for (uint32_t i = 0; i < m; i++) {
        const uint64_t o = off[i], e = o + len[i] + room;
        lo = o < lo ? o : lo;
        hi = e > hi ? e : hi;
    }
    for (uint32_t i = 1; i < m; i++) bad |= (uint64_t)(off[i] < off[i - 1] + len[i - 1] + room);
    HostWindow w;
    w.lo = lo;
    w.hi = hi;
    w.ascending = bad == 0;
    return w;
}

static int slot_reserve(mimic_vm *vm, mimic_vm::Slot &sl, size_t bytes, size_t n) {
    if (bytes <= sl.cap_bytes && n <= sl.cap_n) return 0;
    if (sl.used) HIP_OK(vm, hipEventSynchronize(sl.e_out));   // its last sub-batch is done
    if (bytes > sl.cap_bytes) {
        hipFree(sl.buf);
        sl.buf = nullptr;
        sl.cap_bytes = std::max(bytes, sl.cap_bytes + sl.cap_bytes / 2);
        HIP_OK(vm, hipMalloc(&sl.buf, sl.cap_bytes));
    }
    if (n > sl.cap_n) {
        for (void *q : {(void *)sl.off, (void *)sl.len, (void *)sl.r0, (void *)sl.st}) hipFree(q);
        sl.off = nullptr;
        sl.len = nullptr;
        sl.r0 = nullptr;
        sl.st = nullptr;
        sl.cap_n = std::max(n, sl.cap_n + sl.cap_n / 2);
        HIP_OK(vm, hipMalloc(&sl.off, 8 * sl.cap_n));
        HIP_OK(vm, hipMalloc(&sl.len, 4 * sl.cap_n));
        HIP_OK(vm, hipMalloc(&sl.r0, 8 * sl.cap_n));
        HIP_OK(vm, hipMalloc(&sl.st, sl.cap_n));
    }
    return 0;
}

// Sub-batch pipeline over NB staging slots.  Per sub-batch, on the H2D stream: its descriptors,
// its packet window and its launch parameters; the kernel on the VM stream after them; its r0 /
// status (and packet bytes) on the D2H stream after the kernel.  The host-side scan of sub-batch
// c + 1 runs while sub-batch c's copies are in flight, so no O(n) pass precedes the first copy.
static int run_xdp_host_impl(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                             mimic_ctx *ctx, mimic_ctx *const *ctx_per_packet);
int mimic_run_xdp_host(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks) {
    return run_xdp_host_impl(vm, prog_id, hb, chunks, nullptr, nullptr);
}
int mimic_run_xdp_host_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                           mimic_ctx *ctx) {
    return run_xdp_host_impl(vm, prog_id, hb, chunks, ctx, nullptr);
}
int mimic_run_xdp_host_ctx_pp(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                              mimic_ctx *const *ctx_per_packet) {
    return run_xdp_host_impl(vm, prog_id, hb, chunks, nullptr, ctx_per_packet);
}
static int run_xdp_host_impl(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                             mimic_ctx *ctx, mimic_ctx *const *ctx_pp) {
    if (!vm || !hb) return MIMIC_EINVAL;
    const uint32_t n = hb->n;
    if (n == 0) return 0;
    if (!hb->pkt_data || !hb->pkt_off || !hb->pkt_len || !hb->r0 || !hb->status)
        return fail(vm, MIMIC_EINVAL, "missing host arrays");
    hipSetDevice(vm->s.device);
    const uint64_t room = (uint64_t)hb->headroom_all + hb->tailroom_all;
    if (chunks == 0) {  // auto: ~16 MiB of packet memory per sub-batch, estimated from the batch's ends
        // (measured, 1 M x 64 B: 4 sub-batches 1.76 ms, 8: 2.0 ms, 16: 2.6-9 ms -- per-copy
        // overheads of ~10 us per dependent copy, and stalls in the runtime with many small copies)
        const uint64_t first = hb->pkt_off[0], last = hb->pkt_off[n - 1] + hb->pkt_len[n - 1] + room;
        const uint64_t bytes = last > first ? last - first : (uint64_t)n * (room + 1500);
        chunks = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(2, bytes >> 24));
    }
    chunks = std::max<uint32_t>(1, std::min(chunks, n));
    // pkt_out: each sub-batch copies its whole byte window back, so the packets of the whole batch
    // (not only of one sub-batch) must be ascending and non-overlapping -- checked before any copy
    // or launch, so a refused batch changes nothing (maps, results, pkt_out)
    if (hb->pkt_out && !host_window(hb, 0, n, room).ascending)
        return fail(vm, MIMIC_EINVAL, "pkt_out needs ascending, non-overlapping packets");
    // CHUNKED over the whole batch = EXPLICIT with cpu(i) = vcpu_begin + i / ceil(n / lanes)
    std::vector<int32_t> cpu_chunked;
    uint32_t sched = hb->schedule;
    const int32_t *cpu = hb->cpu;
    if (sched == MIMIC_SCHED_CHUNKED) {
        const uint32_t lanes = (uint32_t)vm->s.vcpu_count;
        const uint64_t per = ((uint64_t)n + lanes - 1) / lanes;
        cpu_chunked.resize(n);
        for (uint32_t i = 0; i < n; i++) cpu_chunked[i] = vm->s.vcpu_begin + (int32_t)(i / per);
        cpu = cpu_chunked.data();
        sched = MIMIC_SCHED_EXPLICIT;
    }
    if (sched == MIMIC_SCHED_EXPLICIT && !cpu) return fail(vm, MIMIC_EINVAL, "explicit schedule needs cpu[]");
    // one context per packet: the whole batch's context words go to the device once, before the
    // pipeline (each sub-batch's kernels read their slice; the array is 8 bytes per packet)
    bool pp_any = false;
    if (ctx_pp) {
        std::vector<const uint32_t *> w(n);
        for (uint32_t i = 0; i < n; i++) {
            w[i] = ctx_pp[i] ? ctx_pp[i]->dword : nullptr;
            pp_any |= w[i] != nullptr;
        }
        if (pp_any) {
            if (vm->cancel_pp_stream) HIP_OK(vm, hipStreamSynchronize(vm->cancel_pp_stream));   // earlier readers
            HIP_OK(vm, hipStreamSynchronize(vm->stream));
            vm->cancel_pp_stream = vm->stream;
            if (n > vm->cancel_pp_cap) {
                hipFree(vm->d_cancel_pp);
                vm->d_cancel_pp = nullptr;
                HIP_OK(vm, hipMalloc(&vm->d_cancel_pp, (size_t)n * sizeof(void *)));
                vm->cancel_pp_cap = n;
            }
            HIP_OK(vm, hipMemcpy(vm->d_cancel_pp, w.data(), (size_t)n * sizeof(void *), hipMemcpyHostToDevice));
        }
    }
    if (!vm->s_h2d) {
        HIP_OK(vm, hipStreamCreateWithFlags(&vm->s_h2d, hipStreamNonBlocking));
        HIP_OK(vm, hipStreamCreateWithFlags(&vm->s_h2d2, hipStreamNonBlocking));
        HIP_OK(vm, hipStreamCreateWithFlags(&vm->s_d2h, hipStreamNonBlocking));
        HIP_OK(vm, hipEventCreateWithFlags(&vm->kp_copy_ev, hipEventDisableTiming));
        for (auto &sl : vm->slot)
            for (hipEvent_t *e : {&sl.e_in, &sl.e_k, &sl.e_out}) HIP_OK(vm, hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    // MIMIC_HOST_TRACE=1: host-side time split of the call on stderr (scan / copy issue / launch / wait)
    static const bool trace = getenv("MIMIC_HOST_TRACE") && getenv("MIMIC_HOST_TRACE")[0] == '1';
    using clk = std::chrono::steady_clock;
    double t_scan = 0, t_copy = 0, t_run = 0;
    auto t_all = clk::now();
    struct CopyStreamScope {   // launch parameters go on the H2D stream for this call only
        mimic_vm *vm;
        ~CopyStreamScope() { vm->kp_copy_stream = nullptr; }
    } scope{vm};
    for (uint32_t c = 0; c < chunks; c++) {
        auto &sl = vm->slot[c % mimic_vm::NB];
        // two H2D streams: one stream's gaps between dependent copies are filled by the other's
        hipStream_t h2d = (c & 1) ? vm->s_h2d2 : vm->s_h2d;
        const uint32_t a = (uint32_t)((uint64_t)n * c / chunks), m = (uint32_t)((uint64_t)n * (c + 1) / chunks) - a;
        if (m == 0) continue;
        auto t0 = clk::now();
        const HostWindow w = host_window(hb, a, m, room);
        auto t1 = clk::now();
        t_scan += std::chrono::duration<double, std::micro>(t1 - t0).count();
        int rc = slot_reserve(vm, sl, std::max<uint64_t>(w.hi - w.lo, 1), m);
        if (rc) return rc;
        if (sl.used) HIP_OK(vm, hipStreamWaitEvent(h2d, sl.e_out, 0));  // the slot's last D2H is done
        HIP_OK(vm, hipMemcpyAsync(sl.off, hb->pkt_off + a, 8ull * m, hipMemcpyHostToDevice, h2d));
        HIP_OK(vm, hipMemcpyAsync(sl.len, hb->pkt_len + a, 4ull * m, hipMemcpyHostToDevice, h2d));
        HIP_OK(vm, hipMemcpyAsync(sl.buf, hb->pkt_data + w.lo, w.hi - w.lo, hipMemcpyHostToDevice, h2d));
        HIP_OK(vm, hipEventRecord(sl.e_in, h2d));
        HIP_OK(vm, hipStreamWaitEvent(vm->stream, sl.e_in, 0));
        auto t2 = clk::now();
        t_copy += std::chrono::duration<double, std::micro>(t2 - t1).count();
        mimic_xdp_batch b{};
        b.n = m;
        b.schedule = sched;
        b.pkt_data = sl.buf - w.lo;  // offsets stay those of the host batch
        b.pkt_off = sl.off;
        b.pkt_len = sl.len;
        b.headroom_all = hb->headroom_all;
        b.tailroom_all = hb->tailroom_all;
        b.ingress_all = hb->ingress_all;
        b.rxq_all = hb->rxq_all;
        b.egress_all = hb->egress_all;
        b.cpu = sched == MIMIC_SCHED_EXPLICIT ? cpu + a : nullptr;
        b.step_budget = hb->step_budget;
        mimic_xdp_results r{};
        r.r0 = sl.r0;
        r.status = sl.st;
        vm->kp_copy_stream = h2d;
        // every sub-batch's kernel reads the run's context, or its packets' slice of the per-packet words
        const CtxRun cx{ctx, pp_any ? ctx_pp + a : nullptr, pp_any ? vm->d_cancel_pp + a : nullptr};
        rc = run_xdp_impl(vm, prog_id, &b, &r, vm->stream, a, nullptr, nullptr, ctx || pp_any ? &cx : nullptr);
        vm->kp_copy_stream = nullptr;
        if (rc) return rc;
        t_run += std::chrono::duration<double, std::micro>(clk::now() - t2).count();
        HIP_OK(vm, hipEventRecord(sl.e_k, vm->stream));
        HIP_OK(vm, hipStreamWaitEvent(vm->s_d2h, sl.e_k, 0));
        HIP_OK(vm, hipMemcpyAsync(hb->r0 + a, sl.r0, 8ull * m, hipMemcpyDeviceToHost, vm->s_d2h));
        HIP_OK(vm, hipMemcpyAsync(hb->status + a, sl.st, m, hipMemcpyDeviceToHost, vm->s_d2h));
        if (hb->pkt_out) HIP_OK(vm, hipMemcpyAsync(hb->pkt_out + w.lo, sl.buf, w.hi - w.lo, hipMemcpyDeviceToHost, vm->s_d2h));
        HIP_OK(vm, hipEventRecord(sl.e_out, vm->s_d2h));
        sl.used = true;
    }
    auto t3 = clk::now();
    HIP_OK(vm, hipStreamSynchronize(vm->s_d2h));
    if (trace)
        fprintf(stderr, "mimic_run_xdp_host: n %u chunks %u | scan %.0f us, copy issue %.0f us, launch %.0f us, issue loop %.0f us, wait %.0f us, total %.0f us\n",
                n, chunks, t_scan, t_copy, t_run, std::chrono::duration<double, std::micro>(t3 - t_all).count(),
                std::chrono::duration<double, std::micro>(clk::now() - t3).count(),
                std::chrono::duration<double, std::micro>(clk::now() - t_all).count());
    vm->last_stream = nullptr;
    return 0;
}

}  // extern "C"
