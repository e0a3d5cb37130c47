// layout.h -- data layout shared by the host engine (engine.cpp) and the gfx950 batch
// interpreter (interp.hip).  Plain structs only; no torch, no STL.
//
// The virtual 32-bit address space reproduces the reference's MemoryController layout
// (memory_controller.go:58-112: first fit from 0x10000, one unused byte between entries).
// Static entries (maps, programs) are created once on the host; every process of a batch
// then gets the SAME three per-process entries appended after them (stack, packet,
// xdp_md -- vm.go:218, context_xdp_md.go:66,107), because Cleanup removes them again
// (vm.go:363-374).  So each lane can compute its addresses in O(1):
//   St = static_next            stack  [St, St+S]            (S = frame_size*frame_count)
//   P  = St + S + 1             packet [P, P+M]              (M = headroom+len+tailroom)
//   X  = P + M + 1              xdp_md [X, X+24]
// Static entries are summarised as a short sorted segment table (one segment per
// entry, except the V per-CPU sub-arrays of a per-CPU array map, which are one strided
// group segment, emulator_linux_map_array.go:185-215).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__) || defined(__HIP__) || defined(__HIPCC_RTC__)
#define HHD_LAYOUT static __host__ __device__ inline
#else
#define HHD_LAYOUT static inline
#endif

#define MIMIC_MAX_FRAMES 32u          // engine bound on BPF-to-BPF call depth (oracle: ORC_MAX_FRAMES)
#define MIMIC_DEFAULT_BUDGET (1ull << 22)
#define MIMIC_MEM_START 0x10000u      // memStart + 1, memory_controller.go:55,70
#define MIMIC_PC_BITS 24u             // max program length = 2^24 slots
#define MIMIC_XDP_MD_SIZE 24u         // context_xdp_md.go:57
#define MIMIC_FRAME_QWORDS 5u         // saved PC + R6..R9 (inst.go:277-296)

enum SegKind : uint32_t {
    SEG_PLAIN = 1,            // PlainMemory backing in the arena
    SEG_ARRAY_OBJ = 2,        // LinuxArrayMap object (8 B): LinuxMap; VMMem only if datasec
    SEG_MAP_OBJ = 3,          // per-CPU array / hash / per-CPU hash object: LinuxMap, not VMMem
    SEG_PROG = 4,             // *ebpf.ProgramSpec: neither
    SEG_PERCPU_ARRAY = 5,     // V x [sub-array object (8 B) | gap | backing (E*S) | gap]
    SEG_PERCPU_VALUES = 6,    // V x [values backing (E*S) | gap]   (per-CPU hash values)
};

enum MapFamily : uint32_t { FAM_ARRAY = 1, FAM_PERCPU_ARRAY = 2, FAM_HASH = 3, FAM_PERCPU_HASH = 4 };

struct Seg {
    uint32_t lo, hi;        // [lo, hi] inclusive address range covered
    uint32_t kind;          // SegKind
    uint32_t id;            // map index (objects, groups, plain backings of maps) or prog index
    uint64_t dev_off;       // arena offset: PLAIN backing / group cpu-0 backing
    uint32_t size;          // PLAIN: backing size; groups: per-cpu backing size (E*S)
    uint32_t period;        // groups: address distance between consecutive cpus
    uint32_t count;         // groups: number of cpus
    uint32_t datasec;       // ARRAY_OBJ / SEG_PERCPU_ARRAY sub-objects: Spec.Value is *btf.Datasec
    uint64_t dev_stride;    // groups: arena distance between consecutive cpu backings
};

struct DMap {
    uint32_t family, type, key_size, value_size, max_entries, datasec;
    uint32_t obj_addr;       // map object address
    uint32_t backing_addr;   // ARRAY: values backing; PERCPU_ARRAY: cpu-0 backing; HASH: values; PERCPU_HASH: cpu-0 values
    uint32_t addr_period;    // per-CPU: address distance between cpu backings
    uint32_t ncpu;           // per-CPU: number of cpus (len(arrayMaps) / len(values))
    uint64_t dev_off;        // arena offset of cpu-0 backing
    uint64_t dev_stride;     // arena distance between cpu backings
    // hash maps: device open-addressing index over the reference's key/value slots
    // (hashmap.h).  The slot a key gets comes from the reference's FIFO freelist.
    uint64_t keys_dev_off;   // arena offset of the VM-visible keys backing (E*K)
    uint32_t keys_addr;
    uint32_t ht_cap;         // buckets, power of two
    uint64_t ht_dev_off;     // hash index region (hashmap.h): records | rebuild copy | locks | freelist | HashCtl
    uint32_t rec_q;          // record size in qwords
    uint32_t nlocks;         // power of two
    uint32_t fl_cap;         // power of two >= 2(E+1)
    uint32_t hflags;         // HT_F_*: set per launch table upload (engine.cpp tables_upload)
};
// the VM's one hash map whose pop-only JIT launches reserve freelist positions in per-block chunks
// (hashmap.h h_chunk_fill; engine.cpp picks it: a FAM_HASH map not shared with another VM,
// E <= HT_CHUNK_MAXE); each such launch is followed by mimic_hash_compact_kernel
#define HT_F_CHUNK 1u
#define HT_CHUNK_MAXE (1u << 17)   // (the compaction kernel keeps the bit words and their prefix counts in LDS)
#define HT_LEFT_CAP 16384u   // blocks of one launch that can hand a chunk remainder back (h_chunk_fini)

// freelist ring + table counters of one hash map (device, agent-scope atomics).  head is on a
// 128-byte line of its own (every inserting wave of the GPU adds to it), and inserts count the
// buckets they fill in HT_USED_SHARDS counters on lines of their own (used = used0 + the shards).
#define HT_USED_SHARDS 16
struct HashCtl {
    unsigned long long head;   // next ring position to pop
    uint32_t comb_fault;       // a block combiner gave up waiting (hashmap.h h_comb_reserve): the launch failed
    uint32_t pad0[29];
    unsigned long long tail;   // next ring position to push
    int32_t avail;             // free slots not yet claimed (stale after a pop-only launch: normalised)
    uint32_t used0;            // buckets that are not EMPTY (live + tombstones + busy), minus the shards
    uint32_t pad1[28];
    uint32_t used_sh[HT_USED_SHARDS * 32];   // shard s at [32 s]
    // chunked reservations (hashmap.h h_chunk_fill, interp.hip mimic_hash_compact_kernel); all zero
    // outside a chunk launch and its compaction
    uint32_t cminv;            // 0xffffffff - the lowest position a chunk refill took this launch (0: none)
    uint32_t full;             // a chunk launch proved every position live (E2BIG from then on)
    uint32_t cdone;            // compaction blocks done
    uint32_t nleft;            // 1 + the highest block index that handed a remainder back (left[])
    uint32_t pad2[28];
    uint32_t live_sh[HT_USED_SHARDS * 32];   // positions chunk launches gave to inserts, shard s at [32 s]
};
// after HashCtl (hashmap.h h_used8 / h_s2b / h_left): a byte per slot (inserted by the chunk launch),
// the bucket of each such slot, the blocks' handed-back chunk remainders (end << 32 | next)
HHD_LAYOUT uint64_t ht_ext_bytes(uint32_t E) {
    const uint64_t e32 = ((uint64_t)E + 1023) & ~1023ull;   // slots rounded to whole 128-byte lines of bits
    return e32 + e32 * 4 + (uint64_t)HT_LEFT_CAP * 8;
}
#define HT_EMPTY 0xffffffffu
#define HT_TOMB 0xfffffffeu
#define HT_BUSY 0xfffffffdu

struct DProg {
    uint32_t base;   // first instruction in the concatenated instruction array
    uint32_t n;      // len(Program.Instructions)
    uint32_t addr;   // program object address
    uint32_t pad;
};

// A decoded instruction slot: w = op | dst<<8 | src<<12 | (uint16)off<<16, k = asm.Instruction.Constant,
// aux = handler id and facts the host predecodes at load time.  All lanes executing a slot
// share its PC, so "is PC+1 / the jump target inside the program" and every error that
// depends only on the instruction (bad register numbers, unsupported opcodes, helper ids,
// constant divisors ...) are properties of the slot.
enum Handler : uint32_t {
    H_SLOW = 0,        // full generic decode (rare forms: END, per-lane-ordered errors ...)
    H_ERR = 1,         // instruction-determined fatal status in AUX_ARG
    H_NOP = 2,
    H_ALU64 = 3,       // ADD SUB MUL DIV/MOD(K, k!=0) OR AND LSH RSH XOR MOV NEG ARSH, dst<=9
    H_ALU32 = 4,
    H_LDIMM = 5,
    H_JA = 6,
    H_JCC = 7,         // conditional jump; AUX_ARG = jump op, AUX_W32 / AUX_X flags
    H_LDX = 8,         // dst<=9, src<=10; AUX_SZ = size
    H_ST = 9,
    H_STX = 10,
    H_EXIT = 11,
    H_CALL = 12,       // helper 1/2/3/8/12/65
    H_CALL_LOCAL = 13, // BPF-to-BPF
    H_LDABS = 14,      // LD_ABS / LD_IND (AUX_X = IND); R6 must be the sk_buff (emulator_linux_.go:198-288)
};
#define AUX_H(a) ((a) & 0xffu)
#define AUX_FALL_OK (1u << 8)    // PC+1 < len(Instructions)
#define AUX_JT_OK (1u << 9)      // jump / BPF-to-BPF call target (after Step's PC++) in [0, len)
#define AUX_JT_NEG (1u << 10)    // target < 0: the next Step panics
#define AUX_W32 (1u << 11)       // 32-bit compare
#define AUX_X (1u << 12)         // register source
#define AUX_ARG(a) (((a) >> 16) & 0xffu)
#define AUX_SZ(a) ((a) >> 24)
// H_LDIMM only: 1 + the id of the array / per-CPU array map whose object address the constant
// is (set at upload, engine.cpp); the JIT's inline lookup reads it at run time, so the kernel
// source does not depend on it
#define AUX_MAPHINT(a) ((a) >> 16)
struct DInsn {
    uint32_t w;
    uint32_t aux;
    uint64_t k;
};

enum Sched : uint32_t { SCHED_CHUNKED = 0, SCHED_INTERLEAVED = 1, SCHED_EXPLICIT = 2 };

// context of a batch: LinuxContextXDP (context_xdp_md.go) or LinuxContextSKBuff (context_sk_buff.go)
enum CtxKind : uint32_t { CTX_XDP = 0, CTX_SKB = 1 };
struct SkbRec;

// mimic_run_xdp_many: the k-th batch of a multi-batch launch (its packets and results; every
// batch of the launch has the same n, schedule and scalar context fields)
#define MIMIC_MANY_MAX 8u
struct BatchRef {
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    uint64_t *r0;
    uint8_t *status;
    uint32_t *steps;
    int32_t *err_pc;
    uint64_t pad;
};

struct KParams {
    // program / static memory
    const DInsn *insns;
    const DProg *progs;
    const Seg *segs;
    const DMap *maps;
    uint8_t *arena;
    uint32_t nprogs, nsegs, nmaps, entry_prog;
    uint32_t static_next;       // St
    uint32_t stack_size;        // S
    uint32_t frame_size;
    uint32_t chunk_shift;       // lazy-zero granule of the stack above 512 B (bytes = 1 << shift)
    uint32_t max_tail_calls;
    uint32_t total_vcpus;       // V (VMSettings.VirtualCPUs)
    uint32_t vcpu_begin;        // first vCPU executed by this launch
    uint32_t lanes;             // vCPUs executed by this launch (= lanes used)
    uint32_t priv_lanes;        // interleave stride of private memory (>= lanes)
    uint8_t *priv;              // per-lane private memory, qword-interleaved
    uint32_t priv_xdp_q;        // qword index of the xdp_md overlay
    uint32_t priv_frame_q;      // qword index of the saved-frame area
    uint32_t priv_key_q;        // qword index of the hash-key scratch (ceil(K/8) words, max over hash maps)
    uint32_t cpu_lanes;         // lanes [0, cpu_lanes) are vCPUs vcpu_begin + g; lane cpu_lanes runs the
                                // processes whose CPU ID was never set (-1), lane cpu_lanes + 1 those
                                // with ID == V (SetCPUID accepts it, vm.go:214, 268-283)
    uint64_t budget;
    // batch
    uint32_t n;
    uint32_t sched;
    uint32_t per_lane;          // CHUNKED: chunk; INTERLEAVED/EXPLICIT: max packets per lane
    uint32_t sched_shift;       // INTERLEAVED: index of packet 0 in the whole batch, mod lanes (sub-batches)
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    const uint32_t *headroom_arr;
    const uint32_t *tailroom_arr;
    const int32_t *ingress_arr;
    const int32_t *rxq_arr;
    const int32_t *egress_arr;
    uint32_t headroom, tailroom;
    int32_t ingress, rxq, egress;
    uint32_t step_gen;          // single-process stepping: the generation the process's StepState must carry
    const uint32_t *sched_start;   // EXPLICIT: CSR over local lanes [lanes+1]
    const uint32_t *sched_pkts;
    // results
    uint64_t *r0;
    uint8_t *status;
    uint32_t *steps;
    int32_t *err_pc;
    uint64_t *lane_steps;          // optional: per-lane executed steps (insns/s accounting)
    // sk_buff batches (skb.h): per-packet records, exclusive prefix of the leak footprints,
    // and the device word holding the first leak address of this batch
    uint32_t ctx_kind;             // CtxKind
    uint32_t skb_ifindex;          // NetDev.IFIndex
    SkbRec *skb_rec;
    const uint64_t *skb_prefix;
    const uint64_t *skb_base;
    // single-process stepping (Process.Step, vm.go:291-340): one lane, one packet, interpreter
    // only.  The process state is restored from / saved to *step around the launch, and the
    // step budget suspends the process instead of ending it.
    struct StepState *step;
    // no program of this launch deletes from a hash map: freelist pops need no `avail`
    // semaphore (no push can run concurrently) -- one head reservation per wave round
    uint32_t hash_pop_only;
    // no program of this launch writes a hash map (no update / delete helper): the tables are
    // read-only while it runs, so lookups read a bucket record with plain (cached) loads at once
    uint32_t hash_ro;
    // JIT kernels built with deferred slow paths (jit.cpp, defer mode): a lane whose process
    // reaches a slow path saves it in defer[lane] (flag = defer_epoch), sets *defer_any =
    // defer_epoch and stops; the interpreter's resume kernel then finishes that process and the
    // lane's remaining packets.  The epoch changes every launch, so nothing is ever cleared.
    struct DeferRec *defer;
    uint32_t *defer_any;
    uint32_t defer_epoch;
    // sk_buff batches: 1 when the prep kernel wrote every packet's SkbRec; 0 when the JIT kernel
    // builds them itself (skb_load_walk) -- then the interpreter builds the ones it needs; 2 when
    // the prep wrote the derived words of the frames skb_fast rejects only (skb_prefix flag
    // SKB_PFX_EXC, skb.h) and the JIT kernel derives the rest (skb_load_fast)
    uint32_t skb_rec_built;
    // spread launches (jit.cpp analyze_spread): a vCPU's packets run on many lanes; a generic
    // access that reaches per-CPU map memory would break that mode's exactness and sets *spread_bad
    // (never cleared: the host reports it as an engine error).  nullptr in every other launch.
    uint32_t *spread_bad;
    // sk_buff batches: the user-given sock / flow keys (mimic_skb_custom [n], packet-indexed), or null
    const void *skb_custom;
    // sk_buff batches: the prep kernel's derived record words, SKB_DERIVED_Q per packet with no gaps
    // (skb.hip), or null (a stepped process's own record holds them)
    const uint64_t *skb_drv;
    // spread launches with an LDS table covering every vCPU lane: each block's table goes here,
    // [block][lane][counter], summed into the map by mimic_spread_reduce_kernel (interp.hip)
    void *spread_part;
    // Run(ctx) (vm.go:343-350): the contexts of the launch's processes, mimic_ctx words in pinned
    // host memory (0 = not done, 1 = canceled, 2 = deadline exceeded).  cancel: one word for every
    // packet; cancel_pp: one word pointer per packet (null: context.Background()).  cancel_any = 0:
    // neither (no check at all).  Checked before each process's first step (ctx_done, runtime.h).
    const uint32_t *cancel;
    const uint32_t *const *cancel_pp;
    uint32_t cancel_any;
    // owned spread launches (jit.cpp spread_own): packets per thread, a divisor of per_lane
    uint32_t own_q;
    // multi-batch owned launches (mimic_run_xdp_many): many_n batches, run one after another by
    // every thread (0: the one batch above)
    uint32_t many_n;
    struct BatchRef many[MIMIC_MANY_MAX];
    // single-process stepping: the process's first launch copies its NewProcess image (pinned,
    // device-mapped host memory) into its device block itself (no copy ahead of the launch), and
    // the stepping kernel stages the first step_ins_n instruction slots in LDS (dynamic LDS)
    const uint8_t *step_img;
    uint8_t *step_dst;
    uint32_t step_img_n;
    uint32_t step_ins_n;
    // sk_buff batches: the batch's rooms-clean word (mimic_skb_batch.rooms_state) or null; a program
    // store into a head- or tailroom sets it to 0
    uint32_t *skb_rooms_state;
};

// A process a JIT lane suspended at a slow path (defer mode): the registers the slot and its
// successors can read, the slot (PC) and program, the steps before the slot, the process's
// dynamic lane state (stack validity, xdp_md overlay flag, frames, tail calls), and where the
// lane is in its schedule.  Everything else of the lane (packet entry, sk_buff record, ...)
// follows from the packet and is derived again; the resume kernel re-executes the slot on the
// generic path.
struct DeferRec {
    uint64_t r[11];
    int32_t pc;
    uint32_t prog;
    uint32_t steps;       // Step() calls before the slot
    uint32_t j;           // iteration of the lane's packet loop
    uint64_t lane_steps;  // steps of the lane's earlier packets in this launch
    uint64_t sm0, sm1;
    uint32_t xdp_dirty, nframes, tailcalls;
    uint32_t flag;        // == KParams::defer_epoch: suspended in that launch
};

// The state of one stepped process between launches (engine.cpp mimic_process_*; it lives in the
// process's pinned, device-mapped host block, read and written in place by the stepping kernel): the
// reference's Registers (PC, R0-R10), the current program, the step count, and the lane
// state (stack validity, xdp_md overlay, frames, tail calls, translation cache) -- the stack,
// frames and xdp_md overlay themselves stay in the process's own private memory.
struct StepState {
    uint64_t r[11];
    int32_t pc;           // Registers.PC: the next instruction (or the offending / exit one)
    uint32_t prog;        // current program (tail calls change it)
    uint32_t steps;       // Step() calls executed so far
    int32_t status;       // final MIMIC status (finished only)
    uint32_t started;     // NewProcess + Load done
    uint32_t finished;    // exited (status OK) or terminated by a fatal error
    int32_t cpu;          // Process.cpuID (-1 until SetCPUID)
    uint32_t gen;         // the process's NewProcess number (KParams::step_gen of its launches)
    uint8_t lane[256];    // the kernel's Lane record (runtime.h), opaque to the host
};
