/*
 * mimic_oracle.h -- CPU restatement of dylandreimerink/mimic's Process.Run hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (mimic_amd/) links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / the CPU baseline.
 *
 * Parity pinning: the reference is Go and cannot be compiled or imported in this
 * image (no Go toolchain; see DESIGN.md "Oracle").  This restatement is pinned by
 *   (1) the reference's own golden values (emulator_linux_helpers_test.go:11-113,
 *       :185-220, emulator_linux_map_array_test.go:10-103), and
 *   (2) hand-derived known-answer vectors for every opcode and quirk, written
 *       independently in tests/golden/make_golden.py from the cited Go lines.
 *
 * Every function in mimic_oracle.c cites the reference file:line it restates.
 */
#ifndef MIMIC_ORACLE_H
#define MIMIC_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status classes of a finished process.  The numbering is shared with the
 * product header include/mimic_amd.h (checked by tests/test_abi.py). */
enum {
    ORC_OK = 0,                   /* program exited (errExit), inst.go:277-296 */
    ORC_ERR_PC_OOB = 1,           /* errInvalidProgramCount, vm.go:297-299, :328-334 */
    ORC_ERR_UNSUPPORTED_OP = 2,   /* emulator_linux_.go:287 */
    ORC_ERR_MEM_UNRESOLVED = 3,   /* inst.go:302-305 */
    ORC_ERR_MEM_NOT_VMMEM = 4,    /* inst.go:307-310 */
    ORC_ERR_MEM_BOUNDS = 5,       /* memory_plain.go:27-34, :57-64 */
    ORC_ERR_MEM_NOT_DATASEC = 6,  /* emulator_linux_map_array.go:136-138 */
    ORC_ERR_R10_WRITE = 7,        /* vm.go:459-460 */
    ORC_ERR_HELPER_MAP_PTR = 8,   /* regToMap, emulator_linux_helpers.go:415-447 */
    ORC_ERR_HELPER_KEY = 9,       /* derefMapKey, :449-471 */
    ORC_ERR_HELPER_VALUE = 10,    /* value deref, :525-541 */
    ORC_ERR_HELPER_MAP_OP = 11,   /* non-errno map errors (cpuid, key len, not updatable/deletable) */
    ORC_ERR_HELPER_TAILCALL = 12, /* :674-710 */
    ORC_ERR_HELPER_UNIMPLEMENTED = 13, /* emulator_linux_.go:184-191 */
    ORC_ERR_HELPER_CANT_EMULATE = 14,  /* emulator_linux_helpers.go:473-475 */
    ORC_ERR_LDABS = 15,           /* emulator_linux_.go:200-285 on a non-sk_buff ctx */
    ORC_PANIC_DIV0 = 16,          /* Go runtime panic: integer divide by zero, inst_gen.go:73-92,183-202 */
    ORC_PANIC_SHIFT = 17,         /* Go runtime panic: negative shift amount, inst.go:118,129 */
    ORC_PANIC_BADREG = 18,        /* vm.go:431-432, :461-462 */
    ORC_PANIC_CALLX = 19,         /* inst.go:270-273 */
    ORC_PANIC_PC = 20,            /* negative PC indexes Instructions, vm.go:300 */
    ORC_PANIC_HELPER_NEG = 21,    /* negative helper id indexes the tables, emulator_linux_.go:126,188 */
    ORC_ERR_STEP_LIMIT = 22,      /* engine watchdog (stands for ctx deadline, vm.go:344-350) */
    ORC_ERR_CALL_DEPTH = 23,      /* engine bound on BPF-to-BPF frames (reference: unbounded) */
    ORC_ERR_ENGINE_HELPER = 24,   /* helper the reference emulates but the engine does not */
    ORC_ERR_NO_CPU = 25,          /* never produced by the batch runner (cpu always set) */
    ORC_ERR_CTX_ACCESS = 26,      /* __sk_buff / bpf_sock / bpf_flow_keys Load/Store error (read-only, invalid offset,
                                     not implemented), emulator_linux_sk_buff.go convertAccess */
    ORC_PANIC_SLICE = 27,         /* Go slice-bounds panic inside convertAccess (cb loads, IP slices, flow_keys IP) */
    ORC_ERR_CTX_LOAD = 28,        /* NewProcess: Context.Load failed (SKBuffFromBytes error, out of memory) */
    ORC_ERR_CANCELED = 29,        /* Run: ctx.Done() before a step, ctx.Err() = context.Canceled (vm.go:344-350) */
    ORC_ERR_DEADLINE = 30,        /* Run: the same with context.DeadlineExceeded */
    ORC_STATUS_COUNT
};

/* Linux map type numbers (cilium/ebpf v0.9.0 ebpf.MapType follows the kernel enum). */
enum {
    ORC_MAP_HASH = 1, ORC_MAP_ARRAY = 2, ORC_MAP_PROG_ARRAY = 3, ORC_MAP_PERF_EVENT_ARRAY = 4,
    ORC_MAP_PERCPU_HASH = 5, ORC_MAP_PERCPU_ARRAY = 6, ORC_MAP_STACK_TRACE = 7,
    ORC_MAP_CGROUP_ARRAY = 8, ORC_MAP_LRU_HASH = 9, ORC_MAP_LRU_PERCPU_HASH = 10,
    ORC_MAP_LPM_TRIE = 11, ORC_MAP_ARRAY_OF_MAPS = 12, ORC_MAP_HASH_OF_MAPS = 13,
    ORC_MAP_DEVMAP = 14, ORC_MAP_SOCKMAP = 15, ORC_MAP_CPUMAP = 16, ORC_MAP_XSKMAP = 17,
    ORC_MAP_SOCKHASH = 18, ORC_MAP_CGROUP_STORAGE = 19, ORC_MAP_REUSEPORT_SOCKARRAY = 20,
    ORC_MAP_PERCPU_CGROUP_STORAGE = 21, ORC_MAP_QUEUE = 22, ORC_MAP_STACK = 23,
    ORC_MAP_SK_STORAGE = 24, ORC_MAP_DEVMAP_HASH = 25, ORC_MAP_STRUCT_OPS = 26,
    ORC_MAP_RINGBUF = 27, ORC_MAP_INODE_STORAGE = 28, ORC_MAP_TASK_STORAGE = 29
};

typedef struct orc_vm orc_vm;
typedef struct orc_proc orc_proc;

typedef struct {
    uint32_t slot;    /* raw instruction slot of the LD_IMM64 that references the map */
    uint32_t map_id;  /* map id returned by orc_map_create */
} orc_reloc;

/* NewLinuxEmulator + NewVM(VMOptEmulator, VMOptSetvCPUs), vm.go:54-76, emulator_linux_.go:67-94 */
orc_vm *orc_vm_new(int vcpus, int stack_frame_size, int stack_frame_count, int max_tail_calls);
void orc_vm_free(orc_vm *vm);
const char *orc_last_error(orc_vm *vm);

/* MapSpecToLinuxMap + LinuxEmulator.AddMap, emulator_linux_map.go:57-113, emulator_linux_.go:97-116.
 * Returns map id >= 0, or -1. */
int orc_map_create(orc_vm *vm, const char *name, uint32_t type, uint32_t key_size,
                   uint32_t value_size, uint32_t max_entries, int datasec);
/* LinuxMap host methods.  Return 0, a positive errno (graceful), or -1 (fatal). */
int orc_map_update(orc_vm *vm, int map_id, const void *key, const void *value, uint32_t flags, int cpu);
/* lookup: *addr_out = virtual address (0 = none). */
int orc_map_lookup(orc_vm *vm, int map_id, const void *key, int cpu, uint32_t *addr_out);
int orc_map_delete(orc_vm *vm, int map_id, const void *key);
/* Dump the value backing of (map, cpu) -- E*S bytes (slot order for hash maps). */
int orc_map_values(orc_vm *vm, int map_id, int cpu, void *out, size_t cap);
/* Hash maps: occupied slot list (slot indices) and key bytes; returns count. */
int orc_map_slots(orc_vm *vm, int map_id, int32_t *slot_of_key_out, uint8_t *keys_out, size_t cap_keys);
uint32_t orc_map_addr(orc_vm *vm, int map_id);

/* VM.AddProgram with LinuxEmulator.RewriteProgram, vm.go:98-139, emulator_linux_.go:292-339.
 * raw = n_slots little-endian 8-byte BPF instruction slots. Returns prog id or -1. */
int orc_prog_load(orc_vm *vm, const char *name, const uint8_t *raw, uint32_t n_slots,
                  const orc_reloc *relocs, uint32_t n_relocs);
uint32_t orc_prog_addr(orc_vm *vm, int prog_id);

/* MemoryController helpers for host-side inspection (memory_controller.go). */
uint32_t orc_mem_add_scratch(orc_vm *vm, uint32_t size);        /* AddEntry(&PlainMemory{size}) */
int orc_mem_read(orc_vm *vm, uint32_t addr, void *buf, uint32_t len); /* GetEntry + VMMem.Read */
int orc_mem_write(orc_vm *vm, uint32_t addr, const void *buf, uint32_t len);
int orc_mem_load(orc_vm *vm, uint32_t addr, int size, uint64_t *out); /* GetEntry + VMMem.Load */
uint32_t orc_mem_next_free(orc_vm *vm);   /* address the next AddEntry would return (first-fit) */

/* Process-level access used by the reference's helper tests. */
orc_proc *orc_proc_new(orc_vm *vm, int prog_id);   /* NewProcess(id, nil) */
void orc_proc_free(orc_proc *p);                   /* Cleanup */
int orc_proc_set_cpu(orc_proc *p, int cpu);        /* SetCPUID */
uint64_t orc_proc_get_reg(orc_proc *p, int r);
void orc_proc_set_reg(orc_proc *p, int r, uint64_t v);
/* Single-process stepping: NewProcess with an xdp_md context, Process.Step (0 continue, -1
 * exited, > 0 fatal status), Registers.PC and the current program. */
orc_proc *orc_proc_new_xdp(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t H, uint32_t T,
                           int32_t ingress, int32_t rxq, int32_t egress);
/* NewProcess with a LinuxContextSKBuff (its Load runs here); NULL + *status when it fails */
orc_proc *orc_proc_new_skb(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t ifindex, int *status);
/* the same with a user-given SK / FlowKeys (custom may be NULL) */
orc_proc *orc_proc_new_skb_ctx(orc_vm *vm, int prog_id, const uint8_t *pkt, uint32_t L, uint32_t ifindex,
                               const void *custom, int *status);
int orc_proc_step(orc_proc *p, int32_t *err_pc);
int64_t orc_proc_get_pc(orc_proc *p);
int orc_proc_get_prog(orc_proc *p);
/* emulator.CallHelperFunction directly (as the reference tests call linuxHelper* directly). */
int orc_proc_call_helper(orc_proc *p, int32_t helper);

/* One xdp_md batch, run sequentially in packet order: for each packet i:
 * NewProcess(prog, LinuxContextXDP{H,T,pkt,ingress,rxq,egress}), SetCPUID(cpu[i]),
 * Run (with step budget), read R0, copy packet memory back, Cleanup.
 * pkt_mem[i] region = pkt_data + pkt_off[i], length H+L+T with the packet at +H
 * (the caller lays the headroom/tailroom out; they are re-zeroed on load as the
 * reference allocates fresh zeroed memory, context_xdp_md.go:52-64).
 * Arrays may be NULL: ingress/rxq/egress -> 0; headroom/tailroom -> the scalar. */
typedef struct {
    uint32_t n;
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    const uint32_t *headroom_arr; uint32_t headroom;
    const uint32_t *tailroom_arr; uint32_t tailroom;
    const int32_t *ingress_ifindex;
    const int32_t *rx_queue_index;
    const int32_t *egress_ifindex;
    const int32_t *cpu;
    uint64_t step_budget;   /* 0 = default (1<<22) */
    int write_back;         /* copy packet memory back into pkt_data after Run */
    /* Run(ctx) of packet i: ctx_done[i] = 0 (ctx not done: context.Background()), 1 (canceled) or
     * 2 (deadline exceeded) -- the state ctx.Done() / ctx.Err() show before every step (vm.go:343-350).
     * NULL = every ctx is context.Background(). */
    const uint8_t *ctx_done;
    /* ctx_done_step[i]: the ctx is seen done before step ctx_done_step[i] (0: before the first);
     * NULL = before the first.  (A cancel while a process runs, at the step the engine saw it.) */
    const uint32_t *ctx_done_step;
} orc_xdp_batch;

typedef struct {
    uint64_t *r0;
    uint8_t *status;
    uint32_t *steps;
    int32_t *err_pc;
} orc_results;

int orc_run_xdp_batch(orc_vm *vm, int prog_id, const orc_xdp_batch *b, orc_results *out);

/* sk_buff batches (LinuxContextSKBuff, context_sk_buff.go): packet i is pkt_len[i] bytes at
 * pkt_data + pkt_off[i] + 32; the process sees packet memory [pkt_off[i], +32+L+64) (headroom
 * 32, tailroom 64, emulator_linux_sk_buff.go:113-121), written back when write_back is set. */
/* A user-given SK / FlowKeys of one context (LinuxContextSKBuff.SK / .FlowKeys, context_sk_buff.go:
 * 24-26, put in place at Load :53-66): the same layout as the engine's mimic_skb_custom.  sk_ip_len
 * = len() of the SK's srcIP4 / dstIP4 / srcIP6 / dstIP6 net.IP (0 = nil), sk_ip their bytes. */
#define ORC_SKB_CUSTOM_SK 1u
#define ORC_SKB_CUSTOM_FLOWKEYS 2u
typedef struct {
    uint32_t flags;
    uint32_t sk_bound_dev_if, sk_family, sk_type, sk_protocol, sk_mark, sk_priority;
    uint32_t sk_src_port, sk_dst_port, sk_state;
    int32_t sk_rx_queue_mapping;
    uint8_t sk_ip_len[4];
    uint8_t sk_ip[4][16];
    uint16_t fk_nhoff, fk_thoff, fk_addr_proto;
    uint8_t fk_is_frag, fk_is_first_frag, fk_is_encap, fk_ip_proto;
    uint16_t fk_n_proto, fk_sport, fk_dport;
    uint32_t fk_flags, fk_flow_label;
} orc_skb_custom;

typedef struct {
    uint32_t n;
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    uint32_t ifindex;       /* NetDev.IFIndex (ctx "dev") */
    const int32_t *cpu;
    uint64_t step_budget;
    int write_back;
    const orc_skb_custom *custom;   /* [n] or NULL: the contexts' user-given SK / FlowKeys */
    const uint8_t *ctx_done;        /* as in orc_xdp_batch */
    const uint32_t *ctx_done_step;  /* as in orc_xdp_batch */
} orc_skb_batch;
int orc_run_skb_batch(orc_vm *vm, int prog_id, const orc_skb_batch *b, orc_results *out);

#ifdef __cplusplus
}
#endif
#endif
