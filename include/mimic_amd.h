/*
 * mimic_amd.h -- C ABI of the MI355X batch-eBPF engine (the drop-in boundary).
 *
 * The reference (dylandreimerink/mimic, Go) exposes the hot path as
 *   NewLinuxEmulator / NewVM              vm.go:54-76, emulator_linux_.go:67-94
 *   MapSpecToLinuxMap + emu.AddMap        emulator_linux_map.go:57-113, emulator_linux_.go:97-116
 *   LinuxMap Lookup/Update/Delete/Keys    emulator_linux_map.go:14-54
 *   VM.AddProgram                         vm.go:98-139 (+ RewriteProgram, emulator_linux_.go:292-339)
 *   VM.NewProcess + Process.SetCPUID + Process.Run + Process.Cleanup
 *                                         vm.go:198-374 with LinuxContextXDP, context_xdp_md.go:47-133
 *   MemoryController.GetEntry + VMMem.Load/Read (host inspection)  memory_controller.go:117-145
 * Each entry point below names the reference interface it replaces.  A Go maintainer
 * binds them with cgo; tests bind them with ctypes.
 *
 * Conventions: every function returns 0 on success, a negative MIMIC_E* on failure
 * (text via mimic_last_error), or -- for map operations only -- a positive errno that
 * the reference returns gracefully as a syscall.Errno (E2BIG = 7).
 * Host pointers are host memory unless a field says DEVICE.  The engine owns all device
 * memory it allocates; the caller owns batch/result buffers.  One mimic_vm is one HIP
 * device + one command stream.  Batch and map calls on one vm must be serialised by the
 * caller; the mimic_process_* calls may come from several threads at once (processPool's
 * workers and Handoff goroutines, vm.go:548-573, clean up while others create and run
 * processes): the engine serialises them per vm.  Distinct vms may run concurrently.
 */
#ifndef MIMIC_AMD_H
#define MIMIC_AMD_H

#if !defined(__HIPCC_RTC__)  /* hipRTC (the JIT kernels) provides these types itself */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define MIMIC_ABI_VERSION 4  /* 2: mimic_skb_batch.custom, statuses 29-30, MIMIC_EXEC_SPREAD; 3: MIMIC_EXEC_SPREAD_OWN;
                                4: status 31, thread-safe process calls, mimic_run_xdp_many */

/* errors */
#define MIMIC_EINVAL (-1)
#define MIMIC_ENOMEM (-2)
#define MIMIC_EDEVICE (-3)
#define MIMIC_ENOTSUP (-4)
#define MIMIC_ENOENT (-5)
#define MIMIC_EFAULT (-6)
#define MIMIC_ECANCELED (-7)   /* mimic_process_run_ctx: the context was canceled ("context canceled") */
#define MIMIC_EDEADLINE (-8)   /* mimic_process_run_ctx: its deadline passed ("context deadline exceeded") */

/* Per-process status classes (one byte per packet).  Same numbering as the oracle. */
enum mimic_status {
    MIMIC_OK = 0,                    /* exited via EXIT (inst.go:277-296) */
    MIMIC_ERR_PC_OOB = 1,            /* errInvalidProgramCount (vm.go:285,297,328) */
    MIMIC_ERR_UNSUPPORTED_OP = 2,    /* emulator_linux_.go:287 */
    MIMIC_ERR_MEM_UNRESOLVED = 3,    /* inst.go:302-305 */
    MIMIC_ERR_MEM_NOT_VMMEM = 4,     /* inst.go:307-310 */
    MIMIC_ERR_MEM_BOUNDS = 5,        /* memory_plain.go:27,57 */
    MIMIC_ERR_MEM_NOT_DATASEC = 6,   /* emulator_linux_map_array.go:136-138 */
    MIMIC_ERR_R10_WRITE = 7,         /* vm.go:459-460 */
    MIMIC_ERR_HELPER_MAP_PTR = 8,    /* emulator_linux_helpers.go:415-447 */
    MIMIC_ERR_HELPER_KEY = 9,        /* :449-471 */
    MIMIC_ERR_HELPER_VALUE = 10,     /* :525-541 */
    MIMIC_ERR_HELPER_MAP_OP = 11,    /* non-errno LinuxMap errors */
    MIMIC_ERR_HELPER_TAILCALL = 12,  /* :674-710 */
    MIMIC_ERR_HELPER_UNIMPLEMENTED = 13, /* emulator_linux_.go:184-191 */
    MIMIC_ERR_HELPER_CANT_EMULATE = 14,  /* emulator_linux_helpers.go:473-475 */
    MIMIC_ERR_LDABS = 15,            /* emulator_linux_.go:200-285 on an xdp_md ctx */
    MIMIC_PANIC_DIV0 = 16,           /* Go panic, inst_gen.go:73-92,183-202 */
    MIMIC_PANIC_SHIFT = 17,          /* Go panic, inst.go:118,129 */
    MIMIC_PANIC_BADREG = 18,         /* vm.go:431-432,461-462 */
    MIMIC_PANIC_CALLX = 19,          /* inst.go:270-273 */
    MIMIC_PANIC_PC = 20,             /* negative PC, vm.go:300 */
    MIMIC_PANIC_HELPER_NEG = 21,     /* negative helper id, emulator_linux_.go:126 */
    MIMIC_ERR_STEP_LIMIT = 22,       /* step budget: the engine's watchdog next to Run's ctx (mimic_run_*_ctx) */
    MIMIC_ERR_CALL_DEPTH = 23,       /* > MIMIC_MAX_FRAMES nested BPF-to-BPF calls */
    MIMIC_ERR_ENGINE_HELPER = 24,    /* helper the reference emulates but this engine does not */
    MIMIC_ERR_NO_CPU = 25,
    MIMIC_ERR_CTX_ACCESS = 26,       /* __sk_buff / bpf_sock / bpf_flow_keys field error, emulator_linux_sk_buff.go */
    MIMIC_PANIC_SLICE = 27,          /* Go slice-bounds panic in those accessors */
    MIMIC_ERR_CTX_LOAD = 28,         /* Context.Load failed (SKBuffFromBytes error, out of address space) */
    MIMIC_ERR_CANCELED = 29,         /* Run's ctx was canceled: ctx.Err() = context.Canceled (vm.go:344-350) */
    MIMIC_ERR_DEADLINE = 30,         /* Run's ctx deadline passed: context.DeadlineExceeded (vm.go:344-350) */
    MIMIC_ERR_ENGINE_STATE = 31      /* engine assertion: a stepping launch found another process's state (never expected) */
};

/* Linux map types (ebpf.MapType). */
#define MIMIC_MAP_HASH 1
#define MIMIC_MAP_ARRAY 2
#define MIMIC_MAP_PROG_ARRAY 3
#define MIMIC_MAP_PERCPU_HASH 5
#define MIMIC_MAP_PERCPU_ARRAY 6

#define MIMIC_MAP_F_DATASEC 1u  /* Spec.Value is a *btf.Datasec (.data/.bss/.rodata) */

/* schedules: which vCPU runs packet i (the caller's SetCPUID, vm.go:268) */
#define MIMIC_SCHED_CHUNKED 0      /* contiguous chunks of ceil(N/V) packets per vCPU */
#define MIMIC_SCHED_INTERLEAVED 1  /* packet i on vCPU i % V */
#define MIMIC_SCHED_EXPLICIT 2     /* cpu[i] given; each vCPU runs its packets in index order */

typedef struct mimic_vm mimic_vm;

typedef struct {
    int32_t vcpus;              /* VMSettings.VirtualCPUs (vm.go:21-22, VMOptSetvCPUs) */
    int32_t stack_frame_size;   /* VMSettings.StackFrameSize, default 256 (vm.go:60) */
    int32_t stack_frame_count;  /* VMSettings.StackFrameCount, default 8 (vm.go:62) */
    int32_t max_tail_calls;     /* LinuxEmulatorSettings.MaxTailCalls, default 33 (emulator_linux_.go:78) */
    int32_t device;             /* HIP device ordinal */
    int32_t vcpu_begin;         /* this engine executes vCPUs [vcpu_begin, vcpu_begin+vcpu_count) */
    int32_t vcpu_count;         /* 0 = all */
    int32_t exec_mode;          /* MIMIC_EXEC_*: 0 = default (env MIMIC_EXEC=interp|jit, else JIT) */
} mimic_vm_settings;

#define MIMIC_EXEC_DEFAULT 0
#define MIMIC_EXEC_INTERP 1   /* the batch interpreter kernel (interp.hip) */
#define MIMIC_EXEC_JIT 2      /* per-program-set kernels generated from the loaded programs, hipRTC-compiled */
#define MIMIC_EXEC_SPREAD 3   /* mimic_last_exec only: the JIT's spread kernel (a vCPU's packets on many lanes) */
#define MIMIC_EXEC_SPREAD_OWN 4   /* mimic_last_exec only: its owned form (a block runs every packet of its vCPUs) */

typedef struct {
    const char *name;
    uint32_t type, key_size, value_size, max_entries, flags;
} mimic_map_spec;

typedef struct {
    uint32_t slot;    /* raw slot of an LD_IMM64 with src PseudoMapFD(1)/PseudoMapValue(2) */
    uint32_t map_id;
} mimic_reloc;

/* One batch of xdp_md processes.  All pointers are DEVICE pointers; NULL arrays fall
 * back to the scalar next to them.  Packet memory i is pkt_data[pkt_off[i] ..
 * pkt_off[i]+H+L+T) with the packet at +H (context_xdp_md.go:52-64); the engine zeroes the
 * headroom/tailroom bytes, then runs the program on that memory IN PLACE, so the caller
 * sees every packet write afterwards. */
typedef struct {
    uint32_t n;
    uint32_t schedule;          /* MIMIC_SCHED_* */
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    const uint32_t *headroom;  uint32_t headroom_all;
    const uint32_t *tailroom;  uint32_t tailroom_all;
    const int32_t *ingress_ifindex; int32_t ingress_all;
    const int32_t *rx_queue_index;  int32_t rxq_all;
    const int32_t *egress_ifindex;  int32_t egress_all;
    const int32_t *cpu;         /* HOST array for MIMIC_SCHED_EXPLICIT (the engine builds the per-vCPU lists) */
    uint64_t step_budget;       /* 0 = MIMIC default; the per-process watchdog (contexts: mimic_run_xdp_ctx) */
} mimic_xdp_batch;

typedef struct {                /* DEVICE arrays of n entries, any may be NULL */
    uint64_t *r0;               /* p.Registers.R0 after Run */
    uint8_t *status;            /* enum mimic_status */
    uint32_t *steps;            /* number of Step() calls Run made */
    int32_t *err_pc;            /* PC of the failing instruction, -1 on MIMIC_OK */
} mimic_xdp_results;

int mimic_abi_version(void);
const char *mimic_last_error(const mimic_vm *vm);

/* NewLinuxEmulator(OptMaxTailCalls) + NewVM(VMOptEmulator, VMOptSetvCPUs). vm.go:54-76 */
int mimic_vm_create(const mimic_vm_settings *settings, mimic_vm **out);
void mimic_vm_destroy(mimic_vm *vm);

/* MapSpecToLinuxMap + LinuxEmulator.AddMap. emulator_linux_map.go:57, emulator_linux_.go:97 */
int mimic_map_create(mimic_vm *vm, const mimic_map_spec *spec, uint32_t *map_id);
/* LinuxMapUpdater.Update(key, value, flags, cpuid). emulator_linux_map.go:31-36 */
int mimic_map_update(mimic_vm *vm, uint32_t map_id, const void *key, const void *value, uint32_t flags, int32_t cpu);
/* n mimic_map_update calls in one: keys packed key_size bytes apart, values value_size bytes
 * apart; rc_out[i] (optional) = the i-th call's result (0 or a positive errno).  Not in the
 * reference API (a loop over LinuxMap.Update, emulator_linux_map_hash.go:158-203).  Host map
 * operations run on a host image of the map's index and are staged: they reach the device before
 * the next batch or map read, with no device round trip per call. */
int mimic_map_update_batch(mimic_vm *vm, uint32_t map_id, const void *keys, const void *values, uint32_t n,
                           uint32_t flags, int32_t cpu, int32_t *rc_out);
/* LinuxMap.Lookup(key, cpuid) -> virtual address of the value (0 = not found). emulator_linux_map.go:25-27 */
int mimic_map_lookup(mimic_vm *vm, uint32_t map_id, const void *key, int32_t cpu, uint32_t *addr_out);
/* LinuxMapDeleter.Delete(key). emulator_linux_map.go:38-42 */
int mimic_map_delete(mimic_vm *vm, uint32_t map_id, const void *key);
/* LinuxMap.Keys(cpuid): the live keys packed (key_size bytes each) into out, count in *n_out.
 * emulator_linux_map_hash.go:113-131 (Go map order there, table order here), emulator_linux_map_array.go:64-75 */
int mimic_map_keys(mimic_vm *vm, uint32_t map_id, void *out, size_t cap, uint32_t *n_out);
/* Hash maps: live keys with their slot (LinuxHashMap.KeyToIndex, emulator_linux_map_hash.go:29-30);
 * the value of key i on cpu c is values[c][slot_i * value_size]. */
int mimic_map_entries(mimic_vm *vm, uint32_t map_id, void *keys_out, int32_t *slots_out, size_t cap_entries,
                      uint32_t *n_out);
/* Raw value backing of (map, cpu): E*S bytes, slot order (D2H copy). */
int mimic_map_read_values(mimic_vm *vm, uint32_t map_id, int32_t cpu, void *out, size_t cap);
/* Not in the reference API: the map's state back to a fresh NewLinuxHashMap / NewLinuxArrayMap at
 * the same addresses (values and keys zeroed; hash: every bucket empty, freelist 0..E-1 in order,
 * emulator_linux_map_hash.go:56-64), queued on hip_stream (NULL: the VM's stream).  What a caller
 * re-creating the map per batch would get, without a new layout; the bench's inserting-batch line
 * uses it. */
int mimic_map_reset(mimic_vm *vm, uint32_t map_id, void *hip_stream);
/* Value backings of vCPUs [cpu_begin, cpu_end) of a per-CPU map ([0, 1) otherwise), cpu-major:
 * (cpu_end - cpu_begin) * E*S bytes in one D2H copy -- LinuxMap.Values(cpuid) for every cpu of a range
 * (emulator_linux_map_array.go:223-233, emulator_linux_map_hash.go:628-640). */
int mimic_map_read_values_range(mimic_vm *vm, uint32_t map_id, int32_t cpu_begin, int32_t cpu_end, void *out,
                                size_t cap);
/* Sum over vCPUs [cpu_begin, cpu_end) of a per-CPU map's u64 values -> out[E] (device reduction). */
int mimic_map_sum_u64(mimic_vm *vm, uint32_t map_id, int32_t cpu_begin, int32_t cpu_end, uint64_t *out, size_t cap);
/* One hash table for two VMs (not in the reference API: its LinuxHashMap is shared by every process
 * of a processPool, emulator_linux_map_hash.go:21-255; here by engines that each run a shard of the
 * packets).  vm's map `map_id` uses owner's map `owner_map_id` -- same spec, same device -- as its
 * memory: every insert, E2BIG, lookup and host operation of either VM sees the other's.  Call after
 * both VMs created all their maps; the programs of both must not delete (every launch on the table
 * is pop-only); the owner must outlive the other VM.  Host operations on a shared table wait for
 * the whole device first. */
int mimic_map_share(mimic_vm *vm, uint32_t map_id, mimic_vm *owner, uint32_t owner_map_id);
/* MemoryController.GetEntryByObject(map).Addr */
int mimic_map_addr(mimic_vm *vm, uint32_t map_id, uint32_t *addr_out);

/* VM.AddProgram(spec) with the LinuxEmulator map rewrite. vm.go:98-139, emulator_linux_.go:292-339.
 * insns = n_slots raw little-endian 8-byte instruction slots (ELF .text bytes). */
int mimic_program_load(mimic_vm *vm, const char *name, const void *insns, uint32_t n_slots,
                       const mimic_reloc *relocs, uint32_t n_relocs, uint32_t *prog_id);
/* MemoryController.GetEntryByObject(prog).Addr -- the value a prog array stores. */
int mimic_program_addr(mimic_vm *vm, uint32_t prog_id, uint32_t *addr_out);

/* MemoryController.GetEntry(addr) + VMMem.Read / Load on static entries (maps). */
int mimic_mem_read(mimic_vm *vm, uint32_t addr, void *buf, uint32_t len);
int mimic_mem_load(mimic_vm *vm, uint32_t addr, int32_t size, uint64_t *out);
/* Address the per-process stack entry gets (first free address after the static entries). */
int mimic_stack_addr(mimic_vm *vm, uint32_t *addr_out);

/* Batch form of: for each packet i { p := vm.NewProcess(prog, &LinuxContextXDP{...});
 * p.SetCPUID(cpu(i)); p.Run(ctx); r0[i] = p.Registers.R0; p.Cleanup() }  (vm.go:198-374).
 * Enqueued on `hip_stream` (a hipStream_t, NULL = the vm's own stream); returns when enqueued.
 * Hash inserts of concurrent vCPUs take freelist slots in arrival order (the reference's pool is
 * no different); after the batch the used slots of a hash map are [0, m), as m sequential pops leave
 * them (a compaction kernel follows a launch that reserved positions in chunks, on the same stream),
 * and E2BIG is answered exactly when every slot is live. */
int mimic_run_xdp(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *batch,
                  const mimic_xdp_results *results, void *hip_stream);
/* k batches (DEVICE pointers as above), enqueued like mimic_run_xdp, as few launches as possible: up
 * to 8 batches of the same size, schedule (not EXPLICIT) and scalar fields, with no per-packet arrays,
 * run as ONE launch when the programs allow the owned spread kernel (mimic_set_spread); every vCPU
 * then runs its packets of batch 0, then of batch 1, ... (processPool draining a backlog of batches,
 * vm.go:548-573).  Otherwise one launch per batch.  Not in the reference API. */
int mimic_run_xdp_many(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *batches,
                       const mimic_xdp_results *results, uint32_t k, void *hip_stream);
/* One batch of sk_buff processes (LinuxContextSKBuff, context_sk_buff.go:20-119).  DEVICE
 * pointers as in mimic_xdp_batch.  Process i's packet memory is pkt_data[pkt_off[i] ..
 * pkt_off[i]+32+L+64) with the packet's L = pkt_len[i] bytes at +32 (SKBuffFromBytes'
 * headroom / tailroom, emulator_linux_sk_buff.go:108-121); the engine zeroes the room bytes
 * and runs the program on that memory IN PLACE (BigEndian scalar accesses).  A packet whose
 * Load fails (a second link / network / transport layer) gets MIMIC_ERR_CTX_LOAD and its
 * memory is not touched.  Cleanup leaks the sock / flow-keys / packet entries exactly as the
 * reference does (context_sk_buff.go:110-119), so their addresses keep growing across
 * batches until mimic_skb_release. */
#define MIMIC_CTX_XDP 0
#define MIMIC_CTX_SKB 1
/* A user-given sock and / or flow keys of one sk_buff context (LinuxContextSKBuff.SK / .FlowKeys,
 * JSON "sock" / "flowKeys", context_sk_buff.go:24-26; Load puts them in place of the ones
 * SKBuffFromBytes made, :53-66).  SK fields: emulator_linux_sk_buff.go:698-718; its net.IP fields
 * as SK.UnmarshalJSON leaves them (:721-757): the bytes net.ParseIP returns (16 for any address;
 * To16 for the IPv6 ones), else make(net.IP, 4 / 16); length 0 = nil (an SK built without
 * UnmarshalJSON).  FlowKeys fields (:967-982) are the initial values of the writable flow keys;
 * its SrcIPv6orIPv4 is never readable (convertAccess slices a 16-byte copy at offsets 16..31,
 * :1117-1140: a panic for every access), so it is not carried. */
#define MIMIC_SKB_CUSTOM_SK 1u
#define MIMIC_SKB_CUSTOM_FLOWKEYS 2u
typedef struct {
    uint32_t flags;             /* MIMIC_SKB_CUSTOM_*: which of the two the context gives (0: none) */
    uint32_t sk_bound_dev_if, sk_family, sk_type, sk_protocol, sk_mark, sk_priority;
    uint32_t sk_src_port, sk_dst_port, sk_state;
    int32_t sk_rx_queue_mapping;
    uint8_t sk_ip_len[4];       /* srcIP4, dstIP4, srcIP6, dstIP6: len() of the net.IP (0 = nil, <= 16) */
    uint8_t sk_ip[4][16];
    uint16_t fk_nhoff, fk_thoff, fk_addr_proto;
    uint8_t fk_is_frag, fk_is_first_frag, fk_is_encap, fk_ip_proto;
    uint16_t fk_n_proto, fk_sport, fk_dport;
    uint32_t fk_flags, fk_flow_label;
} mimic_skb_custom;

typedef struct {
    uint32_t n;
    uint32_t schedule;          /* MIMIC_SCHED_* */
    uint8_t *pkt_data;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    uint32_t ifindex;           /* LinuxContextSKBuff.Dev.IFIndex (__sk_buff.ifindex) */
    int32_t pad;
    const int32_t *cpu;         /* HOST array for MIMIC_SCHED_EXPLICIT */
    uint64_t step_budget;       /* 0 = MIMIC default */
    const mimic_skb_custom *custom;   /* DEVICE array [n] of user-given sock / flow keys, or NULL (none) */
    /* DEVICE word (optional) the engine keeps for this batch's packet memory: 1 once a launch left
     * every head- and tailroom byte zero, 0 (the caller's initial value) when unknown.  A launch that
     * finds 1 skips reading the 96 room bytes per packet (Load hands the program zeroed rooms,
     * context_sk_buff.go:42-107); a program store into a room sets it back to 0.  Reset it to 0 after
     * writing the packet memory by other means, and give each set of packets its own word. */
    uint32_t *rooms_state;
} mimic_skb_batch;

/* Batch form of: for each packet i { p := vm.NewProcess(prog, &LinuxContextSKBuff{Packet: pkt_i,
 * Dev: &NetDev{IFIndex}}); p.SetCPUID(cpu(i)); p.Run(ctx); r0[i] = p.Registers.R0; p.Cleanup() }
 * (vm.go:198-374, context_sk_buff.go:42-119).  Enqueued on `hip_stream` like mimic_run_xdp. */
int mimic_run_skb(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *batch,
                  const mimic_xdp_results *results, void *hip_stream);
/* Drop the sock / flow-keys / packet entries earlier sk_buff processes leaked: the state of a
 * fresh VM with the same maps and programs (no reference counterpart; the reference never
 * frees them).  Needed before adding maps / programs or running xdp_md batches again. */
int mimic_skb_release(mimic_vm *vm);

/* ---- single processes: the NewProcess / SetCPUID / Step / Run / Cleanup surface ---------------
 * A process holds its own packet memory, private memory (stack, frames) and register state on
 * the device, so it can be advanced instruction by instruction (the edb debugger's use of
 * Process.Step, Readme.md:8).  Steps run on the batch interpreter with one lane; xdp_md contexts
 * (mimic_process_new) and sk_buff contexts (mimic_process_new_skb / _ctx). */
typedef struct mimic_process mimic_process;
typedef struct {
    uint64_t r[11];             /* Registers.R0 .. R10 */
    int32_t pc;                 /* Registers.PC: next instruction; the offending one after an error */
    uint32_t prog_id;           /* the program PC indexes (tail calls switch it) */
    uint64_t steps;             /* Step() calls that executed an instruction so far */
    int32_t status;             /* MIMIC_OK, or the fatal status once the process terminated */
    uint32_t exited;            /* Step's `exited`: the program exited or hit a fatal error */
} mimic_process_regs;
/* VM.NewProcess(prog, &LinuxContextXDP{Packet, Headroom, Tailroom, ...}). vm.go:198-235,
 * context_xdp_md.go:47-115.  packet = host bytes. */
int mimic_process_new(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t headroom,
                      uint32_t tailroom, int32_t ingress_ifindex, int32_t rx_queue_index, int32_t egress_ifindex,
                      mimic_process **out);
/* Process.SetCPUID: id < 0 or id > V is an error (vm.go:268-283); never called = -1 (vm.go:214). */
/* VM.NewProcess(prog, &LinuxContextSKBuff{Packet, Dev{IFIndex}}) (vm.go:198-235, context_sk_buff.go:42-107):
 * the context's Load runs here (its sk_buff / sock / flow-keys / packet entries take the VM's next
 * leak addresses, as the reference's would); Step / Run / Packet as for xdp_md processes, the
 * packet memory being 32 + len + 64 bytes (headroom, frame, tailroom; emulator_linux_sk_buff.go:113-116). */
int mimic_process_new_skb(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t ifindex,
                          mimic_process **out);
/* The same with a user-given sock / flow keys (custom: HOST pointer, or NULL). */
int mimic_process_new_skb_ctx(mimic_vm *vm, uint32_t prog_id, const void *packet, uint32_t len, uint32_t ifindex,
                              const mimic_skb_custom *custom, mimic_process **out);
int mimic_process_set_cpu(mimic_process *p, int32_t id);
/* n x Process.Step (vm.go:291-340), stopping early when the process exits or fails; the
 * registers after the last step in *out.  Stepping a process that hit a fatal error returns
 * MIMIC_EINVAL ("process has been terminated"); after a clean exit Step reports exited again. */
int mimic_process_step(mimic_process *p, uint32_t n, mimic_process_regs *out);
/* Process.Run (vm.go:343-360): Step until exit / fatal error, or `budget` more steps (0 = the
 * default budget; a suspended process can be run or stepped again). */
int mimic_process_run(mimic_process *p, uint64_t budget, mimic_process_regs *out);
/* ---- Run(ctx): cancellation and deadlines (vm.go:343-360) ----------------------------------------
 * The reference's Run checks ctx.Done() before every step and returns ctx.Err() once it is closed;
 * a process pool job whose context is done before it starts is handed off with ctx.Err()
 * (vm.go:548-573).  A mimic_ctx is that context: context.WithCancel(context.Background()) when
 * timeout_ns = 0, else context.WithTimeout(.., timeout_ns) (a host timer marks it at the deadline).
 * It is a word in pinned, device-mapped host memory that running kernels read: a batch given
 * contexts checks packet i's context before its process's first step -- a done one ends the process
 * there with MIMIC_ERR_CANCELED / MIMIC_ERR_DEADLINE, 0 steps, R0 = 0, err_pc = 0, its context Load
 * done (xdp_md rooms zeroed, sk_buff entries leaked), as Run(ctx) on a done context after NewProcess.
 * A running process reads its context again every 4096 steps and stops before its next step once
 * it is done (status as above, steps and registers where it stopped); mimic_process_run_ctx checks
 * between launch slices.  mimic_ctx_free waits for the launches that read the context. */
typedef struct mimic_ctx mimic_ctx;
int mimic_ctx_new(uint64_t timeout_ns, mimic_ctx **out);
/* the CancelFunc: Err() becomes context.Canceled, unless the context is done already */
void mimic_ctx_cancel(mimic_ctx *c);
/* ctx.Err(): 0 = nil, 1 = context.Canceled, 2 = context.DeadlineExceeded */
int mimic_ctx_err(const mimic_ctx *c);
/* 1 when the word is device-visible (made with a device present; runs refuse other contexts) */
int mimic_ctx_pinned(const mimic_ctx *c);
void mimic_ctx_free(mimic_ctx *c);
/* mimic_run_xdp / mimic_run_skb with contexts: ctx for every packet, or ctx_per_packet = HOST array
 * [n] of contexts (NULL entries: context.Background()); not both.  NULL and NULL = the plain call. */
int mimic_run_xdp_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_batch *batch, const mimic_xdp_results *results,
                      void *hip_stream, mimic_ctx *ctx, mimic_ctx *const *ctx_per_packet);
int mimic_run_skb_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_skb_batch *batch, const mimic_xdp_results *results,
                      void *hip_stream, mimic_ctx *ctx, mimic_ctx *const *ctx_per_packet);
/* Process.Run(ctx) (vm.go:343-360): as mimic_process_run, the context checked between launch
 * slices; a done context returns MIMIC_ECANCELED / MIMIC_EDEADLINE (text: Go's ctx.Err() string)
 * with *out holding the suspended process (Run / Step continue it).  budget 0: no step budget. */
int mimic_process_run_ctx(mimic_process *p, uint64_t budget, mimic_ctx *ctx, mimic_process_regs *out);
/* processPool's workers (vm.go:548-573): n x Process.Run(ctx) of fresh (never stepped or run) sk_buff
 * processes of one VM, program and ifindex, as ONE device launch instead of one launch per process.
 * Each process keeps the sock / flow-keys / packet addresses its Load reserved at NewProcess and runs
 * on its SetCPUID vCPU (-1 and V allowed; cpus: HOST array [n] that sets them first, or NULL); a
 * vCPU's processes run in array order.  ctxs: HOST array [n] of contexts (NULL entries, or ctxs NULL:
 * Background), no step budget.  Afterwards every process is finished: out[i] (optional, [n]) and the
 * process hold R0, status, steps; a batch lane keeps no R1-R10 (zero) and pc is the failing
 * instruction or -1.  Not in the reference API. */
int mimic_process_run_many(mimic_process *const *ps, uint32_t n, const int32_t *cpus, mimic_ctx *const *ctxs,
                           mimic_process_regs *out);
/* n x Process.Cleanup with one wait for the VM's stream (NULL entries skipped). */
void mimic_process_free_many(mimic_process *const *ps, uint32_t n);

/* The process's packet memory (headroom + packet + tailroom) as the program left it. */
int mimic_process_packet(mimic_process *p, void *buf, size_t cap);
/* Process.Cleanup (vm.go:363-374): frees the process. */
void mimic_process_free(mimic_process *p);

/* Wait for all work the vm enqueued on `hip_stream` (NULL = own stream). */
int mimic_sync(mimic_vm *vm, void *hip_stream);
/* Executed Step() count of the last completed mimic_run_xdp (sum over packets). */
int mimic_last_steps(mimic_vm *vm, uint64_t *steps_out);

/* Host-resident batches: packets start and end in host memory (captured pcap, ctx JSON, NIC
 * buffers).  The engine pipelines the batch in sub-batches: H2D of the sub-batch's descriptors,
 * packet window and launch parameters, the kernel, D2H of r0/status (and of the packet memory
 * when pkt_out is set), on separate streams so that copies overlap kernels.  vCPU assignment is
 * that of the whole batch.  pkt_out needs each sub-batch's packets ascending and non-overlapping.
 * Host memory should be pinned (mimic_host_register) for the copies to run asynchronously. */
typedef struct {
    uint32_t n;
    uint32_t schedule;            /* MIMIC_SCHED_*; CHUNKED runs as the equivalent EXPLICIT schedule */
    const uint8_t *pkt_data;      /* host */
    const uint64_t *pkt_off;      /* host, [n] */
    const uint32_t *pkt_len;      /* host, [n] */
    uint32_t headroom_all, tailroom_all;
    int32_t ingress_all, rxq_all, egress_all;
    int32_t pad;
    const int32_t *cpu;           /* host, EXPLICIT */
    uint64_t step_budget;
    uint8_t *pkt_out;             /* optional host: packet memory after the run (needs ascending pkt_off) */
    uint64_t *r0;                 /* host, [n] */
    uint8_t *status;              /* host, [n] */
} mimic_xdp_host_batch;
/* chunks = number of sub-batches (0: about 16 MiB of packet memory each) */
int mimic_run_xdp_host(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks);
/* The same with Run(ctx): every sub-batch's kernel reads ctx (see mimic_run_xdp_ctx). */
int mimic_run_xdp_host_ctx(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                           mimic_ctx *ctx);
/* The same with one context per packet (ctx_per_packet[i], NULL: none) -- processPool's jobs each
 * carry their own ctx (vm.go:548-573); the contexts' words go to the device once per call. */
int mimic_run_xdp_host_ctx_pp(mimic_vm *vm, uint32_t prog_id, const mimic_xdp_host_batch *hb, uint32_t chunks,
                              mimic_ctx *const *ctx_per_packet);
/* Pin / unpin host memory for DMA (hipHostRegister / hipHostUnregister). */
int mimic_host_register(void *p, size_t bytes);
int mimic_host_unregister(void *p);

/* Execution mode the VM resolved to (MIMIC_EXEC_INTERP / MIMIC_EXEC_JIT). */
int mimic_exec_mode(const mimic_vm *vm);
/* Spread launches (no reference counterpart: an engine schedule for processPool's jobs,
 * vm.go:548-573).  When every per-CPU access of the loaded xdp_md programs is a fused counter
 * increment through one per-CPU array lookup, a vCPU's packets may run on many lanes (the final
 * counters are sums; each packet's R0 / status / steps depend on its own bytes only).
 * mode -1: default (env MIMIC_SPREAD, else when a batch has >= 8 packets per vCPU), 0: never,
 * 1: whenever the programs allow it.  The owned form (MIMIC_EXEC_SPREAD_OWN: a workgroup runs every
 * packet of its vCPUs and adds into rows only it touches) takes, by default, every batch of 2..256
 * packets per vCPU, whatever V, when the counted map's rows fit its LDS table of min(256, 32 KiB / row)
 * rows (env MIMIC_SPREAD_OWN=0: never).  Every generic load / store of such a program set must go
 * through a base the analysis can place (derived from R1, R10 or a packet pointer), else the set runs
 * one lane per vCPU.  (mimic_sync / mimic_last_steps would fail if a spread launch still reached
 * per-CPU memory outside a fused increment: an internal assertion.) */
int mimic_set_spread(mimic_vm *vm, int32_t mode);
/* The kernel the last batch ran on (a JIT VM runs batches whose step budget is below its
 * loop-free kernels' step bound on the interpreter). */
int mimic_last_exec(const mimic_vm *vm);
/* JIT diagnostics (host only, no device): the kernel source generated for raw programs, and a
 * hipRTC compile check of a source for gfx950. */
long mimic_jit_source_for(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, char *buf, size_t cap);
int mimic_jit_check(const char *src, char *log, size_t cap, size_t *code_size);
/* Compile the JIT kernel of raw programs into the MIMIC_JIT_CACHE directory (host only). */
int mimic_jit_prebuild(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs);
/* The same for the kernel of a batch context (MIMIC_CTX_XDP / MIMIC_CTX_SKB). */
long mimic_jit_source_for_ctx(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind,
                              char *buf, size_t cap);
int mimic_jit_prebuild_ctx(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind);
/* The kernel source a VM generates when some LD_IMM64 slots name a per-CPU array whose per-vCPU
 * row is at most 128 bytes, a multiple of 8 (the lane value cache, jit.cpp analyze_vc: rows up to
 * 32 bytes in registers, longer ones in LDS): vc_slots holds n_vc (program index, slot, E * S)
 * triples.  mimic_jit_source_for_ctx is this with n_vc = 0. */
long mimic_jit_source_vc(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, int32_t ctx_kind,
                         const uint32_t *vc_slots, uint32_t n_vc, char *buf, size_t cap);
/* The spread kernel's source (mimic_set_spread): pc = (program, slot, map id) triples of the
 * LD_IMM64 slots naming a per-CPU array's object, shapes = (map id, E * S, S) triples, lds_rows =
 * rows of a block's LDS counter table (min(1024, V) when rows * E * S <= 32 KiB, else 0); bit 31 of
 * lds_rows set: the owned form's source (its rows: min(256, 32 KiB / (E * S))).
 * *spread_out = 1 when the programs allow a spread kernel. */
long mimic_jit_source_spread(const void *const *progs, const uint32_t *n_slots, uint32_t n_progs, const uint32_t *pc,
                             uint32_t n_pc, const uint32_t *shapes, uint32_t n_shapes, uint32_t lds_rows,
                             int32_t *spread_out, char *buf, size_t cap);
/* Compile a kernel source (as mimic_jit_source_for_ctx returns it) into the MIMIC_JIT_CACHE
 * directory (host only; a no-op when it is already there).  Lets a test session or a deploy
 * step build many kernels in parallel processes before any device is touched. */
int mimic_jit_cache_source(const char *src);
/* hipRTC-compile a source and copy the gfx950 code object (an ELF whose AMDGPU metadata note
 * holds the kernel's register, scratch and LDS usage) into code (when it fits); its size in
 * *code_size.  Host only. */
int mimic_jit_code(const char *src, void *code, size_t cap, size_t *code_size);

#ifdef __cplusplus
}
#endif
#endif
