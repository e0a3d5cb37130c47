// jit.h -- per-program-set JIT kernels (jit.cpp): source generation, hipRTC build, launch.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "layout.h"

// HIP source of the kernel that runs the loaded programs (aux = predecoded facts)
struct JitInfo {
    bool checks_budget;  // the kernel has the per-block budget checks (loops / BPF-to-BPF calls)
    uint32_t max_n;      // longest program
    bool tail_calls;     // some program calls bpf_tail_call
    bool early_loads;    // the kernel issues packet loads early (analyze_spec)
    bool cold_inline;    // the slow paths are inlined (small kernel, 4-wave register budget)
    bool karg;           // the kernel takes KParams by value (kernarg segment), not a device copy
    bool defer;          // slow paths are deferred to the interpreter's resume kernel (launch it after)
    bool skb_walk;       // sk_buff kernel that builds its SkbRecs itself (prep: footprints only)
    bool skb_fast;       // sk_buff kernel that derives the records of common frames itself (sparse prep)
    bool spread;         // a spread kernel (a vCPU's packets on many lanes; jit.cpp analyze_spread)
    bool spread_own;     // ... in its owned form: a block runs every packet of its vCPUs (SpreadReq::own)
    bool hash_combine;   // pop-only inline inserts through the block combiner (hashmap.h h_comb_reserve)
    bool hash_chunk;     // ... and per-block chunks for the chunk map: mimic_hash_compact_kernel after each launch
    // the single-process form (Process.Run, engine.cpp process_advance): every exit stores the
    // process's registers, PC, program and steps into KParams::step; proc_ok = usable for it
    // (loop-free, no BPF-to-BPF calls, no deferred slow paths, the exit's program known)
    bool proc, proc_ok;
    // spread kernels: the counted per-CPU array, counter width, counters per row, LDS table rows
    uint32_t spread_map, spread_n, spread_roww, spread_rows;
};
// What a spread kernel may be built for (jit.cpp analyze_spread): the VM's per-CPU arrays.
struct SpreadReq {
    std::map<uint32_t, uint32_t> slot_map;   // kernel-wide LD_IMM64 slot -> per-CPU array map id (its object)
    std::map<uint32_t, std::pair<uint32_t, uint32_t>> shape;   // map id -> (E * S, S)
    uint32_t lds_rows = 0;   // rows of a block's LDS counter table (0: agent-scope atomics into the map)
    uint32_t ppb = 1024;     // packets per block
    // owned form: block b runs all P = KParams::per_lane packets of vCPU lanes [b * 256 / P, +256 / P)
    // (2 <= P <= 256), its counters into an LDS table it then adds into the rows it alone owns
    bool own = false;
};
// ctx_kind: CtxKind of the batches the kernel runs
// ctx_check: the variant for launches given Run(ctx) contexts (KParams::cancel_any)
// proc: the single-process form for Process.Run (JitInfo::proc)
// vc_slots: (kernel-wide index, E * S) of the LD_IMM64 slots whose constant is the object of a
// per-CPU array whose row the lane value cache may hold: E * S a multiple of 8, at most
// MIMIC_VC_MAX_ROW bytes (rows up to 32 bytes in registers, longer ones in LDS)
#define MIMIC_VC_MAX_ROW 128u
std::string mimic_jit_source(const std::vector<DProg> &progs, const std::vector<DInsn> &all, uint32_t ctx_kind,
                             JitInfo *info, const std::vector<std::pair<uint32_t, uint32_t>> *vc_slots = nullptr,
                             bool no_early_loads = false,
                             const SpreadReq *spread = nullptr, bool ctx_check = false, bool proc = false);
// 0 when the kernel checks the budget itself; else the most steps one packet can take -- a
// batch with a smaller budget must run on the interpreter
uint64_t mimic_jit_step_bound(const JitInfo &info, uint32_t max_tail_calls);
// hipRTC compile for gfx950 + module load on the current device (cached per device and source)
int mimic_jit_compile(int device, const std::string &src, hipFunction_t *fn, std::string *log);
// d_kp: the launch parameters in device memory
int mimic_jit_launch(hipFunction_t fn, const JitInfo &info, const KParams *kp, const KParams *d_kp, hipStream_t st);
// hipRTC compile only, no device needed
int mimic_jit_check_source(const std::string &src, std::string *log, size_t *code_size);
// source -> gfx950 code object (through the MIMIC_JIT_CACHE directory when set), no device
int mimic_jit_build_code(const std::string &src, std::vector<char> &code, std::string *log);
// compile into the MIMIC_JIT_CACHE directory without a device (prewarming)
int mimic_jit_prebuild_source(const std::string &src, std::string *log);
