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
#include <cstdlib>

#include "runtime.h"
// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
// Process.Step: save the process at the end of a launch (suspended by the step budget, or done)
static_assert(sizeof(Lane) <= sizeof(((StepState *)0)->lane), "StepState::lane too small");
static __device__ void step_save(const KParams &kp, const Lane &L, const uint64_t *RB, int st, int32_t pc, uint32_t steps,
                                 uint32_t prog) {
    StepState *S = kp.step;
    for (int q = 0; q < 11; q++) S->r[q] = RB[q * 64];
    __builtin_memcpy(S->lane, &L, sizeof(Lane));
    S->pc = pc;
    S->prog = prog;
    S->steps = steps;
    S->status = st;
    S->started = 1;
    S->finished = st != MIMIC_ERR_STEP_LIMIT;
}

#define WAVES_PER_BLOCK 4

// Process.Step / Run launch one lane: its instruction fetches, segment / map table reads and its
// packet loads would each be a cold HBM round trip in sequence (the single-lane Run of a 36-slot
// program measured ~30 us of kernel time).  The block's three idle waves touch one dword of every
// 64-byte line of those tables and of the process's descriptor and packet memory first, so the
// lane's fetches find them in L2.  (Volatile loads: nothing is done with the values.)
static __device__ __noinline__ void step_warm(const KParams &kp, uint32_t t, uint32_t nt) {
    const DProg last = kp.progs[kp.nprogs - 1];
    const uint64_t spans[5][2] = {{(uint64_t)(uintptr_t)kp.insns, (uint64_t)(last.base + last.n) * sizeof(DInsn)},
                                  {(uint64_t)(uintptr_t)kp.segs, (uint64_t)kp.nsegs * sizeof(Seg)},
                                  {(uint64_t)(uintptr_t)kp.maps, (uint64_t)kp.nmaps * sizeof(DMap)},
                                  {(uint64_t)(uintptr_t)kp.progs, (uint64_t)kp.nprogs * sizeof(DProg)},
                                  {(uint64_t)(uintptr_t)kp.pkt_data, 512}};
    uint32_t n = 0;
    for (int k = 0; k < 5; k++) {
        const uint64_t lines = (spans[k][1] + 63) / 64;
        for (uint64_t q = t; q < lines && q < 4096; q += nt) n += *(const volatile uint32_t *)(spans[k][0] + q * 64);
    }
    if (t == 0) n += *(const volatile uint32_t *)kp.pkt_off + *(const volatile uint32_t *)kp.pkt_len;
    (void)n;
}
#define NREGS 11
#define KEY_DONE 0xffffffffu

// The batch kernel, the Process.Step kernel and the resume kernel are one body: MODE compiles
// the step-state paths (restore a suspended process, save it at the end) and the resume paths
// (a process a JIT lane deferred, then the lane's remaining packets) in or out, so the batch
// kernel carries none of their registers (146 -> the batch kernel's own budget, 3 -> 4 waves per
// SIMD).
enum { MODE_BATCH = 0, MODE_STEP = 1, MODE_RESUME = 2 };
template <int MODE>
static __device__ __forceinline__ void xdp_body(const KParams *__restrict__ kpp, uint32_t goff = 0) {
    const KParams &kp = *kpp;  // device copy (engine.cpp kp_slot) or the kernarg segment: fields load where used
    StepState *const STP = MODE == MODE_STEP ? kp.step : nullptr;
    // eBPF registers r0..r10 of every lane live in LDS, [wave][reg][lane] (8-byte words): a
    // wave-uniform register number addresses 64 consecutive words (conflict-free ds_read_b64),
    // and multi-register updates (exit, helpers) need no register-array copies.
    __shared__ uint64_t sreg[WAVES_PER_BLOCK][NREGS][64];
    uint64_t *const RB = &sreg[threadIdx.x >> 6][0][threadIdx.x & 63];
#define REG(r) RB[(r) * 64]

    const uint32_t g = goff + blockIdx.x * blockDim.x + threadIdx.x;
    // resume: only the lanes the JIT kernel deferred in this launch (defer_finish, runtime.h) run,
    // from iteration j0 on; a wave without one returns at once
    const DeferRec *DR = nullptr;
    uint32_t j0 = 0;
    if (MODE == MODE_RESUME) {
        if (*kp.defer_any != kp.defer_epoch) return;
        if (g < kp.lanes && kp.defer[g].flag == kp.defer_epoch) {
            DR = kp.defer + g;
            j0 = DR->j;
        }
        if (__ballot(DR != nullptr) == 0) return;
    }
    const bool lane_valid = g < kp.lanes && (MODE != MODE_RESUME || DR);
    // Process.Step / Run: the first launch of a process copies its NewProcess image (pinned host
    // memory) into its device block, 16 bytes per thread and round; the first step_ins_n slots go to
    // LDS (one round trip for all, then LDS reads instead of a cold scalar fetch per instruction)
    extern __shared__ DInsn step_ins_[];
    if (MODE == MODE_STEP) {
        if (kp.step_img) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const uint32_t nq = kp.step_img_n >> 4;
            for (uint32_t q = threadIdx.x; q < nq; q += blockDim.x)
                ((u32x4 *)kp.step_dst)[q] = ((const u32x4 *)kp.step_img)[q];
            for (uint32_t b = (nq << 4) + threadIdx.x; b < kp.step_img_n; b += blockDim.x) kp.step_dst[b] = kp.step_img[b];
        }
        for (uint32_t q = threadIdx.x; q < kp.step_ins_n; q += blockDim.x) step_ins_[q] = kp.insns[q];
        __syncthreads();
        if (threadIdx.x >= 64) step_warm(kp, threadIdx.x - 64, blockDim.x - 64);
    }
    Lane L;
    L.lane = g;
    L.cpu = STP ? STP->cpu : lane_cpu(kp, g);

    uint32_t ex_begin = 0, ex_count = 0;
    if (lane_valid && kp.sched == SCHED_EXPLICIT) {
        ex_begin = kp.sched_start[g];
        ex_count = kp.sched_start[g + 1] - ex_begin;
    }
    uint64_t lane_steps = MODE == MODE_RESUME && DR ? DR->lane_steps : 0;
    const DProg entry = cget(kp.progs, kp.entry_prog);
    const uint32_t P = kp.static_next + kp.stack_size + 1;

    for (uint32_t j = 0; j < kp.per_lane; j++) {
        // ---- which packet does this lane run in iteration j -----------------------------
        uint32_t i = 0xffffffffu;
        if (lane_valid && (MODE != MODE_RESUME || j >= j0)) {
            if (kp.sched == SCHED_CHUNKED) {
                uint64_t ii = (uint64_t)g * kp.per_lane + j;
                if (ii < kp.n) i = (uint32_t)ii;
            } else if (kp.sched == SCHED_INTERLEAVED) {
                uint64_t ii = (uint64_t)j * kp.lanes + (g >= kp.sched_shift ? g - kp.sched_shift : g + kp.lanes - kp.sched_shift);
                if (ii < kp.n) i = (uint32_t)ii;
            } else if (j < ex_count) {
                i = kp.sched_pkts[ex_begin + j];
            }
        }

        // ---- NewProcess + LinuxContextXDP.Load --------------------------------------------
#pragma unroll
        for (int q = 0; q < NREGS; q++) REG(q) = 0;
        uint32_t pn = entry.n, pbase = entry.base;
        uint32_t cur_prog = kp.entry_prog;
        uint32_t key = KEY_DONE;   // global instruction index = pbase + PC; KEY_DONE = not running
        uint32_t steps = 0;
        L.sm0 = 0;
        L.sm1 = 0;
        L.xdp_dirty = 0;
        L.t_n = 0;
        L.t_lo = 0;
        L.t_ptr = nullptr;
        L.nframes = 0;
        L.tailcalls = 0;
        L.M = 0;
        L.pkt = nullptr;
        L.rec = nullptr;
        L.pa = P;
        L.ka = 0;
        // a process ends here: results straight to HBM (Run's return + p.Registers.R0)
#define TERM(st_, epc_)                                                \
        do {                                                           \
            if (kp.r0) kp.r0[i] = REG(0);                              \
            if (kp.status) kp.status[i] = (uint8_t)(st_);              \
            if (kp.steps) kp.steps[i] = steps;                         \
            if (kp.err_pc) kp.err_pc[i] = (int32_t)(epc_);             \
            lane_steps += steps;                                       \
            key = KEY_DONE;                                            \
            if (STP) step_save(kp, L, RB, (st_), (epc_), steps, cur_prog); \
        } while (0)
        // Process.Step: a stepped process resumes where its last launch suspended it
        bool resumed = false, foreign = false;
        if (i != 0xffffffffu && STP && STP->gen != kp.step_gen) {
            // engine assertion: the state is not this process's -- nothing of it is read or written
            foreign = true;
            if (kp.r0) kp.r0[i] = 0;
            if (kp.status) kp.status[i] = (uint8_t)MIMIC_ERR_ENGINE_STATE;
            if (kp.steps) kp.steps[i] = 0;
            if (kp.err_pc) kp.err_pc[i] = -1;
        } else if (i != 0xffffffffu && STP && STP->started) {
            const StepState *S = STP;
#pragma unroll
            for (int q = 0; q < NREGS; q++) REG(q) = S->r[q];
            __builtin_memcpy(&L, S->lane, sizeof(Lane));
            L.cpu = S->cpu;           // SetCPUID may have moved the process between steps
            steps = S->steps;
            cur_prog = S->prog;
            const DProg cp = kp.progs[cur_prog];
            pn = cp.n;
            pbase = cp.base;
            resumed = true;
            if (S->pc < 0) {          // a jump left PC negative: this Step panics on the fetch (vm.go:300)
                steps++;
                TERM(MIMIC_PANIC_PC, S->pc);
            } else {
                key = pbase + (uint32_t)S->pc;
            }
        }
        // resume: the process the JIT lane deferred (packet i, iteration j0) is attached to its
        // packet again without Load's side effects (the room bytes keep what it wrote), then its
        // registers and dynamic lane state come back and its slot runs next
        const bool resume_here = MODE == MODE_RESUME && i != 0xffffffffu && j == j0;
        if (resumed || foreign) {
        } else if (i != 0xffffffffu && kp.ctx_kind == CTX_SKB) {   // LinuxContextSKBuff.Load (skb.h)
            uint64_t r1 = 0;
            const int ls = skb_load<MODE == MODE_RESUME>(kp, L, i, r1, resume_here);
            REG(10) = kp.static_next + kp.frame_size;
            if (ls) {
                TERM(ls, -1);
            } else {
                REG(1) = r1;
                key = pbase;
                if (pn == 0) {
                    steps = 1;
                    TERM(MIMIC_ERR_PC_OOB, 0);
                }
            }
        } else if (i != 0xffffffffu) {
            const uint32_t H = kp.headroom_arr ? kp.headroom_arr[i] : kp.headroom;
            const uint32_t T = kp.tailroom_arr ? kp.tailroom_arr[i] : kp.tailroom;
            const uint32_t len = kp.pkt_len[i];
            L.pkt = kp.pkt_data + kp.pkt_off[i];
            L.M = H + len + T;
            if (!resume_here) {
                for (uint32_t b = 0; b < H; b++) L.pkt[b] = 0;
                for (uint32_t b = 0; b < T; b++) L.pkt[H + len + b] = 0;
            }
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

        if (resume_here) {
#pragma unroll
            for (int q = 0; q < NREGS; q++) REG(q) = DR->r[q];
            L.sm0 = DR->sm0;
            L.sm1 = DR->sm1;
            L.xdp_dirty = DR->xdp_dirty;
            L.nframes = DR->nframes;
            L.tailcalls = DR->tailcalls;
            steps = DR->steps;
            cur_prog = DR->prog;
            const DProg cp = kp.progs[cur_prog];
            pn = cp.n;
            pbase = cp.base;
            key = pbase + (uint32_t)DR->pc;
            resumed = true;
        }

        // ---- Process.Run ------------------------------------------------------------------
        // Run(ctx): a context already done before the first step ends the process there
        // (vm.go:344-349).  A stepped process's context is checked by the host between launches.
        if (MODE != MODE_STEP && kp.cancel_any && !resumed && key != KEY_DONE) {
            const uint32_t cz = ctx_done(kp, i);
            if (cz) TERM(MIMIC_ERR_CANCELED - 1 + (int)cz, (int32_t)(key - pbase));
        }
        uint64_t wsteps = resumed ? steps : 0;   // wave-steps since the packets started: bounds every lane's steps
        uint32_t cand = KEY_DONE;     // speculated next key (where the first executing lane went)
        for (;;) {
            // Run(ctx) while the process runs: every 4096 wave-steps each running lane reads its
            // context again and stops before its next step once it is done (vm.go:344-349)
            if (MODE != MODE_STEP && kp.cancel_any && (wsteps & 4095u) == 4095u && key != KEY_DONE) {
                const uint32_t cz = ctx_done(kp, i);
                if (cz) TERM(MIMIC_ERR_CANCELED - 1 + (int)cz, (int32_t)(key - pbase));
            }
            uint32_t kw;
            uint64_t act;
            if (MODE == MODE_STEP) {
                // one process, on lane 0 of wave 0: no min-PC scheduling (the other lanes are done)
                kw = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
                if (kw == KEY_DONE) break;
                act = 1;
            } else {
                const uint64_t live = __ballot(key != KEY_DONE);
                if (live == 0) break;
                if (cand != KEY_DONE && (__ballot(key != cand) & live) == 0) kw = cand;  // converged
                else kw = wave_min(key);                                                 // min-PC
                kw = (uint32_t)__builtin_amdgcn_readfirstlane((int)kw);
                act = __ballot(key == kw);
            }
            const DInsn in = MODE == MODE_STEP && kw < kp.step_ins_n ? step_ins_[kw] : cget(kp.insns, kw);    // scalar loads
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
                        HelperOut ho = {0, 0, false, false, 0, 0, 0, nullptr};
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
                            if (ho.t_n) { L.t_lo = ho.t_lo; L.t_n = ho.t_n; L.t_ptr = ho.t_ptr; }
                            if (ho.tail) {  // PC = -1, then Step's bounds check on the new program
                                const DProg np = kp.progs[ho.new_prog];
                                L.tailcalls++;
                                cur_prog = ho.new_prog;
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
                    case H_LDABS: {  // emulator_linux_.go:198-288
                        const bool ind = (aux & AUX_X) != 0;
                        const uint32_t x = (uint32_t)k + (ind ? (uint32_t)REG(src < NREGS ? src : 10) : 0u);
                        uint64_t v = 0;
                        st = ld_abs(kp, L, REG(6), x, AUX_SZ(aux), ind && src > 10, v);
                        if (!st) {
                            REG(0) = v;
#pragma unroll
                            for (int q = 1; q <= 5; q++) REG(q) = 0;
                        }
                        break;
                    }
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
                        TERM(MIMIC_OK, STP ? (int32_t)pc : -1);   // a stepped process keeps PC at the exit
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

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void mimic_xdp_kernel(const KParams *__restrict__ kpp) { xdp_body<MODE_BATCH>(kpp); }
// the same body at the compiler's own budget (3 waves per SIMD, no spills): MIMIC_INTERP_WAVES=3
extern "C" __global__ __launch_bounds__(256) void mimic_xdp_kernel_w3(const KParams *__restrict__ kpp) { xdp_body<MODE_BATCH>(kpp); }
// Process.Step / Run: launch parameters by value (no parameter slot, no copy ahead of the launch)
extern "C" __global__ __launch_bounds__(256) void mimic_xdp_step_kernel(const KParams kp_arg) {
    (void)kp_arg;
    const KParams __attribute__((address_space(4))) *k4 =
        (const KParams __attribute__((address_space(4))) *)__builtin_amdgcn_kernarg_segment_ptr();
    xdp_body<MODE_STEP>((const KParams *)k4);
}
// after a JIT kernel with deferred slow paths, with the same launch parameters (by value: read
// in place from the kernarg segment, as the JIT kernels do)
// (a small grid striding over the lanes: a launch that deferred nothing -- the usual case, checked
// first by every wave -- then costs a few waves instead of one per 64 lanes; cfg 5: 4.3 us)
#define RESUME_BLOCKS 64u
extern "C" __global__ __launch_bounds__(256) void mimic_xdp_resume_kernel(const KParams kp_arg) {
    (void)kp_arg;
    const KParams __attribute__((address_space(4))) *k4 =
        (const KParams __attribute__((address_space(4))) *)__builtin_amdgcn_kernarg_segment_ptr();
    const KParams *kp = (const KParams *)k4;
    const uint32_t lanes = kp->lanes, stride = gridDim.x * blockDim.x;
    for (uint32_t off = 0; off < lanes; off += stride) xdp_body<MODE_RESUME>(kp, off);
}

// Sum of a per-CPU u64 array over cpus: out[k] = sum_c base[c*stride + 8k] (the "sum over CPUs"
// readout of a per-CPU counter map).  The per-CPU backings are contiguous ([cpu][key], stride =
// E*8), so the values form one flat u64 array: for E <= 256 every thread walks it with a stride
// that is a multiple of E, so it always adds the same key; the block reduces per key in LDS and
// adds one partial per key to out (out is zeroed first).  For larger E a thread owns a key and
// walks the cpus (consecutive threads read consecutive keys of a cpu).  No contended
// per-element atomics: at most one atomic per (block, key).
#define SUM_THREADS 256
extern "C" __global__ __launch_bounds__(SUM_THREADS) void mimic_sum_u64_kernel(const uint64_t *base, uint64_t stride_q,
                                                                              uint32_t nvals, uint32_t cpus,
                                                                              uint64_t *out) {
    __shared__ uint64_t part[SUM_THREADS];
    const uint32_t t = threadIdx.x;
    if (nvals <= SUM_THREADS && stride_q == nvals) {
        const uint32_t per = SUM_THREADS / nvals * nvals;          // threads of a block that take part
        const uint64_t total = (uint64_t)cpus * nvals;
        const uint64_t step = (uint64_t)gridDim.x * per;
        uint64_t acc = 0;
        if (t < per)
            for (uint64_t i = (uint64_t)blockIdx.x * per + t; i < total; i += step) acc += *gp(base + i);
        part[t] = acc;
        __syncthreads();
        if (t < nvals) {
            uint64_t s = 0;
            for (uint32_t j = t; j < per; j += nvals) s += part[j];
            atomicAdd((unsigned long long *)&out[t], (unsigned long long)s);
        }
        return;
    }
    // one thread per key, cpus walked in groups (blockIdx.y): strided backings, large E
    const uint32_t k = blockIdx.x * SUM_THREADS + t;
    if (k >= nvals) return;
    const uint32_t groups = gridDim.y;
    uint64_t acc = 0;
    for (uint32_t c = blockIdx.y; c < cpus; c += groups) acc += *gp(base + (uint64_t)c * stride_q + k);
    atomicAdd((unsigned long long *)&out[k], (unsigned long long)acc);
}

// One host-side hash-map operation (mimic_map_update/lookup/delete), run by the same device code
// the helpers use so that both sides share the index and the freelist.
// Host map writes staged by engine.cpp (stage_write / flush_host): entry k copies lens[k] bytes
// from data + at[k] to arena + offs[k] (the host deduplicated the offsets: no two entries overlap)
extern "C" __global__ void mimic_scatter_kernel(uint8_t *arena, const uint64_t *offs, const uint32_t *lens,
                                                const uint32_t *at, const uint8_t *data, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint8_t *d = arena + offs[k];
    const uint8_t *s = data + at[k];
    for (uint32_t b = 0; b < lens[k]; b++) d[b] = s[b];
}

// Tombstone compaction: when live + deleted buckets pass 3/4 of the table, rebuild it in
// place (one workgroup; launched before every batch, returns at once otherwise).
extern "C" __global__ __launch_bounds__(1024) void mimic_hash_rebuild_kernel(uint8_t *arena, DMap m, uint32_t force) {
    __shared__ uint32_t go, live;
    const HT t = h_table(arena, m);
    HashCtl *c = h_ctl(t);
    if (threadIdx.x == 0) {
        go = force || (uint64_t)h_used_total(c) * 4 > (uint64_t)m.ht_cap * 3;
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
    if (threadIdx.x == 0) {
        c->used0 = live;
        for (uint32_t sh = 0; sh < HT_USED_SHARDS; sh++) c->used_sh[32 * sh] = 0;
    }
}

// After a pop-only launch (hashmap.h h_insert_wave): head back to at most tail, avail = what is
// left between them -- the state the pops would have left with the semaphore.
extern "C" __global__ void mimic_hash_normalize_kernel(uint8_t *arena, DMap m) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    HashCtl *c = h_ctl(h_table(arena, m));
    const unsigned long long tl = c->tail, hd = c->head < tl ? c->head : tl;
    c->head = hd;
    c->avail = (int32_t)(tl - hd);
}

// After a launch whose chunk map took its freelist positions in per-block chunks (hashmap.h
// MIMIC_HASH_CHUNK): the holes the blocks' chunk remainders left below head are filled with the
// entries above them, so that the used slots are [0, m) again and ring positions [0, m) popped --
// the state m sequential pops leave (emulator_linux_map_hash.go:179-186).  The launch's inserts set
// used bytes (h_used8) in [lo, hi), lo = the lowest position a block reserved, hi = min(head, E); below lo
// every slot is live.  m = lo + inserts; movers = used slots >= m, holes = free slots in [lo, m); the
// r-th mover (slot order) goes to the r-th hole: key and value bytes copied, the source zeroed (a
// slot never popped holds zeros -- nothing was ever pushed, the ring is the identity), the state
// word of its bucket (h_s2b) rewritten.  Every block turns the bit words (<= 8192: E <= 2^18) into
// LDS prefix counts and moves its share of the movers; the last block to finish clears the bits and
// the handed-back remainders, pops ring positions [lo, m) and resets the counters.  A launch that
// reserved no chunk returns at once.
#define HC_MAXW (HT_CHUNK_MAXE / 32u)
static __device__ uint32_t hc_select(uint32_t x, uint32_t n) {   // bit index of x's n-th set bit
    for (uint32_t q = 0; q < n; q++) x &= x - 1u;
    return (uint32_t)__builtin_ctz(x);
}
// n bytes from slot s to slot d of a backing with stride n, the source zeroed: 8-, 4- or 1-byte units
static __device__ void hc_copy(uint8_t *base, uint32_t n, uint32_t s, uint32_t d) {
    uint8_t *src = base + (size_t)s * n, *dst = base + (size_t)d * n;
    if (!(((uintptr_t)base | n) & 7u)) {
        for (uint32_t b = 0; b < n; b += 8) {
            *(uint64_t *)(dst + b) = *(const uint64_t *)(src + b);
            *(uint64_t *)(src + b) = 0;
        }
    } else if (!(((uintptr_t)base | n) & 3u)) {
        for (uint32_t b = 0; b < n; b += 4) {
            *(uint32_t *)(dst + b) = *(const uint32_t *)(src + b);
            *(uint32_t *)(src + b) = 0;
        }
    } else {
        for (uint32_t b = 0; b < n; b++) {
            dst[b] = src[b];
            src[b] = 0;
        }
    }
}
#define HC_T 1024u   // threads per block
extern "C" __global__ __launch_bounds__(HC_T) void mimic_hash_compact_kernel(uint8_t *arena, DMap m, uint32_t meas) {
    const HT t = h_table(arena, m);
    HashCtl *c = h_ctl(t);
    const uint32_t cminv = c->cminv, fullf = c->full;
    if (!cminv && !fullf) return;
    __shared__ uint32_t wd[HC_MAXW], pf[HC_MAXW];   // the bit words of [lo, hi); set bits in words [0, i)
    __shared__ uint32_t wsum[HC_T / 64], total_, last_;
    const uint32_t E = t.E;
    const unsigned long long hd = c->head;
    const uint32_t hi = hd < E ? (uint32_t)hd : E;
    uint32_t lo = cminv ? 0xffffffffu - cminv : hi;
    lo = lo < hi ? lo : hi;
    const uint32_t w0 = lo >> 5, nw = (meas & 8u) ? 0u : ((hi + 31u) >> 5) - w0;
    const uint8_t *used = h_used8(t);
    // the used bytes as bit words (plain loads: the launch that wrote them has ended), below lo
    // counted as used, from hi on as free.  Every load of the thread first (indices clamped, no
    // branch between them: one wait), then the packing (a loop of load-then-use waited per word)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr uint32_t PW = HC_MAXW / HC_T;   // words per thread (4: eight 16-byte loads in flight)
    u32x4 v[2 * PW];
#pragma unroll
    for (uint32_t k = 0; k < PW; k++) {
        const uint32_t i = threadIdx.x + HC_T * k, ic = i < nw ? i : 0u;
        const u32x4 *q = (const u32x4 *)(used + ((size_t)(w0 + ic) << 5));
        v[2 * k] = q[0];
        v[2 * k + 1] = q[1];
    }
#pragma unroll
    for (uint32_t k = 0; k < PW; k++) {
        const uint32_t i = threadIdx.x + HC_T * k;
        if (i >= nw) break;
        uint32_t x = 0;
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const u32x4 u = v[2 * k + h];
            const uint32_t d[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (uint32_t c = 0; c < 16; c++) x |= ((d[c >> 2] >> (8 * (c & 3))) & 1u) << (16 * h + c);
        }
        const uint32_t b0 = (w0 + i) << 5;
        if (b0 < lo) x |= (1u << (lo - b0)) - 1u;   // (word 0 only: lo - b0 in 1..31)
        if (b0 + 32u > hi) x &= hi > b0 ? (1u << (hi - b0)) - 1u : 0u;
        wd[i] = x;
    }
    __syncthreads();
    // exclusive prefix counts: thread t sums words [t * per, +per), the threads' sums are scanned
    const uint32_t per = (nw + HC_T - 1u) / HC_T, beg = threadIdx.x * per;
    uint32_t own = 0;
    for (uint32_t i = beg; i < beg + per && i < nw; i++) own += (uint32_t)__builtin_popcount(wd[i]);
    uint32_t inc = own;   // inclusive scan over the wave
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (__lane_id() >= o) inc += y;
    }
    if (__lane_id() == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t before = inc - own;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) before += wsum[w];
    if (threadIdx.x == HC_T - 1u) total_ = before + own;
    for (uint32_t i = beg; i < beg + per && i < nw; i++) {
        pf[i] = before;
        before += (uint32_t)__builtin_popcount(wd[i]);
    }
    __syncthreads();
    const uint32_t T = total_, mm = (w0 << 5) + T;   // m: the used slots after the moves are [0, m)
    const uint32_t mw = (mm >> 5) - w0, mb = mm & 31u;
    const uint32_t Sm = (mw < nw ? pf[mw] : T) + (mw < nw && mb ? (uint32_t)__builtin_popcount(wd[mw] & ((1u << mb) - 1u)) : 0u);
    const uint32_t H = T - Sm;   // movers = holes
    uint8_t *kb = arena + m.keys_dev_off, *vb = arena + m.dev_off;
    for (uint32_t r = blockIdx.x * HC_T + threadIdx.x; r < ((meas & 1u) ? 0u : H); r += gridDim.x * HC_T) {
        // the mover: the (Sm + r)-th used slot; the hole: the r-th free slot (zeros before word i: 32 i - pf[i])
        const uint32_t j = Sm + r;
        uint32_t a = 0, b = nw;   // the last word with pf <= j
        while (b - a > 1) {
            const uint32_t h = (a + b) >> 1;
            if (pf[h] <= j) a = h; else b = h;
        }
        const uint32_t sl = ((w0 + a) << 5) + hc_select(wd[a], j - pf[a]);
        a = 0;
        b = nw;
        while (b - a > 1) {
            const uint32_t h = (a + b) >> 1;
            if (32u * h - pf[h] <= r) a = h; else b = h;
        }
        const uint32_t d = ((w0 + a) << 5) + hc_select(~wd[a], r - (32u * a - pf[a]));
        const uint32_t p = h_s2b(t)[sl];   // the mover's bucket
        hc_copy(kb, m.key_size, sl, d);
        hc_copy(vb, m.value_size, sl, d);
        *(uint32_t *)h_rec(t, p) = d;   // the state half of the bucket's first word (the tag stays)
    }
    // ring positions [lo, m) popped (every block a share: nothing in this kernel reads the ring)
    int32_t *ring = h_ring(t);
    for (uint32_t q = lo + blockIdx.x * HC_T + threadIdx.x; q < ((meas & 2u) ? lo : mm); q += gridDim.x * HC_T) ring[q] = -1;
    // The last block to get here clears what every block has read (their reads are complete: each
    // block used the values before counting itself).  No fence: nothing written here is read back in
    // this kernel, and the kernel's end publishes it (a release fence per block -- an L2 write-back
    // on gfx950 -- cost 10 of this kernel's 19 us)
    __syncthreads();
    if (threadIdx.x == 0)
        last_ = __hip_atomic_fetch_add(&c->cdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    __syncthreads();
    if (!last_) return;
    typedef uint32_t u32x4z __attribute__((ext_vector_type(4)));
    u32x4z *uz = (u32x4z *)(h_used8(t) + ((size_t)w0 << 5));
    const u32x4z z4 = {0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < ((meas & 4u) ? 0u : 2 * nw); i += HC_T) uz[i] = z4;
    unsigned long long *left = h_left(t);
    const uint32_t nl = c->nleft < HT_LEFT_CAP ? c->nleft : HT_LEFT_CAP;
    for (uint32_t q = threadIdx.x; q < nl; q += HC_T) left[q] = 0;
    if (threadIdx.x < HT_USED_SHARDS) c->live_sh[32 * threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        c->head = mm;
        c->avail = (int32_t)(E - mm);
        c->cminv = 0;
        c->full = 0;
        c->cdone = 0;
        c->nleft = 0;
    }
}

extern "C" int mimic_launch_hash_compact(uint8_t *arena, const DMap *m, hipStream_t st) {
    // every block scans all bit words (<= 4096), then takes a share of the movers: about a mover per
    // thread (MIMIC_COMPACT_BLOCKS=n: n blocks, measurement)
    static const uint32_t forced = [] { const char *e = getenv("MIMIC_COMPACT_BLOCKS"); return e ? (uint32_t)atoi(e) : 0u; }();
    const uint32_t blocks = forced ? forced : std::min<uint32_t>(64u, std::max<uint32_t>(1u, m->max_entries / 4096u));
    // MIMIC_COMPACT_MEAS (measurement only, results wrong): 1 no moves, 2 no ring writes, 4 no clearing
    // of the used bytes, 8 no scan (nothing found)
    static const uint32_t meas = [] { const char *e = getenv("MIMIC_COMPACT_MEAS"); return e ? (uint32_t)atoi(e) : 0u; }();
    hipLaunchKernelGGL(mimic_hash_compact_kernel, dim3(blocks), dim3(HC_T), 0, st, arena, *m, meas);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_hash_normalize(uint8_t *arena, const DMap *m, hipStream_t st) {
    hipLaunchKernelGGL(mimic_hash_normalize_kernel, dim3(1), dim3(64), 0, st, arena, *m);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A hash map's index back to its NewLinuxHashMap state (emulator_linux_map_hash.go:56-64): every
// bucket EMPTY, every stripe lock free, the freelist ring 0..E-1, head 0 / tail E / avail E.
// n bytes at p set to byte b: 16-byte stores for the aligned middle, byte stores at the ends
static __device__ void fill_bytes(uint8_t *p, size_t n, uint8_t b, size_t g, size_t stride) {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    const size_t head = (16 - ((uintptr_t)p & 15)) & 15, h = head < n ? head : n;
    for (size_t i = g; i < h; i += stride) p[i] = b;
    const size_t n16 = (n - h) / 16;
    const uint64_t w = 0x0101010101010101ull * b;
    const u64x2 v = {w, w};
    u64x2 *q = (u64x2 *)(p + h);
    for (size_t i = g; i < n16; i += stride) q[i] = v;
    for (size_t i = h + 16 * n16 + g; i < n; i += stride) p[i] = b;
}
// A fresh map in place (mimic_map_reset): its values and keys backings zeroed, every bucket EMPTY,
// the ring 0..E-1, the counters of a new map -- one launch (round 3: two memsets
// and an 8-byte-store kernel, 18 us per reset of cfg 4's table).
extern "C" __global__ void mimic_hash_reset_kernel(uint8_t *arena, DMap m) {
    const HT t = h_table(arena, m);
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    fill_bytes(t.base, h_rec_bytes(t), 0xff, g, stride);
    // (the stripe locks are not touched: every lock a launch or host operation takes is released
    // before it ends, so between launches they are all free already: 8 MB of cfg 4's 26 MB reset)
    fill_bytes(arena + m.dev_off, (size_t)m.dev_stride * m.ncpu, 0, g, stride);
    fill_bytes(arena + m.keys_dev_off, (size_t)m.max_entries * m.key_size, 0, g, stride);
    int32_t *ring = h_ring(t);
    for (size_t i = g; i < t.fl_cap; i += stride) ring[i] = i < m.max_entries ? (int32_t)i : -1;
    // chunked reservations' used bytes and handed-back remainders (hashmap.h h_used8 / h_left)
    fill_bytes(h_used8(t), h_e32(t), 0, g, stride);
    fill_bytes((uint8_t *)h_left(t), (size_t)HT_LEFT_CAP * 8, 0, g, stride);
    if (g == 0) {
        HashCtl *c = h_ctl(t);
        c->head = 0;
        c->tail = m.max_entries;
        c->avail = (int32_t)m.max_entries;
        c->used0 = 0;
        for (uint32_t sh = 0; sh < HT_USED_SHARDS; sh++) c->used_sh[32 * sh] = c->live_sh[32 * sh] = 0;
        c->cminv = c->full = c->cdone = c->nleft = 0;
    }
}

extern "C" int mimic_launch_hash_reset(uint8_t *arena, const DMap *m, hipStream_t st) {
    const size_t work = std::max<size_t>({(size_t)m->ht_cap * m->rec_q * 8 / 16, (size_t)m->fl_cap,
                                          (size_t)m->dev_stride * m->ncpu / 16});
    const uint32_t blocks = (uint32_t)std::min<size_t>((work + 255) / 256, 4096);
    hipLaunchKernelGGL(mimic_hash_reset_kernel, dim3(blocks), dim3(256), 0, st, arena, *m);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_scatter(uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *at,
                                    const uint8_t *data, uint32_t n, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(mimic_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, st, arena, offs, lens, at, data, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_hash_rebuild(uint8_t *arena, const DMap *m, uint32_t force, hipStream_t st) {
    hipLaunchKernelGGL(mimic_hash_rebuild_kernel, dim3(1), dim3(1024), 0, st, arena, *m, force);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_xdp_resume(const KParams *kp, hipStream_t st) {
    const uint32_t blocks = std::min<uint32_t>((kp->lanes + 255) / 256, RESUME_BLOCKS);
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(mimic_xdp_resume_kernel, dim3(blocks), dim3(256), 0, st, *kp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_xdp(const KParams *kp, const KParams *d_kp, hipStream_t st) {
    const uint32_t blocks = (kp->lanes + 255) / 256;
    if (blocks == 0) return 0;
    static const bool w3 = [] { const char *e = getenv("MIMIC_INTERP_WAVES"); return e && e[0] == '3'; }();
    if (kp->step) hipLaunchKernelGGL(mimic_xdp_step_kernel, dim3(blocks), dim3(256), (size_t)kp->step_ins_n * sizeof(DInsn), st, *kp);
    else if (w3) hipLaunchKernelGGL(mimic_xdp_kernel_w3, dim3(blocks), dim3(256), 0, st, d_kp);
    else hipLaunchKernelGGL(mimic_xdp_kernel, dim3(blocks), dim3(256), 0, st, d_kp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Spread launches whose LDS table covers every vCPU lane (jit.cpp, spread flush): each block left
// its counters in part[block][lane][counter]; thread (w, g) sums counter w over group g's blocks and
// adds the sum into the map with one agent-scope add (groups of blocks, so the reads of a thread are
// independent and few: nblocks / G each).  dst: the map's row of lane 0; lanes `stride` bytes apart.
template <typename T>
__global__ __launch_bounds__(256) void spread_reduce_kernel(const T *__restrict__ part, uint32_t nblocks, uint32_t words,
                                                            uint32_t roww, uint32_t groups, uint8_t *dst, uint64_t stride) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)words * groups) return;
    const uint32_t w = (uint32_t)(t % words), g = (uint32_t)(t / words);
    const uint32_t per = (nblocks + groups - 1) / groups, b0 = g * per, b1 = b0 + per < nblocks ? b0 + per : nblocks;
    T s = 0;
    for (uint32_t b = b0; b < b1; b++) s += part[(size_t)b * words + w];
    if (!s) return;
    const uint32_t lane = w / roww, q = w - lane * roww;
    __hip_atomic_fetch_add((T *)(dst + (size_t)lane * stride) + q, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
extern "C" int mimic_launch_spread_reduce(const void *part, uint32_t nblocks, uint32_t lanes, uint32_t roww, uint32_t n,
                                          uint8_t *dst, uint64_t stride, hipStream_t st) {
    const uint32_t words = lanes * roww;
    if (!words || !nblocks) return 0;
    uint32_t groups = (65536u + words - 1) / words;   // ~64 K threads
    if (groups > nblocks) groups = nblocks;
    const uint64_t threads = (uint64_t)words * groups;
    const dim3 grid((uint32_t)((threads + 255) / 256));
    if (n == 8)
        hipLaunchKernelGGL(spread_reduce_kernel<uint64_t>, grid, dim3(256), 0, st, (const uint64_t *)part, nblocks, words, roww,
                           groups, dst, stride);
    else
        hipLaunchKernelGGL(spread_reduce_kernel<uint32_t>, grid, dim3(256), 0, st, (const uint32_t *)part, nblocks, words, roww,
                           groups, dst, stride);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mimic_launch_sum_u64(const uint8_t *base, uint64_t stride, uint32_t nvals, uint32_t cpus, uint64_t *out,
                                    hipStream_t st) {
    if (hipMemsetAsync(out, 0, (size_t)nvals * 8, st) != hipSuccess) return -1;
    if (!nvals || !cpus) return 0;
    if ((stride & 7) || ((uintptr_t)base & 7)) return -1;
    const uint64_t sq = stride / 8;
    if (nvals <= SUM_THREADS && sq == nvals) {
        const uint64_t total = (uint64_t)cpus * nvals;
        // about 16 values per thread; at most 1024 blocks (= 1024 atomics per key)
        const uint64_t per_block = (uint64_t)(SUM_THREADS / nvals * nvals) * 16;
        const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (total + per_block - 1) / per_block));
        hipLaunchKernelGGL(mimic_sum_u64_kernel, dim3(blocks), dim3(SUM_THREADS), 0, st, (const uint64_t *)base, sq, nvals,
                           cpus, out);
    } else {
        const uint32_t kb = (nvals + SUM_THREADS - 1) / SUM_THREADS;
        const uint32_t groups = std::max<uint32_t>(1, std::min<uint32_t>(cpus, std::max<uint32_t>(1, 2048 / kb)));
        hipLaunchKernelGGL(mimic_sum_u64_kernel, dim3(kb, groups), dim3(SUM_THREADS), 0, st, (const uint64_t *)base, sq,
                           nvals, cpus, out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
