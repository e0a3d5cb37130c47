// jit.cpp -- per-program-set JIT: the loaded eBPF programs become one straight-line HIP
// kernel (compiled with hipRTC for gfx950 at the first run after a program load).
//
// The interpreter (interp.hip) pays for generality on every eBPF step. Each step runs:
//   * a wave-wide minimum-PC reduction;
//   * a scalar instruction fetch;
//   * a dispatch switch;
//   * LDS register traffic.
// Here every instruction of every program is emitted once as HIP statements. Its registers,
// offsets, immediates and opcode are compile-time constants, and r0..r10 are plain 64-bit
// locals (VGPRs). Control flow is `goto` between basic blocks, and the GPU's own
// divergence/reconvergence (EXEC masks) replaces min-PC scheduling. Semantics are those of
// the interpreter, statement for statement: the same runtime.h functions resolve memory, run
// the helpers and compute ALU/jump results, and the same predecoded error facts (layout.h
// aux) decide what each slot does.
//
// Step accounting is exact per lane: `steps++` per instruction. The step budget (Run's
// deadline) is checked once per basic block: a block whose end would exceed the budget is
// executed by a "careful" copy that checks before every instruction.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <unistd.h>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/mimic_amd.h"
#include "layout.h"
#include "jit.h"

namespace {

#include "jit_headers.inc"  // kJitHeaderNames / kJitHeaderSrc / kJitHeaderCount (generated at build)

struct Emitter {
    std::string s;
    void line(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        s += buf;
        s += '\n';
    }
};

struct ProgView {
    uint32_t id, n, base;  // base: first slot in the concatenated instruction table (kp.insns)
    const DInsn *ins;
};

uint32_t insn_op(const DInsn &x) { return x.w & 0xff; }
uint32_t insn_dst(const DInsn &x) { return (x.w >> 8) & 0xf; }
uint32_t insn_src(const DInsn &x) { return (x.w >> 12) & 0xf; }
int32_t insn_off(const DInsn &x) { return (int16_t)(x.w >> 16); }

// does the slot end a basic block (control leaves other than by falling through)?
bool ends_block(const DInsn &x) {
    switch (AUX_H(x.aux)) {
    case H_ERR: case H_JA: case H_JCC: case H_EXIT: case H_CALL_LOCAL: return true;
    case H_CALL: return (uint32_t)x.k == 12;  // a tail call may switch programs
    default: return false;
    }
}

int64_t jump_target(const DInsn &x, int64_t i) {
    return insn_op(x) == 0x85 ? i + (int64_t)(int32_t)(uint32_t)x.k : i + insn_off(x) + 1;
}

class Gen {
  public:
    Gen(const std::vector<ProgView> &progs, uint32_t ctx_kind) : P(progs), ctx(ctx_kind) {
        // tuning knobs (environment; they change the generated source, hence the cache key)
        const char *f = getenv("MIMIC_JIT_FAST");
        fast_paths = !(f && f[0] == '0');
        // MIMIC_JIT_KQ: which once-per-packet KParams fields are read through an opaque pointer
        // (0 none: hoisted into SGPRs; 1 all; 2 the result pointers only).  Measured on MI355X
        // (cfg 2): 0 = 44.6 us per launch, 1 and 2 = 52-54 us -- a scalar load in front of every
        // packet's result stores costs more than the couple of SGPRs spilled into VGPR lanes.
        const char *kq = getenv("MIMIC_JIT_KQ");
        kq_mode = kq ? atoi(kq) : 0;
        // MIMIC_JIT_NT=1: non-temporal packet / descriptor / result accesses.  Measured slower on
        // MI355X (cfg 2: 48 us vs 37 us per launch): a packet is read by several small loads, and
        // evict-first lines make the later ones miss.
        const char *ntv = getenv("MIMIC_JIT_NT");
        nt = ntv && ntv[0] == '1';
        const char *pfv = getenv("MIMIC_JIT_PREFETCH");   // 0: no descriptor prefetch
        prefetch = !(pfv && pfv[0] == '0');
        const char *xv = getenv("MIMIC_JIT_XPF");   // 1: next-packet header window prefetch
        xpf_knob = xv && xv[0] == '1';
        const char *lpv = getenv("MIMIC_JIT_LPF");   // 1: lane-start prefetch of the first packets' windows
        lpf_knob = lpv && lpv[0] == '1';
        const char *hv = getenv("MIMIC_JIT_HINT");   // 1: [[unlikely]] on the slow-path branches (measured: no change)
        hint_knob = hv && hv[0] == '1';
        const char *lq = getenv("MIMIC_JIT_LDSSTK");   // 8-byte words of the LDS stack window (0: none)
        if (lq) lds_stack_q = (uint32_t)std::min(32, std::max(0, atoi(lq)));
        const char *dv = getenv("MIMIC_JIT_DISPATCH");   // 0: a jump table at every tail-call site
        dispatch_knob = !(dv && dv[0] == '0');
        const char *vcv = getenv("MIMIC_JIT_VC");   // 0: no lane value cache
        vc_knob = !(vcv && vcv[0] == '0');
        const char *fw = getenv("MIMIC_JIT_FWD");   // 0: no stack-store -> lookup key forwarding
        forward = !(fw && fw[0] == '0');
        const char *ka = getenv("MIMIC_JIT_KARG");   // 0: launch parameters through a device copy (slots)
        if (ka) karg = atoi(ka);
        const char *nr = getenv("MIMIC_JIT_NTRES");   // 0: per-packet results stored as plain stores
        ntres = !(nr && nr[0] == '0');
        const char *cbv = getenv("MIMIC_JIT_COMBINE");
        combine_knob = !(cbv && cbv[0] == '0');
        const char *hcv = getenv("MIMIC_JIT_HCHUNK");   // 0: no chunked reservations; N: chunks of up to N positions
        if (hcv) hchunk_knob = atoi(hcv);
        const char *dnr = getenv("MIMIC_JIT_DEFER_NOREGS");
        defer_noregs = dnr ? atoi(dnr) : 0;
        const char *sf = getenv("MIMIC_JIT_SKBFIELD");   // 0: sk_buff fields through the generic convertAccess
        skb_fields = !(sf && sf[0] == '0');
        const char *sl = getenv("MIMIC_JIT_SKBLDS");   // 0: sk_buff records read from global memory
        skb_lds_knob = !(sl && sl[0] == '0');
        const char *sw = getenv("MIMIC_JIT_SKBWALK");   // 1: the kernel builds its sk_buff records (measured slower)
        skb_walk_knob = sw && sw[0] == '1';
        const char *sfa = getenv("MIMIC_JIT_SKBFAST");   // 1: common frames' records derived in the kernel
        skb_fast_knob = sfa && sfa[0] == '1';
        const char *stc = getenv("MIMIC_JIT_SKBTOUCH");   // 0: no next-descriptor prefetch / header touch
        skb_touch_knob = stc ? (uint32_t)atoi(stc) : 0u;   // 1: prefetch + touch, 2: the offset prefetch only
        const char *sml = getenv("MIMIC_JIT_SMLDS");
        sm_lds_knob = !(sml && sml[0] == '0');
        const char *ic = getenv("MIMIC_JIT_INC");   // 0: counter increments as three slots
        inc_knob = !(ic && ic[0] == '0');
        const char *hf = getenv("MIMIC_JIT_HASH");   // 0: hash-map lookups always through the generic helper
        hash_fast = !(hf && hf[0] == '0');
        const char *ti = getenv("MIMIC_JIT_TAIL");   // 0: tail calls always through the generic helper
        tail_inline = !(ti && ti[0] == '0');
        const char *ce = getenv("MIMIC_JIT_CENSUS");   // 1: per-packet slow-path call counts in place of steps
        census = ce && ce[0] == '1';
        const char *mt = getenv("MIMIC_JIT_MEMTIME");   // 1: per-packet start / end clocks in place of steps / err_pc
        memtime = mt && mt[0] == '1';
        const char *el = getenv("MIMIC_JIT_ELIDE");   // 0: forwarded key stores are always made
        elide = !(el && el[0] == '0');
        const char *wnd = getenv("MIMIC_JIT_WINDOW");   // 0: early loads one by one
        window = !(wnd && wnd[0] == '0');
        const char *spv = getenv("MIMIC_JIT_SPEC");   // 0: no early packet loads
        if (spv) speculate = atoi(spv);
        const char *wv = getenv("MIMIC_JIT_WAVES");   // minimum waves per SIMD the register budget targets
        if (wv) waves = atoi(wv);
        const char *ol = getenv("MIMIC_JIT_OPAQUE_LANE");
        opaque_lane = ol && ol[0] == '1';
        const char *cm = getenv("MIMIC_JIT_COLD");   // call | inline (default: by kernel size)
        cold_mode = !cm ? 0 : !strcmp(cm, "call") ? 1 : !strcmp(cm, "inline") ? 2 : !strcmp(cm, "defer") ? 3 : 0;
        // MIMIC_JIT_STAGE=1: stage each packet's first 64 bytes in LDS.  Measured slower on MI355X
        // for every config (cfg 2: 74 us vs 37 us, cfg 3: 2.6 ms vs 1.2 ms per launch): the staging
        // waits for all eight qwords before the first use, while direct loads hit L1 / L2 anyway.
        const char *sg = getenv("MIMIC_JIT_STAGE");
        stage = sg && sg[0] == '1';
        for (auto &p : P)
            for (uint32_t i = 0; i < p.n; i++) {
                const DInsn &x = p.ins[i];
                if (AUX_H(x.aux) == H_CALL && (uint32_t)x.k == 12) any_tail = true;
                if (AUX_H(x.aux) == H_CALL_LOCAL) any_local = true;
            }
        // a frame pushed before a tail call returns into the NEW program (the saved PC is an
        // index, vm.go:256-257): then any slot can be a return site
        all_leaders = any_tail && any_local;
        // loop-free programs without BPF-to-BPF calls run at most n steps per program (and at
        // most MaxTailCalls+1 programs): with a budget at least that large, no block needs the
        // careful copy (the engine falls back to the interpreter for smaller budgets)
        bool back = false;
        uint32_t mx = 0;
        for (auto &p : P) {
            mx = std::max(mx, p.n);
            for (uint32_t i = 0; i < p.n; i++) {
                const DInsn &x = p.ins[i];
                const uint32_t h = AUX_H(x.aux);
                if ((h == H_JA || h == H_JCC) && (x.aux & AUX_JT_OK) && jump_target(x, i) <= (int64_t)i) back = true;
            }
        }
        careful_copies = back || any_local;
        max_n = mx;
    }

    bool careful_copies = true;
    uint32_t max_n = 0;
    bool fast_paths = true;    // MIMIC_JIT_FAST=0: every access through resolve()
    int cold_mode = 0;         // MIMIC_JIT_COLD: 0 auto, 1 call, 2 inline, 3 defer
    int kq_mode = 0;           // per-packet KParams fields through an opaque pointer (see MIMIC_JIT_KQ)
    bool opaque_lane = false;  // per-iteration opaque lane index (MIMIC_JIT_OPAQUE_LANE=1)
    bool nt = false;           // MIMIC_JIT_NT=1: streaming accesses non-temporal
    bool skb_fields = true;    // MIMIC_JIT_SKBFIELD=0: no per-field sk_buff access code
    bool skb_lds_knob = true;  // MIMIC_JIT_SKBLDS=0: no LDS copy of the sk_buff record
    bool skb_lds = false;
    // the kernel runs SKBuffFromBytes itself into the LDS slot (skb_load_walk), over a 128-byte
    // header window per thread in LDS: the prep kernel then writes footprints only
    // (MIMIC_JIT_SKBWALK=1; measured slower on MI355X: cfg 5 0.447 -> 0.482 ms per step at
    // V = 128K -- the walk on the chain's critical path costs more than the record round trip)
    bool skb_walk_knob = false;
    bool skb_walk = false;
    // the kernel derives the record of every frame skb_fast takes from the packet's first bytes
    // (skb_load_fast); the prep kernel writes records for the other frames only (sparse prep)
    bool skb_fast_knob = false;   // (measured slower on MI355X: DESIGN.md 6.1)
    bool skb_fast = false;
    // sk_buff kernels (prep records in LDS), MIMIC_JIT_SKBTOUCH=1/2: the next packet's offset is loaded
    // while the current one runs, and (1) a packet's header lines are touched when its record load is
    // issued, so the programs' LD_ABS / direct packet loads find them in L2.  Off: the cfg-5 chain sits
    // at 255 VGPRs, and either form takes it to 256 + 2 AGPRs -- one wave per SIMD, 0.22 -> 0.36 ms
    // (profiles/r05/)
    uint32_t skb_touch_knob = 0;
    bool skb_touch = false;
    bool inc_knob = true;      // MIMIC_JIT_INC=0: no fused counter increments (fusable_inc)
    bool sm_lds_knob = true;   // MIMIC_JIT_SMLDS=0: stack validity masks in VGPRs in defer mode too
    static constexpr uint32_t kSrecQ = 21;   // 8-byte words per LDS record slot (SkbRec is 20)
    int karg = 2;              // MIMIC_JIT_KARG: 2 launch parameters by value in the kernarg segment, read
                               // through an opaque constant-space pointer; 1 the same, plain; 0 a
                               // pointer to a device copy (a copy + event per new batch between kernels)
    bool hash_fast = true;     // MIMIC_JIT_HASH=0: no inline hash-map lookups
    bool tail_inline = true;   // MIMIC_JIT_TAIL=0: no inline tail calls
    bool census = false;       // MIMIC_JIT_CENSUS=1: diagnostics (tools/cold_census.py)
    // MIMIC_JIT_MEMTIME=1 (measurement only, tools/memtime.py): s_memrealtime (100 MHz) when each
    // packet's process starts (err_pc) and when its results are stored (steps)
    bool memtime = false;
    bool elide = true;         // MIMIC_JIT_ELIDE=0: no deferred stack stores
    bool window = true;        // MIMIC_JIT_WINDOW=0: no windowed early loads
    int speculate = 8;         // MIMIC_JIT_SPEC=N: at most N early packet loads per region (0: none)
    int defer_noregs = 0;   // MIMIC_JIT_DEFER_NOREGS=1: deferral sites store no registers, 2: low halves (register census only)
    bool combine_knob = true;  // MIMIC_JIT_COMBINE=0: every wave reserves freelist positions with its own add
    bool hash_combine = false;
    int hchunk_knob = 32;       // MIMIC_JIT_HCHUNK (hashmap.h MIMIC_HCHUNK; 0: off)
    bool hash_chunk = false;    // the chunk map's positions come in per-block chunks (hashmap.h h_chunk_fill)
    bool ntres = true;         // MIMIC_JIT_NTRES=0: r0 / status stores not non-temporal (measured 1-3 % slower)
    bool forward = true;       // MIMIC_JIT_FWD=0: helper-1 keys always reread from the stack
    int waves = 0;             // MIMIC_JIT_WAVES=W: amdgpu_waves_per_eu(W) on the kernel
    bool prefetch = true;      // MIMIC_JIT_PREFETCH=0: no next-packet descriptor prefetch
    bool xpf_knob = false;     // MIMIC_JIT_XPF=1: next-packet header window prefetch (measured slower)
    // Lane prefetch (analyze_xpf's window, lpf_safe): when a lane starts, the descriptors and the
    // entry program's early window of its first kLpfD packets are loaded at once and parked in LDS,
    // so the packets then run without a dependent HBM round trip each (one lane's packets are
    // independent but for per-CPU state, which the programs keep in the lane value cache or in
    // memory they do not prefetch).  Only for program sets that never store into packet memory.
    // Off by default: cfg 2 measured 25.6 -> 32.0 us per launch (the lanes' prologue burst of 1 M
    // descriptor and window loads delays every first packet; tools/memtime.py), the
    // chunked schedule 38.9 -> 36.8 us, cfg 3 / cfg 4 unchanged.
    bool lpf_knob = false;
    bool hint_knob = false;    // MIMIC_JIT_HINT=1: slow-path branches marked [[unlikely]] (laid out after the hot code)
    bool lpf_on = false;
    bool lds_stack_on = false;
    static constexpr uint32_t kLpfD = 4;
    bool vc_knob = true;       // MIMIC_JIT_VC=0: no lane value cache (analyze_vc)
    uint32_t lds_stack_q = 16; // MIMIC_JIT_LDSSTK=Q: LDS window over the top 8Q bytes of frame 0
    bool vc_on = false;
    const SpreadReq *spread_req = nullptr;   // the VM's per-CPU arrays: spread mode is possible (analyze_spread)
    bool ctx_check = false;   // the kernel reads each packet's Run(ctx) context before its first step
    // The single-process form (Process.Run of one process, engine.cpp process_advance): every exit
    // stores r0..r10, the PC (the exit instruction's on a clean exit, as Step leaves it), the
    // program and the steps into KParams::step.  No fused counter increments: their register is
    // dead for the rest of the program, not after it (Run leaves every register readable).
    bool proc = false;
    bool spread_on = false;
    bool spread_own = false;   // the owned form (SpreadReq::own): every packet of a block's vCPUs in the block
    uint32_t spread_map = 0, spread_n = 0, spread_row = 0;   // the counted map, counter width, E * S
    std::map<uint32_t, uint32_t> vc_ok;  // LD_IMM64 slots (kernel-wide) naming a per-CPU array whose row can be cached -> E * S
    uint32_t vc_slot = 0;      // the LD_IMM64 slot (kernel-wide index) whose map hint names the cached map
    uint32_t vc_rb = 0;        // its row bytes
    bool vc_lds = false;       // the row is longer than four registers: an LDS slot per lane
    // The cross-packet window prefetch (analyze_xpf): the entry program `prog` makes its first
    // window of early loads at slot `hp` from register `base` = data + `off` - lo; the window's
    // bytes lie at data offset `off` .. off + 8 * words of the packet.
    struct Xpf {
        bool on = false;
        uint32_t prog = 0, hp = 0, base = 0, words = 0;
        int64_t off = 0;
    } xpf;
    bool cold_inline = true;   // the cold paths are inlined at every site (else called or deferred)
    // Deferred slow paths (large kernels): a slow-path site stores the registers its slot and
    // the slots after it can read (analyze_live), the PC, program and steps into the lane's
    // DeferRec and leaves the packet loop (defer_finish, runtime.h); the interpreter's resume
    // kernel (interp.hip), launched after the kernel, re-executes that slot on the generic path
    // and finishes the lane's packets.  No call remains in the kernel: a call's ABI (caller-saved
    // VGPRs around it, the callees' own registers, the Spill record in scratch) is what made the
    // cfg-5 chain need 380 VGPRs + AGPRs and 240 bytes of scratch at one wave per SIMD.
    bool defer_mode = false;
    std::vector<std::vector<uint16_t>> live;   // [prog][slot]: registers live into the slot
    uint32_t cold_sites = 0;
    static constexpr uint32_t kColdInlineSites = 48;
    bool stage = false;        // MIMIC_JIT_STAGE=1: LDS packet window
    bool has_tail() const { return any_tail; }
    bool has_early_loads() const { return !spec_use.empty(); }
    // Tail calls jump between programs.  With a jump table at every tail-call site as well as at
    // the entry, the programs form a cycle with several entries (irreducible control flow), which
    // the AMDGPU backend must restructure -- at a large register cost (cfg 5: 282 VGPRs without
    // the slow paths).  One dispatch block (D_) that the entry and every tail call go through
    // keeps the cycle single-entry.  MIMIC_JIT_DISPATCH=0: the per-site jump tables.
    bool dispatch_knob = true;
    bool dispatch_on() const { return dispatch_knob && any_tail; }
    std::string nonempty_cases() const {
        std::string c;
        for (auto &q : P)
            if (q.n) c += "    case " + std::to_string(q.id) + "u:";
        return c;
    }
    uint32_t ctx = CTX_XDP;    // the batch context this kernel is generated for

    std::string source() {
        // stage packets in LDS only when some access is expected to hit the packet
        if (stage) {
            bool any = false;
            for (auto &p : P) {
                ctx_hints(p);
                for (uint32_t i = 0; i < p.n; i++) {
                    const DInsn &x = p.ins[i];
                    const uint32_t h = AUX_H(x.aux);
                    if (h == H_LDX && hint(insn_src(x)) == HINT_PKT) any = true;
                    if ((h == H_ST || h == H_STX) && hint(insn_dst(x)) == HINT_PKT) any = true;
                    if (h == H_LDABS && ctx == CTX_SKB) any = true;
                }
            }
            stage = any && fast_paths;
        }
        // cold paths: inlined at each site for small kernels (best register allocation), called
        // for large ones (hipRTC time grows with every inlined copy)
        uint32_t sites = 0;
        for (auto &p : P)
            for (uint32_t i = 0; i < p.n; i++) {
                const uint32_t h = AUX_H(p.ins[i].aux);
                if (h == H_LDX || h == H_ST || h == H_STX || h == H_CALL || h == H_LDABS || h == H_SLOW) sites++;
            }
        if (careful_copies) sites *= 2;
        cold_sites = sites;
        // (the single-process form calls its slow paths: one lane, and hipRTC time is its tier-up cost)
        cold_inline = !proc && (cold_mode == 2 || (cold_mode == 0 && sites <= kColdInlineSites));
        defer_mode = !cold_inline && (cold_mode == 3 || cold_mode == 0) && !census && !stage && fast_paths && !proc;
        if (fast_paths) analyze_live();
        analyze_vc();
        if (forward)
            for (auto &p : P) analyze_fwd(p);
        if (forward && elide)
            for (auto &p : P) analyze_elide(p);
        if (speculate && fast_paths && !stage && !all_leaders)
            for (auto &p : P) analyze_spec(p);
        spread_on = analyze_spread();
        spread_own = spread_on && spread_req->own;
        if (spread_on) vc_on = false;   // no lane owns a vCPU's row in a spread kernel
        // the LDS stack window (runtime.h) when some stack store is made for real (not deferred
        // into a cold path, analyze_elide).  Measured: cfg 4 0.197 -> 0.179 ms per launch; the
        // sk_buff kernels keep their LDS for the SkbRec slots (with the window as well: cfg 5
        // 0.840 -> 0.848 ms)
        const bool skb_lds_planned = ctx == CTX_SKB && fast_paths && skb_fields && skb_lds_knob;
        if (lds_stack_q && fast_paths && !skb_lds_planned) {
            bool any = false;
            for (auto &p : P)
                for (uint32_t i = 0; i < p.n; i++) {
                    const DInsn &x = p.ins[i];
                    const uint32_t h = AUX_H(x.aux);
                    if ((h == H_ST || h == H_STX) && insn_dst(x) == 10 && !elided.count({p.id, i})) any = true;
                }
            if (any) E.line("#define MIMIC_LDS_STACK_Q %u", lds_stack_q);
            lds_stack_on = any;
        }
        if (defer_mode && sm_lds_knob) E.line("#define MIMIC_SM_LDS 1");
        if (const char *rm = getenv("MIMIC_JIT_ROOMS")) E.line("#define MIMIC_ROOMS_MODE %d", atoi(rm));   // measurement knob
        if (const char *dv = getenv("MIMIC_JIT_DEFS")) {   // measurement knob: "A,B=2" -> #define A / #define B 2
            std::string all(dv), d;
            for (size_t a = 0; a <= all.size(); a++) {
                if (a < all.size() && all[a] != ',') { d += all[a]; continue; }
                const size_t eq = d.find('=');
                if (!d.empty()) E.line("#define %s %s", d.substr(0, eq).c_str(), eq == std::string::npos ? "" : d.substr(eq + 1).c_str());
                d.clear();
            }
        }
        // traffic-attribution knobs (set through MIMIC_JIT_DEFS; results are wrong with them on):
        // no packet stores on the fast path, no fused counter adds, no per-packet result stores
        E.line("#ifdef MIMIC_MEAS_NOPKTST\n#define PKT_ST(p_, n_, v_) ((void)(v_))\n#else\n#define PKT_ST(p_, n_, v_) st_n(p_, n_, v_)\n#endif");
        E.line("#ifdef MIMIC_MEAS_NOATOM\n#define CNT_ADD(p_, n_, v_) ((void)(p_))\n#else\n#define CNT_ADD(p_, n_, v_) atomic_add_n(p_, n_, v_)\n#endif");
        if (spread_on) E.line("#define MIMIC_SPREAD 1");
        if (spread_own) E.line("#define MIMIC_SPREAD_OWN 1");
        if (const char *rc = getenv("MIMIC_SKB_ROOMS_CHAIN"))   // measurement: see engine.cpp skb_prepare
            if (rc[0] == '1') E.line("#define MIMIC_SKB_ROOMS_CHAIN 1");
        E.line("#define MIMIC_CTX_FIXED %u", ctx);
        E.line("#define MIMIC_COLD_INLINE %d", cold_inline ? 1 : 0);
        {   // no program of the set updates or deletes: hash tables are read-only in every launch
            // of this kernel (engine.cpp sets KParams.hash_ro from the same program set)
            bool writes = false;
            for (auto &p : P)
                for (uint32_t i = 0; i < p.n; i++)
                    if (AUX_H(p.ins[i].aux) == H_CALL && ((uint32_t)p.ins[i].k == 2 || (uint32_t)p.ins[i].k == 3)) writes = true;
            E.line("#define MIMIC_HASH_RO %d", writes ? 0 : 1);
            // no program of the set deletes: every launch of the kernel is pop-only (engine.cpp
            // KParams.hash_pop_only from the same programs), so only the lock-free insert is built
            bool deletes = false;
            for (auto &p : P)
                for (uint32_t i = 0; i < p.n; i++)
                    if (AUX_H(p.ins[i].aux) == H_CALL && (uint32_t)p.ins[i].k == 3) deletes = true;
            E.line("#define MIMIC_HASH_POPONLY %d", deletes ? 0 : 1);
            // inline inserts of a pop-only kernel: the block's waves combine their freelist
            // reservations (hashmap.h h_comb_reserve); zeroed in the prologue
            hash_combine = combine_knob && writes && !deletes && cold_inline && fast_paths;
            if (hash_combine) E.line("#define MIMIC_HASH_COMBINE 1");
            // ... and the VM's chunk map takes them in per-block chunks (batch kernels only: every
            // launch of one is followed by mimic_hash_compact_kernel, engine.cpp)
            hash_chunk = hash_combine && !proc && hchunk_knob > 0;
            if (hash_chunk) E.line("#define MIMIC_HASH_CHUNK 1\n#define MIMIC_HCHUNK %uu", (uint32_t)hchunk_knob);
        }
        E.line("#include \"runtime.h\"");
        if (spread_on) {
            // the block's counter table: one row of SPREAD_ROWW counters per vCPU its packets run on
            E.line("#define SPREAD_MAP %uu        // the per-CPU array the fused increments go to", spread_map);
            E.line("#define SPREAD_N %uu          // counter width (bytes)", spread_n);
            E.line("#define SPREAD_ROWW %uu       // counters per vCPU row (E * S / N)", spread_row / spread_n);
            E.line("#define SPREAD_ROWS %uu       // LDS table rows (0: agent-scope atomics into the map)", spread_req->lds_rows);
            E.line("#define SPREAD_PPB %uu        // packets per block", spread_req->ppb);
            E.line("typedef %s spread_t;", spread_n == 8 ? "unsigned long long" : "uint32_t");
            E.line("#if SPREAD_ROWS");
            E.line("#define spread_add(k_) __hip_atomic_fetch_add(&sacc_[srow_ * SPREAD_ROWW + (uint32_t)(ga_ - L.t_lo) / SPREAD_N], (spread_t)(k_), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)");
            E.line("#else");
            E.line("#define spread_add(k_) __hip_atomic_fetch_add((GAS spread_t *)(L.t_ptr + (uint32_t)(ga_ - L.t_lo)), (spread_t)(k_), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)");
            E.line("#endif");
        }
        if (proc) {   // PGID_: the program whose code the TERM is in (program() redefines it)
            E.line("#define PGID_ kp.entry_prog");
            E.line("#define TERM(s_, pc_) do { st_ = (int)(s_); epc_ = (int32_t)(pc_); pg_ = PGID_; goto L_term; } while (0)");
        } else {
            E.line("#define TERM(s_, pc_) do { st_ = (int)(s_); epc_ = (int32_t)(pc_); goto L_term; } while (0)");
        }
        // Around a cold call the lane state and the argument / result registers go through the
        // Spill record (runtime.h); only what a cold path can change comes back.
        E.line("#define SPILL() do { sp_.L = L; sp_.r[0] = r0; sp_.r[1] = r1; sp_.r[2] = r2; sp_.r[3] = r3; sp_.r[4] = r4; "
               "sp_.r[5] = r5; sp_.r[6] = r6; } while (0)");
        E.line("#define FILL() do { r0 = sp_.r[0]; r1 = sp_.r[1]; r2 = sp_.r[2]; r3 = sp_.r[3]; r4 = sp_.r[4]; r5 = sp_.r[5]; "
               "L.sm0 = sp_.L.sm0; L.sm1 = sp_.L.sm1; L.xdp_dirty = sp_.L.xdp_dirty; L.t_lo = sp_.L.t_lo; L.t_n = sp_.L.t_n; "
               "L.t_ptr = sp_.L.t_ptr; } while (0)");
        if (getenv("MIMIC_JIT_NOCOLD") && getenv("MIMIC_JIT_NOCOLD")[0] == '1')   // measurement only: no slow paths
            E.line("#define COLD_CALL(call_, pc_) TERM(MIMIC_ERR_ENGINE_HELPER, pc_)");
        else
            E.line("#define COLD_CALL(call_, pc_) do { VC_FLUSH(); SPILL(); call_; FILL(); if (sp_.st) TERM(sp_.st, pc_); } while (0)");
        // defer mode: the site stored the live registers; the rest is the lane's (defer_finish)
        // (the lane value cache is written back once, at L_defer: not inlined at every site)
        E.line("#define DFR(pc_, prog_) do { dr_->pc = (int32_t)(pc_); dr_->prog = (prog_); dr_->steps = steps - 1u; goto L_defer; } while (0)");
        // a cold path may read or write the cached row in memory: write it back and stop caching
        if (vc_on && vc_lds)
            E.line("#define VC_FLUSH() do { if (vcd_) { lvc_writeback(vcp_, vcb_, lvt_); vcd_ = 0u; } vcv_ = 0u; } while (0)");
        else if (vc_on)
            E.line("#define VC_FLUSH() do { if (vcd_) { vc_writeback(vcp_, vcb_, vc0_, vc1_, vc2_, vc3_); vcd_ = 0u; } vcv_ = 0u; } while (0)");
        else
            E.line("#define VC_FLUSH() do { } while (0)");
        // KParams is read through a pointer to a device copy: fields are loaded (scalar) where
        // they are used instead of all being preloaded into SGPRs from the kernarg segment
        // (which spills SGPRs and costs VGPRs / occupancy)
        // Register budget: kernels small enough to inline their slow paths are built for 4 waves
        // per SIMD -- 262 144 lanes then run in one round on the 1 024 SIMDs.  cfg 4 (169 VGPRs,
        // 2 waves): 0.172 -> 0.137 ms per launch; cfg 2 and 3 fit 4 waves anyway.  Large kernels
        // (cfg 5) keep the compiler's choice: forcing 2 waves there spills 264 VGPRs (1.2 vs 0.7 ms).
        const int wv = proc ? 0 : waves > 0 ? waves : (cold_inline ? 4 : 0);
        const std::string param = karg ? "const KParams kp_arg_" : "const KParams *__restrict__ kpp";
        if (wv > 0)
            E.line("%s", (std::string("extern \"C\" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(") +
                          std::to_string(wv) + "))) void mimic_jit_kernel(" + param + ") {").c_str());
        else
            E.line("%s", ("extern \"C\" __global__ __launch_bounds__(256) void mimic_jit_kernel(" + param + ") {").c_str());
        if (karg == 2) {
            // the parameters stay in the kernarg segment (constant address space): an opaque
            // constant-space pointer keeps every field a scalar load where it is used (not all
            // preloaded into SGPRs at entry)
            E.line("  (void)kp_arg_;   // the first (only) kernel argument: at offset 0 of the kernarg segment");
            E.line("  const KParams __attribute__((address_space(4))) *kp4_ = (const KParams __attribute__((address_space(4))) *)__builtin_amdgcn_kernarg_segment_ptr();");
            E.line("  asm volatile(\"\" : \"+s\"(kp4_));");
            E.line("  const KParams *kpp = (const KParams *)kp4_;");
        } else if (karg == 1) {
            E.line("  const KParams *kpp = &kp_arg_;");
        }
        E.line("  const KParams &kp = *kpp;");
        E.line("  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;");
        if (hash_chunk) E.line("  h_chunk_init(%s);   // (its waves: those the early return below keeps)", spread_on ? "0xffffffffu" : "kp.lanes");
        if (hash_combine) E.line("  h_comb_init();   // before any thread of the block can leave");
        if (!spread_on) E.line("  if (g >= kp.lanes) return;");
        if (stage && fast_paths) {
            E.line("  __shared__ PWin pwin_;");
            E.line("  const uint32_t tl0_ = threadIdx.x;");
        }
        skb_lds = ctx == CTX_SKB && fast_paths && skb_fields && skb_lds_knob;
        // the sk_buff records of the block's lanes, 168 bytes apart (an odd number of 8-byte
        // words: lanes reading the same field hit different banks); nothing reads them back
        if (skb_lds) E.line("  __shared__ uint64_t srec_[%uu * 256u];", kSrecQ);
        skb_walk = skb_lds && skb_walk_knob;
        skb_fast = skb_lds && !skb_walk && skb_fast_knob;
        if (skb_walk) E.line("  __shared__ uint32_t swin_[(SKB_WIN / 4u) * 256u];   // header windows (skb_load_walk)");
        E.line("  Lane L;");
        E.line("  Spill sp_;");
        if (census) {
            E.line("  uint32_t coldn_ = 0;");
            E.line("#define COLD_CALL_K(k_, call_, pc_) do { coldn_ += 1u << (k_); COLD_CALL(call_, pc_); } while (0)");
        }
        E.line("  L.lane = g;");
        if (spread_own) {
            // Owned spread: block b runs every packet of vCPU lanes [b * R, b * R + R), R = 256 / P
            // (P = packets per lane): thread t the j-th packet (j = t / R) of lane b * R + t % R, so
            // a wave's lanes take consecutive lanes' j-th packets (consecutive descriptors, packets
            // and results).  Fused increments add into the block's LDS table, one row per lane; the
            // block then adds its rows into the map with plain read-modify-writes: no other block
            // touches those vCPUs' rows in this launch.
            // Q = KParams::own_q packets per thread: R = 256 Q / P lanes, thread t their packets j,
            // j + P / Q, ... in order (the engine picks Q so that the launch about fills the chip once)
            E.line("  const uint32_t oP_ = kp.per_lane, oQ_ = kp.own_q, oS_ = oP_ / oQ_, oR_ = 256u / oS_;");
            E.line("  const uint32_t orow_ = threadIdx.x %% oR_, oj_ = threadIdx.x / oR_, olane_ = blockIdx.x * oR_ + orow_;");
            E.line("  const uint32_t osh_ = olane_ >= kp.sched_shift ? olane_ - kp.sched_shift : olane_ + kp.cpu_lanes - kp.sched_shift;");
            // the thread's k-th packet.  Interleaved: packet j = oj_ + k (P / Q) of its lane.  Chunked
            // (a lane's packets are contiguous): the block's 256 Q packets in order, thread t taking
            // t, t + 256, ... -- consecutive threads on consecutive packets, whose lane is i / P
            E.line("#define OWN_IDX_I(k_) ((oj_ < oS_ && olane_ < kp.cpu_lanes && (uint64_t)(oj_ + (k_) * oS_) * kp.cpu_lanes + osh_ < kp.n) ? (uint32_t)((uint64_t)(oj_ + (k_) * oS_) * kp.cpu_lanes + osh_) : NO_PKT)");
            E.line("#define OWN_IDX_C(k_) ((threadIdx.x + 256u * (k_) < oR_ * oP_ && (uint64_t)blockIdx.x * oR_ * oP_ + threadIdx.x + 256u * (k_) < kp.n) ? (uint32_t)((uint64_t)blockIdx.x * oR_ * oP_ + threadIdx.x + 256u * (k_)) : NO_PKT)");
            E.line("#define OWN_IDX(k_) (kp.sched == SCHED_CHUNKED ? OWN_IDX_C(k_) : OWN_IDX_I(k_))");
            E.line("  const uint32_t oi_ = OWN_IDX(0u);");
            E.line("  const DMap SM_ = cget(kp.maps, SPREAD_MAP);");
            E.line("  __shared__ spread_t sacc_[SPREAD_ROWS * SPREAD_ROWW];");
            E.line("  for (uint32_t w_ = threadIdx.x; w_ < SPREAD_ROWS * SPREAD_ROWW; w_ += 256u) sacc_[w_] = 0;");
            E.line("  __syncthreads();");
            E.line("  uint32_t srow_ = orow_, sbase_ = 0;");
            // the row words this thread adds into at the end, loaded now (their round trip overlaps
            // the packet's): word threadIdx.x of the block's rows (R * SPREAD_ROWW <= 256 words)
            E.line("  const bool ofw_ = threadIdx.x < oR_ * SPREAD_ROWW && blockIdx.x * oR_ + threadIdx.x / SPREAD_ROWW < kp.cpu_lanes;");
            E.line("  GAS spread_t *const ofd_ = (GAS spread_t *)(kp.arena + SM_.dev_off + (size_t)(kp.vcpu_begin + blockIdx.x * oR_ + threadIdx.x / SPREAD_ROWW) * SM_.dev_stride) + threadIdx.x %% SPREAD_ROWW;");
            E.line("  const spread_t ofv_ = ofw_ ? *ofd_ : (spread_t)0;");
        } else if (spread_on) {
            // Spread: block b runs packets [b * SPREAD_PPB, +SPREAD_PPB) of the batch, thread t the
            // ones at t, t + 256, ... (consecutive threads, consecutive packets); each packet's
            // vCPU comes from the schedule.  Fused increments add into the block's LDS table, one
            // row per vCPU lane its packets map to, (lane - lane0) mod V: at most SPREAD_PPB rows.
            E.line("  const uint32_t blo_ = blockIdx.x * SPREAD_PPB, bhi_ = blo_ + SPREAD_PPB < kp.n ? blo_ + SPREAD_PPB : kp.n;");
            E.line("  const uint32_t lam0_ = spread_lane(kp, blo_);");
            E.line("  const DMap SM_ = cget(kp.maps, SPREAD_MAP);");
            E.line("#if SPREAD_ROWS");
            E.line("  __shared__ spread_t sacc_[SPREAD_ROWS * SPREAD_ROWW];");
            E.line("  for (uint32_t w_ = threadIdx.x; w_ < SPREAD_ROWS * SPREAD_ROWW; w_ += 256u) sacc_[w_] = 0;");
            E.line("  __syncthreads();");
            E.line("#endif");
            E.line("  uint32_t srow_ = 0, sbase_ = 0;");
            // the lane of the thread's next packet: interleaved schedules step it by 256 mod V
            // (no division per packet), chunked ones divide
            E.line("  const uint32_t lstep_ = 256u %% kp.cpu_lanes;");
            E.line("  uint32_t lam_ = spread_lane(kp, blo_ + threadIdx.x);");
        } else {
            E.line("  L.cpu = lane_cpu(kp, g);");
        }
        if (vc_on) {
            // the lane's own row of the per-CPU array the hint names (analyze_vc)
            if (vc_lds) {
                // rows over 32 bytes: the lane's row in its LDS slot, dword d at lvc_[d * 256 + thread]
                // (two spare dwords: an unaligned read at the row's end stays in the array)
                E.line("  __shared__ uint32_t lvc_[(%uu / 4u + 2u) * 256u];", vc_rb);
                E.line("  uint32_t *const lvt_ = lvc_ + threadIdx.x;");
                E.line("  constexpr uint32_t vcb_ = %uu;   // the row's bytes", vc_rb);
                E.line("  uint32_t vcv_ = 0u, vcd_ = 0u, vclo_ = 0u; uint8_t *vcp_ = nullptr;");
                E.line("  { const uint32_t mh_ = AUX_MAPHINT(cget(kp.insns, %uu).aux);", vc_slot);
                E.line("    if (mh_) lvc_open(kp, cget(kp.maps, mh_ - 1u), L.cpu, vcb_, vcp_, vclo_, vcv_, lvt_); }");
            } else {
                E.line("  uint64_t vc0_ = 0, vc1_ = 0, vc2_ = 0, vc3_ = 0; uint32_t vcv_ = 0u, vcd_ = 0u, vclo_ = 0u, vcb_ = 0u; uint8_t *vcp_ = nullptr;");
                E.line("  { const uint32_t mh_ = AUX_MAPHINT(cget(kp.insns, %uu).aux);", vc_slot);
                E.line("    if (mh_) vc_open(kp, cget(kp.maps, mh_ - 1u), L.cpu, vcp_, vclo_, vcb_, vcv_, vc0_, vc1_, vc2_, vc3_); }");
            }
        }
        E.line("  uint32_t ex_begin = 0, ex_count = 0;");
        E.line("  if (kp.sched == SCHED_EXPLICIT) { ex_begin = *gp(kp.sched_start + g); ex_count = *gp(kp.sched_start + g + 1) - ex_begin; }");
        E.line("  uint64_t lane_steps = 0;");
        E.line("  const uint32_t P = kp.static_next + kp.stack_size + 1;");
        if (ctx == CTX_SKB) E.line("  const uint32_t SK_ = P;   // the sk_buff entry (skb.h)");
        E.line("  uint32_t ga_ = 0;   // the address of the current memory access");
        for (auto &f : fwd_store) E.line("  uint32_t fwd%u_%u_ = 0;   // value of the stack store at P%u slot %u", f.first, f.second, f.first, f.second);
        for (auto &u : spec_use)
            E.line("  %s sp%u_%u_ = 0;   // packet load of P%u slot %u, issued early", u.second == 8 ? "uint64_t" : "uint32_t",
                   u.first.first, u.first.second, u.first.first, u.first.second);
        if (!spec_use.empty()) E.line("  uint32_t spv_ = 1;   // 0 once a store through R10 left the stack: early values void");
        // The packet loop is software-pipelined by one descriptor: packet j+1's index, offset and
        // length are loaded while packet j runs (they travel with packet j's first loads), which
        // takes one dependent HBM round trip off every packet after the first.
        const bool pf = ctx == CTX_XDP && prefetch;
        skb_touch = ctx == CTX_SKB && skb_lds && !skb_walk && !skb_fast && skb_touch_knob != 0 && !spread_on;
        if (skb_touch) {
            E.line("  uint64_t noff_ = 0;   // the next packet's offset (skb_touch)");
            E.line("  { const uint32_t n_ = pkt_index(kp, g, 0u, ex_begin, ex_count); if (n_ != NO_PKT) noff_ = *gp(kp.pkt_off + n_); }");
        }
        if (!spec_use.empty() && !spread_on) analyze_xpf();
        // (LDS budget: 4 blocks of 256 lanes per CU with the window alone; no other LDS user)
        lpf_on = pf && xpf.on && lpf_knob && !xpf_knob && !spread_on && !stage && !vc_lds && !lds_stack_on && !defer_mode &&
                 !hash_combine && lpf_safe();
        if (!lpf_on && !xpf_knob) xpf.on = false;   // (the one-packet-ahead form only on request)
        if (spread_own) {
            // Multi-batch launches (mimic_run_xdp_many): every thread runs its packets of batch 0, then
            // of batch 1, ... (all batches have the same n, so the same packet indices), the block's
            // LDS counter table accumulating over all of them and flushed once; the last packet of a
            // batch prefetches the next batch's first descriptor.  many_n = 0: the one batch in kp.
            if (pf) E.line("  uint64_t noff_ = 0; uint32_t nlen_ = 0;");
            E.line("  const uint32_t nb_ = kp.many_n ? kp.many_n : 1u;");
            E.line("  bool bpre_ = false;   // this batch's first descriptor came with the previous batch's last packet");
            E.line("  for (uint32_t bt_ = 0; bt_ < nb_; bt_++) {");
            E.line("  const BatchRef br_ = kp.many_n ? cget(kp.many, bt_) : BatchRef{kp.pkt_data, kp.pkt_off, kp.pkt_len, kp.r0, kp.status, kp.steps, kp.err_pc, 0};");
        }
        if (lpf_on) {
            const uint32_t D = kLpfD, XW = xpf.words;
            E.line("  // lane prefetch: packets 0..%u of the lane, descriptors + P%u slot %u window (data + %u, %u words)", D - 1,
                   xpf.prog, xpf.hp, (uint32_t)xpf.off, XW);
            E.line("  __shared__ uint64_t lpfo_[%uu * 256u];", D);
            E.line("  __shared__ uint32_t lpfl_[%uu * 256u];", D);
            E.line("  __shared__ uint64_t lpfw_[%uu * 256u];", D * XW);
            E.line("  uint32_t lpf_n_ = 0u, xc_ok_ = 0u;");
            E.line("  if (kp.entry_prog == %uu && !kp.headroom_arr && !kp.tailroom_arr && kp.headroom == 0u && kp.tailroom == 0u) {", xpf.prog);
            for (uint32_t d = 0; d < D; d++) {
                E.line("    const uint32_t lx%u_ = pkt_index(kp, g, %uu, ex_begin, ex_count);", d, d);
                E.line("    uint64_t lo%u_ = 0; uint32_t ll%u_ = 0;", d, d);
                E.line("    if (lx%u_ != NO_PKT) { lo%u_ = *gp(kp.pkt_off + lx%u_); ll%u_ = *gp(kp.pkt_len + lx%u_); }", d, d, d, d, d);
            }
            for (uint32_t d = 0; d < D; d++) {
                for (uint32_t q = 0; q < XW; q++) E.line("    uint64_t lw%u_%u_ = 0;", d, q);
                E.line("    const bool lk%u_ = lx%u_ != NO_PKT && %uu <= ll%u_;", d, d, (uint32_t)xpf.off + 8 * XW, d);
                E.line("    if (lk%u_) {", d);
                E.line("      const uint8_t *xp_ = kp.pkt_data + lo%u_ + %uu;", d, (uint32_t)xpf.off);
                for (uint32_t q = 0; q < XW; q++) E.line("      lw%u_%u_ = ld_n(xp_ + %uu, 8u);", d, q, 8 * q);
                E.line("    }");
            }
            for (uint32_t d = 0; d < D; d++) {
                E.line("    lpfo_[%uu * 256u + threadIdx.x] = lo%u_;", d, d);
                E.line("    lpfl_[%uu * 256u + threadIdx.x] = ll%u_ | (lk%u_ ? 0x80000000u : 0u);", d, d, d);
                for (uint32_t q = 0; q < XW; q++) E.line("    lpfw_[%uu * 256u + threadIdx.x] = lw%u_%u_;", d * XW + q, d, q);
            }
            E.line("    lpf_n_ = lx0_ == NO_PKT ? 0u : lx1_ == NO_PKT ? 1u : lx2_ == NO_PKT ? 2u : lx3_ == NO_PKT ? 3u : 4u;");
            E.line("  }");
            static_assert(kLpfD == 4, "the lpf_n_ line above");
        } else if (pf && xpf.on) {
            // descriptors two packets ahead, the window one packet ahead (analyze_xpf)
            E.line("  const bool xpf_on_ = kp.entry_prog == %uu && !kp.headroom_arr;   // P%u slot %u window, data + %u, %u words",
                   xpf.prog, xpf.prog, xpf.hp, (uint32_t)xpf.off, xpf.words);
            E.line("  uint64_t noff_ = 0, noff2_ = 0; uint32_t nlen_ = 0, nlen2_ = 0, nidx_ = NO_PKT, nidx2_ = NO_PKT, xn_ok_ = 0u, xc_ok_ = 0u;");
            for (uint32_t q = 0; q < xpf.words; q++) E.line("  uint64_t xn%u_ = 0;", q);
            E.line("  nidx_ = pkt_index(kp, g, 0u, ex_begin, ex_count);");
            E.line("  if (nidx_ != NO_PKT) { noff_ = *gp(kp.pkt_off + nidx_); nlen_ = *gp(kp.pkt_len + nidx_); }");
            emit_xpf_issue("  ");
            E.line("  nidx2_ = nidx_ != NO_PKT ? pkt_next(kp, nidx_, 1u, ex_begin, ex_count) : NO_PKT;");
            E.line("  if (nidx2_ != NO_PKT) { noff2_ = *gp(kp.pkt_off + nidx2_); nlen2_ = *gp(kp.pkt_len + nidx2_); }");
        } else if (pf) {
            if (spread_own)
                E.line("  if (!bpre_ && oi_ != NO_PKT) { noff_ = *gp(br_.pkt_off + oi_); nlen_ = *gp(br_.pkt_len + oi_); } bpre_ = false;");
            else
                E.line("  uint64_t noff_ = 0; uint32_t nlen_ = 0;");
            if (spread_own) {
            } else if (spread_on)
                E.line("  { const uint32_t n_ = blo_ + threadIdx.x; if (n_ < bhi_) { noff_ = *gp(kp.pkt_off + n_); nlen_ = *gp(kp.pkt_len + n_); } }");
            else
                E.line("  { const uint32_t n_ = pkt_index(kp, g, 0u, ex_begin, ex_count); if (n_ != NO_PKT) { noff_ = *gp(kp.pkt_off + n_); nlen_ = *gp(kp.pkt_len + n_); } }");
        }
        if (spread_own) {
            E.line("  for (uint32_t j = 0; j < oQ_; j++) {   // the thread's packets of its lane, in order");
            E.line("    const uint32_t i = j ? OWN_IDX(j) : oi_;");
            E.line("    if (i == NO_PKT) break;");
        } else if (spread_on) {
            E.line("  for (uint32_t j = 0; j < SPREAD_PPB / 256u; j++) {");
            E.line("    const uint32_t i = blo_ + j * 256u + threadIdx.x;");
            E.line("    if (i >= bhi_) break;");
        } else {
            E.line("  for (uint32_t j = 0; j < kp.per_lane; j++) {");
            E.line("    uint32_t i;");
            E.line("    if (kp.sched == SCHED_CHUNKED) { const uint64_t ii = (uint64_t)g * kp.per_lane + j; if (ii >= kp.n) break; i = (uint32_t)ii; }");
            E.line("    else if (kp.sched == SCHED_INTERLEAVED) { const uint64_t ii = (uint64_t)j * kp.lanes + (g >= kp.sched_shift ? g - kp.sched_shift : g + kp.lanes - kp.sched_shift); if (ii >= kp.n) break; i = (uint32_t)ii; }");
            E.line("    else { if (j >= ex_count) break; i = ld_nt(kp.sched_pkts + ex_begin + j); }");
        }
        if (lpf_on) {
            E.line("    uint64_t poff_; uint32_t plen_;");
            for (uint32_t q = 0; q < xpf.words; q++) E.line("    uint64_t xc%u_ = 0;", q);
            E.line("    if (j < lpf_n_) {   // parked in LDS when the lane started");
            E.line("      poff_ = lpfo_[j * 256u + threadIdx.x];");
            E.line("      const uint32_t lw_ = lpfl_[j * 256u + threadIdx.x];");
            E.line("      plen_ = lw_ & 0x7fffffffu;");
            E.line("      xc_ok_ = lw_ >> 31;");
            for (uint32_t q = 0; q < xpf.words; q++)
                E.line("      if (xc_ok_) xc%u_ = lpfw_[(j * %uu + %uu) * 256u + threadIdx.x];", q, xpf.words, q);
            E.line("    } else {");
            E.line("      poff_ = *gp(kp.pkt_off + i); plen_ = *gp(kp.pkt_len + i); xc_ok_ = 0u;");
            E.line("    }");
        } else if (pf && xpf.on) {
            E.line("    const uint64_t poff_ = noff_; const uint32_t plen_ = nlen_;");
            E.line("    xc_ok_ = xn_ok_;");
            for (uint32_t q = 0; q < xpf.words; q++) E.line("    const uint64_t xc%u_ = xn%u_;", q, q);
            E.line("    noff_ = noff2_; nlen_ = nlen2_; nidx_ = nidx2_;");
            emit_xpf_issue("    ");
            E.line("    nidx2_ = nidx_ != NO_PKT ? pkt_next(kp, nidx_, j + 2u, ex_begin, ex_count) : NO_PKT;");
            E.line("    if (nidx2_ != NO_PKT) { noff2_ = *gp(kp.pkt_off + nidx2_); nlen2_ = *gp(kp.pkt_len + nidx2_); }");
        } else if (pf) {
            E.line("    const uint64_t poff_ = noff_; const uint32_t plen_ = nlen_;");
            if (nt) E.line("    { const uint32_t n_ = pkt_next(kp, i, j + 1, ex_begin, ex_count); if (n_ != NO_PKT) { noff_ = ld_nt(kp.pkt_off + n_); nlen_ = ld_nt(kp.pkt_len + n_); } }");
            else if (spread_own) {
                E.line("    if (j + 1u < oQ_) { const uint32_t n_ = OWN_IDX(j + 1u); if (n_ != NO_PKT) { noff_ = *gp(br_.pkt_off + n_); nlen_ = *gp(br_.pkt_len + n_); } }");
                E.line("    else if (bt_ + 1u < nb_ && oi_ != NO_PKT) { const BatchRef nx_ = cget(kp.many, bt_ + 1u); noff_ = *gp(nx_.pkt_off + oi_); nlen_ = *gp(nx_.pkt_len + oi_); bpre_ = true; }");
            }
            else if (spread_on) E.line("    { const uint32_t n_ = i + 256u; if (n_ < bhi_) { noff_ = *gp(kp.pkt_off + n_); nlen_ = *gp(kp.pkt_len + n_); } }");
            else E.line("    { const uint32_t n_ = pkt_next(kp, i, j + 1, ex_begin, ex_count); if (n_ != NO_PKT) { noff_ = *gp(kp.pkt_off + n_); nlen_ = *gp(kp.pkt_len + n_); } }");
        }
        if (memtime) E.line("    const uint32_t mt0_ = (uint32_t)__builtin_amdgcn_s_memrealtime();");
        // fields used once per packet are read through an opaque copy of the parameter pointer:
        // loaded where used instead of hoisted out of the packet loop into SGPRs
        if (kq_mode == 1) E.line("    const KParams *kqp_ = kpp; asm volatile(\"\" : \"+s\"(kqp_)); const KParams &kq_ = *kqp_;");
        else E.line("    const KParams &kq_ = kp;");
        if (spread_own) {   // the packet's vCPU and its row of the spread map (chunked: per packet)
            E.line("    { const uint32_t ol_ = kp.sched == SCHED_CHUNKED ? i / oP_ : olane_;");
            E.line("      srow_ = ol_ - blockIdx.x * oR_;");
            E.line("      L.cpu = (int32_t)(kp.vcpu_begin + ol_);");
            E.line("      sbase_ = SM_.backing_addr + (uint32_t)L.cpu * SM_.addr_period; }");
        } else if (spread_on) {   // this packet's vCPU (the schedule's lane for it) and its row of the spread map
            E.line("    { if (kp.sched == SCHED_CHUNKED) lam_ = i / kp.per_lane;");
            E.line("      else if (j) { lam_ += lstep_; if (lam_ >= kp.cpu_lanes) lam_ -= kp.cpu_lanes; }");
            E.line("      L.cpu = (int32_t)(kp.vcpu_begin + lam_);");
            E.line("      srow_ = lam_ >= lam0_ ? lam_ - lam0_ : lam_ + kp.cpu_lanes - lam0_;");
            E.line("      sbase_ = SM_.backing_addr + (uint32_t)L.cpu * SM_.addr_period; }");
        }
        // The lane's private-memory and LDS addresses are loop-invariant; hoisted out of the packet
        // loop they would stay live (one VGPR pair per stack slot) through every packet.  An opaque
        // per-iteration copy of the lane index keeps each address next to its use.
        if (opaque_lane) {
            E.line("    { uint32_t ln_ = g; asm volatile(\"\" : \"+v\"(ln_)); L.lane = ln_; }");
            if (stage && fast_paths) E.line("    uint32_t tl_ = tl0_; asm volatile(\"\" : \"+v\"(tl_));");
        } else if (stage && fast_paths) {
            E.line("    const uint32_t tl_ = tl0_;");
        }
        if (ctx == CTX_SKB) {
            // NewProcess + LinuxContextSKBuff.Load (context_sk_buff.go:42-107, skb.h)
            E.line("    uint64_t r1 = 0;");
            if (skb_walk)   // the process's SkbRec built in this lane's LDS slot: every field access reads LDS
                E.line("    const int ls_ = skb_load_walk(kp, L, i, r1, srec_ + %uu * threadIdx.x, swin_);", kSrecQ);
            else if (skb_fast)   // derived here from the header bytes (exception frames: the prep's words), into the LDS slot
                E.line("    const int ls_ = skb_load_fast(kp, L, i, r1, srec_ + %uu * threadIdx.x, *gp(kq_.pkt_off + i), *gp(kq_.pkt_len + i), *gp(kq_.skb_prefix + i));", kSrecQ);
            else if (skb_touch) {
                E.line("    const uint64_t poff_ = noff_;");
                E.line("    { const uint32_t n_ = pkt_next(kp, i, j + 1, ex_begin, ex_count); if (n_ != NO_PKT) noff_ = *gp(kp.pkt_off + n_); }");
                // two dwords: packet bytes 14 and 38 (the Ethernet / IP / transport headers span at most
                // two 64-byte halves of a 128-byte line whatever the slot's alignment); consumed at the
                // packet's end, so the wait for them is long past
                if (skb_touch_knob == 1) {
                    E.line("    const uint32_t th0_ = *gp((const uint32_t *)(kq_.pkt_data + poff_ + SKB_HEADROOM + 12u));");
                    E.line("    const uint32_t th1_ = *gp((const uint32_t *)(kq_.pkt_data + poff_ + SKB_HEADROOM + 36u));");
                }
                E.line("    const int ls_ = skb_load_lds_po(kp, L, i, r1, srec_ + %uu * threadIdx.x, poff_);", kSrecQ);
                // consumed where the record's own wait already covers them (issued before it)
                if (skb_touch_knob == 1) E.line("    asm volatile(\"\" :: \"v\"(th0_), \"v\"(th1_));");
            } else if (skb_lds)   // the process's SkbRec into this lane's LDS slot: every field access reads LDS
                E.line("    const int ls_ = skb_load_lds(kp, L, i, r1, srec_ + %uu * threadIdx.x);", kSrecQ);
            else
                E.line("    const int ls_ = skb_load(kp, L, i, r1);");
            // the window starts at the packet (skb.data = packet memory + 32)
            if (stage && fast_paths)
                E.line("    const uint32_t W_ = ls_ ? 0u : win_stage(pwin_, tl_, L.pkt + SKB_HEADROOM, L.M - SKB_HEADROOM);");
        } else {
            // NewProcess + LinuxContextXDP.Load (vm.go:198-235, context_xdp_md.go:47-115)
            E.line("    const uint32_t H = kq_.headroom_arr ? ld_nt(kq_.headroom_arr + i) : kq_.headroom;");
            E.line("    const uint32_t T = kq_.tailroom_arr ? ld_nt(kq_.tailroom_arr + i) : kq_.tailroom;");
            if (pf) {
                E.line("    const uint32_t len = plen_;");
                E.line("    L.pkt = %s + poff_;", spread_own ? "br_.pkt_data" : "kq_.pkt_data");
            } else if (spread_own) {
                E.line("    const uint32_t len = *gp(br_.pkt_len + i);");
                E.line("    L.pkt = br_.pkt_data + *gp(br_.pkt_off + i);");
            } else if (nt) {
                E.line("    const uint32_t len = ld_nt(kq_.pkt_len + i);");
                E.line("    L.pkt = kq_.pkt_data + ld_nt(kq_.pkt_off + i);");
            } else {
                E.line("    const uint32_t len = *gp(kq_.pkt_len + i);");
                E.line("    L.pkt = kq_.pkt_data + *gp(kq_.pkt_off + i);");
            }
            E.line("    L.M = H + len + T;");
            E.line("    L.pa = P;");
            E.line("    L.rec = nullptr;");
            E.line("    for (uint32_t b = 0; b < H; b++) *gp(L.pkt + b) = 0;");
            E.line("    for (uint32_t b = 0; b < T; b++) *gp(L.pkt + H + len + b) = 0;");
            E.line("    L.data = P + H;");
            E.line("    L.data_end = P + H + len;");
            E.line("    L.ingress = (uint32_t)(kq_.ingress_arr ? ld_nt(kq_.ingress_arr + i) : kq_.ingress);");
            E.line("    L.rxq = (uint32_t)(kq_.rxq_arr ? ld_nt(kq_.rxq_arr + i) : kq_.rxq);");
            E.line("    L.egress = (uint32_t)(kq_.egress_arr ? ld_nt(kq_.egress_arr + i) : kq_.egress);");
            if (stage && fast_paths) E.line("    const uint32_t W_ = win_stage(pwin_, tl_, L.pkt, L.M);");
            E.line("    uint64_t r1 = P + L.M + 1;");
        }
        E.line("    SM0(L) = 0; SM1(L) = 0; L.xdp_dirty = 0; L.nframes = 0; L.tailcalls = 0; L.t_lo = 0; L.t_n = 0; L.t_ptr = nullptr;");
        E.line("    uint64_t r0 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0, r8 = 0, r9 = 0;");
        E.line("    uint64_t r10 = kp.static_next + kp.frame_size;");
        E.line("    uint32_t steps = 0;");
        if (census) E.line("    coldn_ = 0;");
        if (!spec_use.empty()) E.line("    spv_ = 1;");
        E.line("    int st_ = 0;");
        E.line("    int32_t epc_ = -1;");
        if (proc) E.line("    uint32_t pg_ = kp.entry_prog;");
        if (ctx == CTX_SKB) E.line("    if (ls_) TERM(ls_, -1);");
        // Run(ctx): a context already done when the process would take its first step ends it
        // there (vm.go:344-349); a launch without contexts skips this on a uniform scalar test
        // (a variant of its own, built for launches given contexts: the check costs ~2 % on cfg 2)
        if (ctx_check) E.line("    { const uint32_t cz_ = ctx_done(kq_, i); if (cz_) TERM(MIMIC_ERR_CANCELED - 1u + cz_, 0); }");
        if (dispatch_on()) {
            // one dispatch block for the entry and every tail call (see dispatch_on)
            E.line("    uint32_t cur_;   // no initializer: the TERM gotos above jump past it");
            E.line("    cur_ = kp.entry_prog;");
            E.line("    switch (cur_) {");
            for (auto &p : P)
                if (p.n == 0) E.line("    case %u: steps = 1; TERM(MIMIC_ERR_PC_OOB, 0);", p.id);  // vm.go:297-299
            E.line("%s", nonempty_cases().c_str());
            E.line("      break;");
            E.line("    default: TERM(MIMIC_ERR_PC_OOB, 0);");
            E.line("    }");
            E.line("  D_:");
            E.line("    switch (cur_) {");
            for (auto &p : P)
                if (p.n) E.line("    case %u: goto P%u_0;", p.id, p.id);
            E.line("    default: TERM(MIMIC_ERR_ENGINE_HELPER, -1);");
            E.line("    }");
        } else {
            E.line("    switch (kp.entry_prog) {");
            for (auto &p : P) {
                if (p.n == 0) E.line("    case %u: steps = 1; TERM(MIMIC_ERR_PC_OOB, 0);", p.id);  // vm.go:297-299
                else E.line("    case %u: goto P%u_0;", p.id, p.id);
            }
            E.line("    default: TERM(MIMIC_ERR_PC_OOB, 0);");
            E.line("    }");
        }
        for (auto &p : P) program(p);
        E.line("    TERM(MIMIC_ERR_ENGINE_HELPER, -1);");
        if (defer_mode) {
            E.line("  L_defer:");
            E.line("    VC_FLUSH();");
            E.line("    defer_finish(kp, L, g, i, j, lane_steps);");
            E.line("    break;");
        }
        E.line("  L_term:");
        if (kq_mode == 2)   // the result pointers are loaded here, once per packet, not held in SGPRs
            E.line("    { const KParams *kqp_ = kpp; asm volatile(\"\" : \"+s\"(kqp_)); const KParams &kq_ = *kqp_;");
        else
            E.line("    {");
        E.line("#ifndef MIMIC_MEAS_NORES");
        {   // the owned form's results go to the batch of this iteration (br_)
            const char *rb = spread_own ? "br_" : "kq_";
            if (nt || ntres) {
                E.line("    if (%s.r0) st_nt(%s.r0 + i, r0);", rb, rb);
                E.line("    if (%s.status) st_nt(%s.status + i, (uint8_t)st_);", rb, rb);
            } else {
                E.line("    if (%s.r0) *gp(%s.r0 + i) = r0;", rb, rb);
                E.line("    if (%s.status) *gp(%s.status + i) = (uint8_t)st_;", rb, rb);
            }
            if (census) E.line("    if (%s.steps) st_nt(%s.steps + i, coldn_);   // census: slow-path calls, not steps", rb, rb);
            else if (memtime) E.line("    if (%s.steps) st_nt(%s.steps + i, (uint32_t)__builtin_amdgcn_s_memrealtime());", rb, rb);
            else E.line("    if (%s.steps) st_nt(%s.steps + i, steps);", rb, rb);
            if (memtime) E.line("    if (%s.err_pc) st_nt(%s.err_pc + i, (int32_t)mt0_);", rb, rb);
            else E.line("    if (%s.err_pc) st_nt(%s.err_pc + i, epc_);", rb, rb);
        }
        E.line("#endif");
        E.line("    }");
        if (proc) {   // Process.Run: the whole state (interp.hip step_save), the process done
            E.line("    if (kq_.step) { StepState *S_ = kq_.step;");
            E.line("      S_->r[0] = r0; S_->r[1] = r1; S_->r[2] = r2; S_->r[3] = r3; S_->r[4] = r4; S_->r[5] = r5;");
            E.line("      S_->r[6] = r6; S_->r[7] = r7; S_->r[8] = r8; S_->r[9] = r9; S_->r[10] = r10;");
            E.line("      S_->pc = epc_; S_->prog = pg_; S_->steps = steps; S_->status = st_; S_->started = 1u; S_->finished = 1u; }");
        }
        E.line("    lane_steps += steps;");
        E.line("  }");
        if (spread_own) E.line("  }   // batches");
        if (vc_on) E.line("  VC_FLUSH();");
        if (spread_own) {
            // the block's rows into the map: plain read-modify-writes (the block owns these vCPUs)
            E.line("#if !defined(MIMIC_MEAS_NOFLUSH)   // (measurement knob: no flush, counters wrong)");
            E.line("  __syncthreads();");
            E.line("  if (ofw_ && sacc_[threadIdx.x]) *ofd_ = ofv_ + sacc_[threadIdx.x];");
            E.line("  for (uint32_t w_ = threadIdx.x + 256u; w_ < oR_ * SPREAD_ROWW; w_ += 256u) {   // rows past 256 words");
            E.line("    const spread_t v_ = sacc_[w_];");
            E.line("    if (!v_) continue;");
            E.line("    const uint32_t r_ = w_ / SPREAD_ROWW, q_ = w_ - r_ * SPREAD_ROWW;");
            E.line("    GAS spread_t *d_ = (GAS spread_t *)(kp.arena + SM_.dev_off + (size_t)(kp.vcpu_begin + blockIdx.x * oR_ + r_) * SM_.dev_stride) + q_;");
            E.line("    *d_ += v_;");
            E.line("  }");
            E.line("#endif");
        } else if (spread_on) {
            // the block's counters into the map: one agent-scope add per non-zero counter (a row's
            // counters are contiguous in the arena, so consecutive threads add consecutive words)
            E.line("#if SPREAD_ROWS && !defined(MIMIC_MEAS_NOFLUSH)   // (measurement knob: no flush, counters wrong)");
            E.line("  __syncthreads();");
            // a table that covers every vCPU lane (V <= packets per block): the block writes it,
            // rotated to absolute lanes, into its slice of kp.spread_part with plain stores, and
            // mimic_spread_reduce_kernel adds the blocks' slices into the map (one agent-scope add per
            // counter per group of blocks, not per block: the per-block adds were 43 % of the kernel)
            E.line("  if (kp.spread_part && kp.cpu_lanes == SPREAD_ROWS) {");
            E.line("    spread_t *pt_ = (spread_t *)kp.spread_part + (size_t)blockIdx.x * (SPREAD_ROWS * SPREAD_ROWW);");
            E.line("    for (uint32_t w_ = threadIdx.x; w_ < SPREAD_ROWS * SPREAD_ROWW; w_ += 256u) {");
            E.line("      const uint32_t r_ = w_ / SPREAD_ROWW, q_ = w_ - r_ * SPREAD_ROWW;");
            E.line("      const uint32_t lr_ = lam0_ + r_ < SPREAD_ROWS ? lam0_ + r_ : lam0_ + r_ - SPREAD_ROWS;");
            E.line("      pt_[lr_ * SPREAD_ROWW + q_] = sacc_[w_];");
            E.line("    }");
            E.line("  } else");
            E.line("  for (uint32_t w_ = threadIdx.x; w_ < SPREAD_ROWS * SPREAD_ROWW; w_ += 256u) {");
            E.line("    const spread_t v_ = sacc_[w_];");
            E.line("    if (!v_) continue;");
            E.line("    const uint32_t r_ = w_ / SPREAD_ROWW, q_ = w_ - r_ * SPREAD_ROWW;");
            E.line("    const uint32_t lr_ = lam0_ + r_ < kp.cpu_lanes ? lam0_ + r_ : lam0_ + r_ - kp.cpu_lanes;");
            E.line("    spread_t *d_ = (spread_t *)(kp.arena + SM_.dev_off + (size_t)(kp.vcpu_begin + lr_) * SM_.dev_stride) + q_;");
            E.line("    __hip_atomic_fetch_add((GAS spread_t *)d_, v_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);");
            E.line("  }");
            E.line("#endif");
        }
        E.line("  if (kp.lane_steps) st_nt(kp.lane_steps + g, lane_steps);");
        if (hash_chunk) E.line("  h_chunk_fini();   // the block's last wave hands its chunk's remainder back");
        E.line("}");
        if (census) {   // diagnostics: each slow-path call adds 1 to its kind's 4-bit field of coldn_
            static const char *kinds[] = {"cold_load(", "cold_store(", "cold_lookup(", "cold_update(", "cold_delete(",
                                          "cold_tailcall(", "cold_ldabs(", "cold_adjust_tail("};
            for (int k = 0; k < 8; k++) {
                const std::string from = std::string("COLD_CALL(") + kinds[k], to = "COLD_CALL_K(" + std::to_string(4 * k) + ", " + kinds[k];
                for (size_t q = E.s.find(from); q != std::string::npos; q = E.s.find(from, q + to.size())) E.s.replace(q, from.size(), to);
            }
        }
        return E.s;
    }

  private:
    const std::vector<ProgView> &P;
    Emitter E;
    // packet-entry fast paths: the entry's address, the window's offset in packet memory, and
    // the byte order of scalar accesses (sk_buff packets are BigEndian PlainMemory)
    const char *pa() const { return ctx == CTX_SKB ? "L.pa" : "P"; }
    uint32_t wb() const { return ctx == CTX_SKB ? SKB_HEADROOM_J : 0u; }
    std::string ord(const std::string &v, uint32_t n) const {
        return ctx == CTX_SKB && n > 1 ? "bswap_n(" + v + ", " + std::to_string(n) + "u)" : v;
    }
    static constexpr uint32_t SKB_HEADROOM_J = 32;
    bool any_tail = false, any_local = false, all_leaders = false;
    uint32_t blk_start = 0;   // first slot of the basic block being emitted
    uint32_t cur_prog = 0;    // program being emitted

    std::vector<uint32_t> leaders(const ProgView &p) const {
        std::set<uint32_t> lead = {0};
        for (uint32_t i = 0; i < p.n; i++) {
            const DInsn &x = p.ins[i];
            const uint32_t h = AUX_H(x.aux);
            if ((h == H_JA || h == H_JCC || h == H_CALL_LOCAL) && (x.aux & AUX_JT_OK))
                lead.insert((uint32_t)jump_target(x, i));
            if (ends_block(x) && i + 1 < p.n) lead.insert(i + 1);
            if (all_leaders) lead.insert(i);
        }
        return std::vector<uint32_t>(lead.begin(), lead.end());
    }

    // Stack-store forwarding into helper 1's key (per basic block): which 4-byte store to
    // R10 + c the key at R2 = R10 + c was written by, with no possibly-aliasing store between.
    // Registers are tracked only as "R10 + constant"; a store through any other base clears it.
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> fwd_call;   // (prog, call slot) -> store slot
    std::set<std::pair<uint32_t, uint32_t>> fwd_store;            // (prog, store slot) to capture
    // Forwarded stores whose memory write is deferred into the lookup's cold path: in a program
    // that never reads the stack other than through forwarded lookup keys (no load through R10
    // or a register derived from it, no other helper call, no BPF-to-BPF call, no tail call in
    // the set), the stack is dead at exit and nothing else observes the word, so the store is
    // only made when the generic lookup (which reads the key from memory) runs.
    std::set<std::pair<uint32_t, uint32_t>> elided;
    void analyze_elide(const ProgView &p) {
        if (any_tail || any_local || p.n == 0) return;
        // forward may-analysis over the CFG: which registers may hold a stack address
        const std::vector<uint32_t> Lb = leaders(p);
        std::map<uint32_t, size_t> blk;
        for (size_t b = 0; b < Lb.size(); b++) blk[Lb[b]] = b;
        std::vector<uint32_t> in(Lb.size(), 0);
        std::vector<bool> seen(Lb.size(), false);
        in[0] = 1u << 10;
        seen[0] = true;
        auto transfer = [&](uint32_t t, const DInsn &x) {
            const uint32_t h = AUX_H(x.aux), d = insn_dst(x), sr = insn_src(x), op = insn_op(x);
            if (d > 10) return t;
            if (h == H_ALU64 || h == H_ALU32) {
                const bool mov = (op & 0xf0) == 0xb0;
                const bool src_t = (x.aux & AUX_X) && sr <= 10 && ((t >> sr) & 1);
                const bool res = mov ? src_t : (((t >> d) & 1) || src_t);
                return res ? (t | (1u << d)) : (t & ~(1u << d));
            }
            if (h == H_LDX || h == H_LDIMM) return t & ~(1u << d);
            if (h == H_CALL) return t & ~1u;
            return t;
        };
        for (bool changed = true; changed;) {
            changed = false;
            for (size_t b = 0; b < Lb.size(); b++) {
                if (!seen[b]) continue;
                const uint32_t s0 = Lb[b], e = b + 1 < Lb.size() ? Lb[b + 1] : p.n;
                uint32_t t = in[b];
                for (uint32_t i = s0; i < e; i++) {
                    const DInsn &x = p.ins[i];
                    const uint32_t h = AUX_H(x.aux), sr = insn_src(x);
                    if (h == H_LDX && sr <= 10 && ((t >> sr) & 1)) return;   // reads the stack
                    if (h == H_STX && sr <= 10 && ((t >> sr) & 1)) return;   // a stack address escapes to memory
                    if (h == H_SLOW || h == H_LDABS || h == H_CALL_LOCAL) return;
                    if (h == H_CALL && !((uint32_t)x.k == 1 && fwd_call.count({p.id, i})) && (uint32_t)x.k != 8) return;
                    t = transfer(t, x);
                }
                const DInsn &last = p.ins[e - 1];
                const uint32_t h = AUX_H(last.aux);
                std::vector<int64_t> succ;
                if ((!ends_block(last) || h == H_JCC) && (last.aux & AUX_FALL_OK)) succ.push_back(e);
                if ((h == H_JA || h == H_JCC) && (last.aux & AUX_JT_OK)) succ.push_back(jump_target(last, e - 1));
                for (int64_t sx : succ) {
                    auto it = blk.find((uint32_t)sx);
                    if (it == blk.end()) continue;
                    const uint32_t nin = in[it->second] | t;
                    if (!seen[it->second] || nin != in[it->second]) {
                        in[it->second] = nin;
                        seen[it->second] = true;
                        changed = true;
                    }
                }
            }
        }
        for (auto &f : fwd_store)
            if (f.first == p.id && AUX_H(p.ins[f.second].aux) == H_STX && insn_dst(p.ins[f.second]) == 10) elided.insert(f);
    }
    void analyze_fwd(const ProgView &p) {
        if (!fast_paths || p.n == 0) return;
        const std::vector<uint32_t> Lb = leaders(p);
        for (size_t b = 0; b < Lb.size(); b++) {
            const uint32_t s0 = Lb[b], e = b + 1 < Lb.size() ? Lb[b + 1] : p.n;
            bool known[11] = {};
            int64_t rel[11] = {};
            known[10] = true;
            std::map<int64_t, std::pair<uint32_t, uint32_t>> recs;   // offset -> (size, slot)
            for (uint32_t i = s0; i < e; i++) {
                const DInsn &x = p.ins[i];
                const uint32_t h = AUX_H(x.aux), op = insn_op(x), d = insn_dst(x), sr = insn_src(x);
                if (h == H_CALL && (uint32_t)x.k == 1 && known[2]) {
                    auto it = recs.find(rel[2]);
                    if (it != recs.end() && it->second.first == 4) {
                        fwd_call[{p.id, i}] = it->second.second;
                        fwd_store.insert({p.id, it->second.second});
                    }
                }
                if (h == H_ST || h == H_STX) {
                    const uint32_t n = AUX_SZ(x.aux);
                    if (d <= 10 && known[d]) {
                        const int64_t o = rel[d] + insn_off(x);
                        for (auto it = recs.begin(); it != recs.end();) {
                            if (it->first < o + (int64_t)n && o < it->first + (int64_t)it->second.first) it = recs.erase(it);
                            else ++it;
                        }
                        recs[o] = {n, i};
                    } else {
                        recs.clear();
                    }
                }
                if (h == H_ALU64 && op == 0xbf && sr <= 10 && known[sr]) {           // mov rD, (R10 + c)
                    known[d] = true;
                    rel[d] = rel[sr];
                } else if (h == H_ALU64 && op == 0x07 && d <= 10 && known[d]) {      // add rD, imm
                    rel[d] += (int64_t)(int32_t)(uint32_t)x.k;
                } else if ((h == H_ALU64 || h == H_ALU32 || h == H_LDIMM || h == H_LDX || h == H_SLOW) && d <= 10) {
                    known[d] = d == 10;
                }
                if (h == H_CALL) known[0] = false;
                if (h == H_LDABS) for (int r = 0; r <= 5; r++) known[r] = false;
            }
        }
    }

    // Early packet loads.  A "region" is a run of basic blocks entered only at its first block:
    // every later block's only predecessor is the fall-through from the block before it.  A
    // packet load in a region whose base register is not written, and with no store, call or
    // other memory-changing slot, between an earlier point of the region and the load is issued
    // at that point (into sp<prog>_<slot>_), ahead of the branches in between: the loads of
    // several headers then travel together instead of one round trip per basic block.  The
    // early load reads only the packet memory [P, P + M) of the lane (the same bounds test as
    // the fast path); the load itself still runs its full test and uses the early value only
    // when that test passes, so results never change.
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> spec_use;                  // (prog, load slot) -> size
    std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> spec_at;     // (prog, slot) -> loads issued before it
    void analyze_spec(const ProgView &p) {
        if (p.n == 0) return;
        ctx_hints(p);
        const std::vector<uint32_t> Lb = leaders(p);
        std::vector<uint32_t> preds(p.n + 1, 0);
        std::vector<bool> special(p.n + 1, false);
        special[0] = true;
        for (uint32_t i = 0; i < p.n; i++) {
            const DInsn &x = p.ins[i];
            const uint32_t h = AUX_H(x.aux);
            if ((h == H_JA || h == H_JCC || h == H_CALL_LOCAL) && (x.aux & AUX_JT_OK)) {
                const int64_t t = jump_target(x, i);
                if (t >= 0 && t <= (int64_t)p.n) {
                    preds[t]++;
                    if (h == H_CALL_LOCAL) special[t] = true;
                }
            }
            if (h == H_CALL_LOCAL) special[i + 1] = true;   // return site
            if ((!ends_block(x) || h == H_JCC || (h == H_CALL && (uint32_t)x.k == 12)) && (x.aux & AUX_FALL_OK)) preds[i + 1]++;
        }
        uint32_t def[11] = {}, kill = 0, start = 0, live = 0;
        bool mapv[11] = {};   // holds a helper's result (a map value, not a packet address)
        int last_jcc = -1;
        for (size_t b = 0; b < Lb.size(); b++) {
            const uint32_t s0 = Lb[b], e = b + 1 < Lb.size() ? Lb[b + 1] : p.n;
            const DInsn &prev = p.ins[s0 ? s0 - 1 : 0];
            const bool cont = s0 > 0 && !special[s0] && preds[s0] == 1 && (AUX_H(prev.aux) == H_JCC || !ends_block(prev)) &&
                              (prev.aux & AUX_FALL_OK);
            if (!cont) {   // a new region
                start = s0;
                kill = s0;
                for (auto &d : def) d = s0;
                for (auto &m : mapv) m = false;
                live = 0;
                last_jcc = -1;
            }
            for (uint32_t i = s0; i < e; i++) {
                const DInsn &x = p.ins[i];
                const uint32_t h = AUX_H(x.aux), d = insn_dst(x), sr = insn_src(x);
                // xdp_md: packet loads through a packet pointer; sk_buff: LD_ABS / LD_IND
                const bool xdp_ld = ctx == CTX_XDP && h == H_LDX && sr <= 10 && hint(sr) == HINT_PKT && !mapv[sr];
                const bool ind = (x.aux & AUX_X) != 0;
                const bool skb_abs = ctx == CTX_SKB && h == H_LDABS && (!ind || sr <= 10);
                if ((xdp_ld || skb_abs) && live < (uint32_t)speculate) {
                    const uint32_t hp = skb_abs && !ind ? std::max(kill, start) : std::max(std::max(def[sr], kill), start);
                    if (last_jcc >= (int)hp) {   // a branch lies between the issue point and the load
                        spec_use[{p.id, i}] = AUX_SZ(x.aux);
                        spec_at[{p.id, hp}].push_back(i);
                        live++;
                    }
                }
                switch (h) {
                case H_ALU64: case H_ALU32: case H_LDIMM: case H_LDX:
                    if (d <= 10) {
                        def[d] = i + 1;
                        mapv[d] = h == H_ALU64 && insn_op(x) == 0xbf && insn_src(x) <= 10 && mapv[insn_src(x)];
                    }
                    break;
                case H_JCC: case H_JA:
                    last_jcc = (int)i;
                    break;
                case H_NOP:
                    break;
                case H_ST: case H_STX:
                    // a store through R10 stays in the stack on its fast path; its slow path (an
                    // address outside the stack) clears spv_, which voids every early value
                    if (d == 10) break;
                    kill = i + 1;
                    for (auto &r : def) r = i + 1;
                    for (auto &m : mapv) m = false;
                    break;
                case H_LDABS:   // writes R0-R5, no memory
                    for (int r = 0; r <= 5; r++) {
                        def[r] = i + 1;
                        mapv[r] = false;
                    }
                    break;
                default:   // stores, calls, anything generic: nothing moves above it
                    kill = i + 1;
                    for (auto &r : def) r = i + 1;
                    for (auto &m : mapv) m = false;
                    if (h == H_CALL) mapv[0] = true;
                    break;
                }
            }
        }
    }
    // Cross-packet window prefetch.  When the entry program's first early-load window is made in
    // its first region from a register that provably holds `data + c` (traced from slot 0: r1 is
    // the xdp_md, a 4-byte load of its offset 0 is `data` while nothing has been stored, moves and
    // constant adds keep the form) and no slot before the window writes memory or calls, the
    // window's bytes depend only on the packet: packet j + 1's window is loaded while packet j
    // runs (its descriptor is loaded two packets ahead), and the window code takes the
    // prefetched words instead of loading them.  Every packet then waits on one dependent HBM
    // round trip less.  The prefetch only reads the packet's data bytes [0, len) (room bytes are
    // zeroed at packet start); a packet too short, a per-packet headroom array or another entry
    // program takes the normal window code.  Any jump or call to slot 0 disables it; a tail call
    // clears the flag, so only the packet's own first pass through slot 0 uses the words.
    // Lane prefetch is exact when no packet's bytes can change between the lane's start and the
    // packet's own run: no program of the set stores through a base that may be a packet pointer.
    // Every store (ST / STX / atomics) must go through R10 (+ a constant) or through a map value
    // pointer a lookup just returned; helpers other than map lookup / update / delete,
    // get_smp_processor_id and tail calls, and BPF-to-BPF calls, turn it off.
    bool lpf_safe() const {
        for (auto &p : P) {
            if (!p.n) continue;
            const std::vector<uint32_t> Lb = leaders(p);
            std::map<uint32_t, size_t> blk;
            for (size_t b = 0; b < Lb.size(); b++) blk[Lb[b]] = b;
            // per register: bit r of `ns` = may be something other than a stack or map-value pointer
            constexpr uint16_t ALLR = 0x7ff;
            std::vector<uint16_t> in(Lb.size(), 0);
            std::vector<bool> seen(Lb.size(), false);
            seen[0] = true;
            in[0] = (uint16_t)(ALLR & ~(1u << 10));
            for (bool changed = true; changed;) {
                changed = false;
                for (size_t b = 0; b < Lb.size(); b++) {
                    if (!seen[b]) continue;
                    const uint32_t s0 = Lb[b], e = b + 1 < Lb.size() ? Lb[b + 1] : p.n;
                    uint16_t ns = in[b];
                    auto bad = [&](uint32_t r) { return r > 10 || ((ns >> r) & 1); };
                    auto setb = [&](uint32_t r, bool v) {
                        if (r <= 10) ns = v ? (uint16_t)(ns | (1u << r)) : (uint16_t)(ns & ~(1u << r));
                    };
                    for (uint32_t i = s0; i < e; i++) {
                        const DInsn &x = p.ins[i];
                        const uint32_t h = AUX_H(x.aux), d = insn_dst(x), sr = insn_src(x), op = insn_op(x);
                        const bool X = (x.aux & AUX_X) != 0;
                        switch (h) {
                        case H_NOP: case H_JA: case H_JCC: case H_EXIT: case H_ERR:
                            break;
                        case H_ALU64: {   // a pointer moved, or moved by a constant, stays one
                            const uint32_t alu = op & 0xf0;
                            if (alu == 0xb0) setb(d, !X || bad(sr));
                            else if ((alu == 0x00 || alu == 0x10) && !X) setb(d, bad(d));
                            else setb(d, true);
                            break;
                        }
                        case H_ALU32: case H_LDIMM: case H_LDX:
                            setb(d, true);
                            break;
                        case H_ST: case H_STX:
                            if (bad(d)) return false;
                            break;
                        case H_CALL: {
                            const uint32_t k = (uint32_t)x.k;
                            if (k != 1 && k != 2 && k != 3 && k != 8 && k != 12) return false;
                            ns |= 0x3f;
                            if (k == 1) ns &= (uint16_t)~1u;   // R0: a map value pointer (or 0)
                            break;
                        }
                        case H_SLOW:
                            if (((op & 7) == 2 || (op & 7) == 3) && bad(d)) return false;
                            if ((op & 7) == 0 || (op & 7) == 1 || (op & 7) == 4 || (op & 7) == 7) setb(d, true);
                            break;
                        default:   // BPF-to-BPF calls, LD_ABS / LD_IND
                            return false;
                        }
                    }
                    const DInsn &last = p.ins[e - 1];
                    const uint32_t lh = AUX_H(last.aux);
                    std::vector<int64_t> succ;
                    if ((!ends_block(last) || lh == H_JCC) && (last.aux & AUX_FALL_OK)) succ.push_back(e);
                    if ((lh == H_JA || lh == H_JCC) && (last.aux & AUX_JT_OK)) succ.push_back(jump_target(last, e - 1));
                    for (int64_t sx : succ) {
                        auto it = blk.find((uint32_t)sx);
                        if (it == blk.end()) continue;
                        const uint16_t nin = (uint16_t)(in[it->second] | ns);
                        if (!seen[it->second] || nin != in[it->second]) {
                            in[it->second] = nin;
                            seen[it->second] = true;
                            changed = true;
                        }
                    }
                }
            }
        }
        return true;
    }
    void analyze_xpf() {
        if (!(xpf_knob || lpf_knob) || ctx != CTX_XDP || !prefetch || !window || stage || !fast_paths) return;
        for (auto &p : P) {
            if (p.n == 0) continue;
            bool to0 = false;
            std::vector<uint32_t> preds(p.n + 1, 0);
            std::vector<bool> special(p.n + 1, false);
            for (uint32_t i = 0; i < p.n; i++) {
                const DInsn &x = p.ins[i];
                const uint32_t h = AUX_H(x.aux);
                if ((h == H_JA || h == H_JCC || h == H_CALL_LOCAL) && (x.aux & AUX_JT_OK)) {
                    const int64_t t = jump_target(x, i);
                    if (t == 0) to0 = true;
                    if (t >= 0 && t <= (int64_t)p.n) {
                        preds[t]++;
                        if (h == H_CALL_LOCAL) special[t] = true;
                    }
                }
                if (h == H_CALL_LOCAL) special[i + 1] = true;
                if ((!ends_block(x) || h == H_JCC || (h == H_CALL && (uint32_t)x.k == 12)) && (x.aux & AUX_FALL_OK)) preds[i + 1]++;
            }
            if (to0) continue;
            // the first issue point of the program's early loads
            uint32_t hp = UINT32_MAX;
            for (auto &s : spec_at)
                if (s.first.first == p.id) hp = std::min(hp, s.first.second);
            if (hp == UINT32_MAX) continue;
            // symbolic scan of slots [0, hp): 0 unknown, 1 the xdp_md, 2 data + rel[r]
            int kind[11] = {};
            int64_t rel[11] = {};
            kind[1] = 1;
            bool ok = true;
            for (uint32_t i = 1; i <= hp; i++) {   // slots 1..hp are reached only by falling through
                const DInsn &prev = p.ins[i - 1];
                if (special[i] || preds[i] != 1 || !(AUX_H(prev.aux) == H_JCC || !ends_block(prev)) || !(prev.aux & AUX_FALL_OK)) ok = false;
            }
            for (uint32_t i = 0; i < hp && ok; i++) {
                const DInsn &x = p.ins[i];
                const uint32_t h = AUX_H(x.aux), op = insn_op(x), d = insn_dst(x), sr = insn_src(x);
                switch (h) {
                case H_NOP: case H_JCC: break;
                case H_ALU64:
                    if (d > 10) { ok = false; break; }
                    if (op == 0xbf && sr <= 10) { kind[d] = kind[sr]; rel[d] = rel[sr]; }
                    else if (op == 0x07 && kind[d] == 2) rel[d] += (int64_t)(int32_t)(uint32_t)x.k;
                    else kind[d] = 0;
                    break;
                case H_ALU32: case H_LDIMM:
                    if (d > 10) { ok = false; break; }
                    kind[d] = 0;
                    break;
                case H_LDX:
                    if (d > 10 || sr > 10) { ok = false; break; }
                    if (op == 0x61 && kind[sr] == 1 && insn_off(x) == 0) { kind[d] = 2; rel[d] = 0; }
                    else kind[d] = 0;
                    break;
                default: ok = false;   // stores, calls, jumps, exits: not traced
                }
            }
            if (!ok) continue;
            // the window group the emitter makes at hp (emit_spec's grouping)
            std::map<uint32_t, std::vector<uint32_t>> by_base;
            for (uint32_t j : spec_at[{p.id, hp}])
                if (AUX_H(p.ins[j].aux) != H_LDABS) by_base[insn_src(p.ins[j])].push_back(j);
            for (auto &bb : by_base) {
                int64_t lo = INT64_MAX, hi = INT64_MIN;
                for (uint32_t j : bb.second) {
                    lo = std::min<int64_t>(lo, insn_off(p.ins[j]));
                    hi = std::max<int64_t>(hi, (int64_t)insn_off(p.ins[j]) + AUX_SZ(p.ins[j].aux));
                }
                if (bb.second.size() < 2 || hi - lo > 32 || kind[bb.first] != 2) continue;
                const int64_t off = rel[bb.first] + lo;
                if (off < 0 || off > 4096) continue;
                xpf.on = true;
                xpf.prog = p.id;
                xpf.hp = hp;
                xpf.base = bb.first;
                xpf.off = off;
                xpf.words = (uint32_t)((hi - lo + 7) / 8);
                return;
            }
        }
    }
    // Lane value cache.  One lane runs every packet of its vCPU, so the lane's row of a per-CPU
    // array (vCPU c's E * S bytes, at most 32) is touched by no other lane during a launch: the
    // row is loaded into four registers when the lane starts, loads and stores that fall inside it
    // become register operations, and it is written back once when the lane ends (only if it was
    // written).  Before any cold path (which may touch the row in memory: map update, generic
    // loads and stores) the row is written back and the cache is switched off for the rest of the
    // lane.  The cached map is the one named by the map hint of the first helper-1 site whose R1
    // comes from an LD_IMM64 in the same block that names a per-CPU array with E * S <= 32, a
    // multiple of 8 (vc_ok, from the VM's maps: the choice is part of the source, so kernels for
    // other maps carry no cache registers); the row is cached when the lane's CPU ID is in [0, V)
    // (the map is checked again at run time).
    // cfg 2 measured: one 32-byte load and store per vCPU instead of a counter read-modify-write
    // (and its L2 write-back) per packet.
    void analyze_vc() {
        if (!vc_knob || !fast_paths) return;
        for (auto &p : P) {
            if (p.n == 0) continue;
            const std::vector<uint32_t> Lb = leaders(p);
            size_t b = 0;
            for (uint32_t i = 0; i < p.n; i++) {
                while (b + 1 < Lb.size() && Lb[b + 1] <= i) b++;
                const DInsn &x = p.ins[i];
                if (AUX_H(x.aux) != H_CALL || (uint32_t)x.k != 1) continue;
                const uint32_t save = blk_start;
                blk_start = Lb[b];
                const int64_t j = r1_def(p, i);
                blk_start = save;
                if (j >= 0 && vc_ok.count(p.base + (uint32_t)j)) {
                    vc_on = true;
                    vc_slot = p.base + (uint32_t)j;
                    vc_rb = vc_ok.at(vc_slot);
                    vc_lds = vc_rb > 32;
                    return;
                }
            }
        }
    }
    // Spread mode.  processPool gives each vCPU one worker (vm.go:548-573), so the engine runs a
    // vCPU's packets on one lane, in order -- with V = runtime.NumCPU() (vm.go:64) a few hundred
    // lanes for a whole GPU.  When the only per-CPU state the programs touch is counters they
    // increment (fused increments, fusable_inc) through a lookup of one per-CPU array, and no
    // other memory, register or helper sees the looked-up value region, a vCPU's final counters
    // are the sum of its packets' increments in any order, and each packet's R0 / status / steps
    // depend on its own bytes only: then a vCPU's packets may run on many lanes at once.  Checked
    // here over every program: a forward may-analysis of the registers that may hold a value
    // pointer from such a lookup (taint); a value pointer may be compared, copied, moved by
    // arithmetic, returned in R0 (the address is a function of the packet's vCPU and key), and be
    // the base of a fused increment -- nothing else (no load or store through it, no store of it,
    // no helper argument).  Allowed helpers: map_lookup_elem on that per-CPU array (R1 an
    // LD_IMM64 of its object in the block) and get_smp_processor_id; no tail calls, BPF-to-BPF
    // calls or loops (no budget checks).  Every other load or store must go through a base the
    // analysis can place (base provenance, `u` below): derived from R1 (the xdp_md context), R10 (the
    // stack) or a packet pointer loaded from the context's data / data_end / data_meta fields.  A
    // base built from an LD_IMM64 constant, loaded from memory, returned by a helper or computed from
    // scalars alone may address per-CPU memory (memory_controller.go:117-145 resolves any address),
    // so such a program set runs one lane per vCPU.  resolve()'s SPREAD_GUARD stays as an internal
    // assertion of this analysis.
    bool analyze_spread() {
        if (!spread_req || ctx != CTX_XDP || !fast_paths || !cold_inline || careful_copies || any_local || any_tail ||
            stage || census || !inc_knob || live.empty())
            return false;
        int64_t map = -1;
        uint32_t n = 0;
        for (auto &p : P) {
            if (!p.n) continue;
            const std::vector<uint32_t> Lb = leaders(p);
            std::map<uint32_t, size_t> blk;
            for (size_t b = 0; b < Lb.size(); b++) blk[Lb[b]] = b;
            // may-sets per register (bit r): t = may hold a value pointer of the spread map's
            // lookup; u = may be an address of unknown provenance; nc = may not be the context pointer
            constexpr uint16_t ALLR = 0x7ff;
            std::vector<uint16_t> in(Lb.size(), 0), in_u(Lb.size(), 0), in_nc(Lb.size(), 0);
            std::vector<bool> seen(Lb.size(), false);
            seen[0] = true;
            in_u[0] = (uint16_t)(ALLR & ~((1u << 1) | (1u << 10)));
            in_nc[0] = (uint16_t)(ALLR & ~(1u << 1));
            for (bool changed = true; changed;) {
                changed = false;
                for (size_t b = 0; b < Lb.size(); b++) {
                    if (!seen[b]) continue;
                    const uint32_t s0 = Lb[b], e = b + 1 < Lb.size() ? Lb[b + 1] : p.n;
                    uint16_t t = in[b], u = in_u[b], nc = in_nc[b];
                    auto tn = [&](uint32_t r) { return r <= 10 && ((t >> r) & 1); };
                    auto un = [&](uint32_t r) { return r > 10 || ((u >> r) & 1); };
                    auto setb = [](uint16_t &m, uint32_t r, bool v) {
                        if (r <= 10) m = v ? (uint16_t)(m | (1u << r)) : (uint16_t)(m & ~(1u << r));
                    };
                    for (uint32_t i = s0; i < e; i++) {
                        const DInsn &x = p.ins[i];
                        const uint32_t h = AUX_H(x.aux), d = insn_dst(x), sr = insn_src(x), op = insn_op(x);
                        const bool X = (x.aux & AUX_X) != 0;
                        switch (h) {
                        case H_NOP: case H_JA: case H_JCC: case H_EXIT: case H_ERR:
                            break;
                        case H_ALU64: case H_ALU32: {
                            if (d > 10) break;
                            const bool mov = (op & 0xf0) == 0xb0;
                            const bool v = (X && tn(sr)) || (!mov && tn(d));
                            t = v ? (uint16_t)(t | (1u << d)) : (uint16_t)(t & ~(1u << d));
                            // provenance: a move copies it (an immediate has none); arithmetic keeps the
                            // pointer operand's (pointer + scalar), scalars alone have none
                            if (mov) setb(u, d, !X || un(sr));
                            else setb(u, d, un(d) && (!X || un(sr)));
                            setb(nc, d, !mov || !X || ((nc >> sr) & 1));
                            break;
                        }
                        case H_LDIMM:   // a constant (map object, map value address, number): no provenance
                            if (d <= 10) t &= (uint16_t)~(1u << d);
                            setb(u, d, true);
                            setb(nc, d, true);
                            break;
                        case H_LDX:
                            if (tn(sr)) {   // through a value pointer: a fused increment, nothing else
                                if (!(i + 2 < e && fusable_inc(p, i))) return false;
                                const uint32_t w = AUX_SZ(x.aux);
                                if (n && n != w) return false;
                                n = w;
                                t &= (uint16_t)~(1u << d);   // the counter register, dead after the store
                                setb(u, d, true);
                                setb(nc, d, true);
                                i += 2;
                                break;
                            }
                            if (un(sr)) return false;   // a base of unknown provenance
                            if (d <= 10) t &= (uint16_t)~(1u << d);
                            // the xdp_md packet pointers (data, data_end, data_meta: context_xdp_md.go:
                            // 117-133) keep a provenance; any other loaded value has none
                            setb(u, d, !(sr <= 10 && !((nc >> sr) & 1) && (insn_off(x) == 0 || insn_off(x) == 4 || insn_off(x) == 8)));
                            setb(nc, d, true);
                            break;
                        case H_ST: case H_STX:
                            if (tn(d)) return false;                  // a store through a value pointer
                            if (h == H_STX && tn(sr)) return false;   // a value pointer stored to memory
                            if (un(d)) return false;                  // a base of unknown provenance
                            break;
                        case H_CALL: {
                            const uint32_t k = (uint32_t)x.k;
                            u |= 0x3f;   // R0 - R5 after a helper: a result or clobbered
                            nc |= 0x3f;
                            if (k == 8) {   // get_smp_processor_id: R0 = the packet's vCPU
                                t &= (uint16_t)~1u;
                                break;
                            }
                            if (k != 1 || tn(1) || tn(2)) return false;
                            const uint32_t save = blk_start;
                            blk_start = s0;
                            const int64_t j = r1_def(p, i);
                            blk_start = save;
                            if (j < 0) return false;
                            auto it = spread_req->slot_map.find(p.base + (uint32_t)j);
                            if (it == spread_req->slot_map.end() || (map >= 0 && map != (int64_t)it->second)) return false;
                            map = it->second;
                            t |= 1u;   // R0: the value pointer (or 0)
                            break;
                        }
                        case H_SLOW:
                            if ((op & 7) == 1) return false;   // an LDX error form (generic load)
                            // ST / STX class forms (atomics ...): a store through dst
                            if (((op & 7) == 2 || (op & 7) == 3) && (tn(d) || un(d))) return false;
                            if (d <= 10) t = (tn(d) || (X && tn(sr))) ? (uint16_t)(t | (1u << d)) : (uint16_t)(t & ~(1u << d));
                            if ((op & 7) == 0 || (op & 7) == 4 || (op & 7) == 7) {   // LD / ALU forms: no provenance kept
                                setb(u, d, true);
                                setb(nc, d, true);
                            }
                            break;
                        default:   // LD_ABS / LD_IND, BPF-to-BPF
                            return false;
                        }
                    }
                    const DInsn &last = p.ins[e - 1];
                    const uint32_t lh = AUX_H(last.aux);
                    std::vector<int64_t> succ;
                    if ((!ends_block(last) || lh == H_JCC) && (last.aux & AUX_FALL_OK)) succ.push_back(e);
                    if ((lh == H_JA || lh == H_JCC) && (last.aux & AUX_JT_OK)) succ.push_back(jump_target(last, e - 1));
                    for (int64_t sx : succ) {
                        auto it = blk.find((uint32_t)sx);
                        if (it == blk.end()) continue;
                        const size_t q = it->second;
                        const uint16_t nin = (uint16_t)(in[q] | t), nu = (uint16_t)(in_u[q] | u), nn = (uint16_t)(in_nc[q] | nc);
                        if (!seen[q] || nin != in[q] || nu != in_u[q] || nn != in_nc[q]) {
                            in[q] = nin;
                            in_u[q] = nu;
                            in_nc[q] = nn;
                            seen[q] = true;
                            changed = true;
                        }
                    }
                }
            }
        }
        if (map < 0 || !n) return false;
        auto sh = spread_req->shape.find((uint32_t)map);
        if (sh == spread_req->shape.end() || sh->second.first == 0 || sh->second.first % n) return false;
        spread_map = (uint32_t)map;
        spread_n = n;
        spread_row = sh->second.first;
        return true;
    }
    // issue the prefetch of the window of the packet at (noff_, nlen_)
    void emit_xpf_issue(const char *pre) {
        E.line("%sif (xpf_on_ && nidx_ != NO_PKT && %uu <= nlen_) {", pre, (uint32_t)xpf.off + 8 * xpf.words);
        E.line("%s  const uint8_t *xp_ = kp.pkt_data + noff_ + kp.headroom + %uu;", pre, (uint32_t)xpf.off);
        for (uint32_t q = 0; q < xpf.words; q++) E.line("%s  xn%u_ = ld_n(xp_ + %uu, 8u);", pre, q, 8 * q);
        E.line("%s  xn_ok_ = 1u; } else xn_ok_ = 0u;", pre);
    }
    void emit_spec_one(const ProgView &p, uint32_t j, const char *pre) {
        const DInsn &x = p.ins[j];
        const uint32_t n = AUX_SZ(x.aux);
        if (AUX_H(x.aux) == H_LDABS) {   // packet bytes at 32 + imm (+ index register), BigEndian applied at the use
            const bool ind = (x.aux & AUX_X) != 0;
            E.line("%sga_ = (uint32_t)%s%s;   // early LD_ABS for slot %u", pre, imm(x.k).c_str(), ind ? (" + (uint32_t)" + reg(insn_src(x))).c_str() : "", j);
            E.line("%sif ((uint64_t)(uint32_t)(%uu + ga_) + %uu <= L.M) sp%u_%u_ = (%s)ld_n(L.pkt + (uint32_t)(%uu + ga_), %uu);", pre,
                   SKB_HEADROOM_J, n, p.id, j, n == 8 ? "uint64_t" : "uint32_t", SKB_HEADROOM_J, n);
            return;
        }
        E.line("%sga_ = %s;   // early load for slot %u", pre, addr(insn_src(x), insn_off(x)).c_str(), j);
        E.line("%sif ((uint64_t)(uint32_t)(ga_ - P) + %uu <= L.M) sp%u_%u_ = (%s)%s(L.pkt + (uint32_t)(ga_ - P), %uu);", pre, n, p.id, j,
               n == 8 ? "uint64_t" : "uint32_t", nt ? "ld_n_nt" : "ld_n", n);
    }
    // Early loads from one base register that fall in a 32-byte span are made as one window of
    // 8-byte loads (fewer memory instructions per packet); the fields are cut out of the window
    // with constant shifts.  A packet too short for the whole window takes the loads one by one.
    void emit_spec(const ProgView &p, uint32_t i) {
        auto it = spec_at.find({p.id, i});
        if (it == spec_at.end()) return;
        std::map<uint32_t, std::vector<uint32_t>> by_base;
        for (uint32_t j : it->second) {
            if (AUX_H(p.ins[j].aux) == H_LDABS) emit_spec_one(p, j, "    ");
            else by_base[insn_src(p.ins[j])].push_back(j);
        }
        for (auto &bb : by_base) {
            const std::vector<uint32_t> &js = bb.second;
            int64_t lo = INT64_MAX, hi = INT64_MIN;
            for (uint32_t j : js) {
                lo = std::min<int64_t>(lo, insn_off(p.ins[j]));
                hi = std::max<int64_t>(hi, (int64_t)insn_off(p.ins[j]) + AUX_SZ(p.ins[j].aux));
            }
            if (!window || js.size() < 2 || hi - lo > 32) {
                for (uint32_t j : js) emit_spec_one(p, j, "    ");
                continue;
            }
            const uint32_t words = (uint32_t)((hi - lo + 7) / 8);
            auto cut = [&](const char *wn) {   // the fields out of the window words <wn><q>_
                const std::string w(wn);
                for (uint32_t j : js) {
                    const uint32_t o = (uint32_t)(insn_off(p.ins[j]) - lo), n = AUX_SZ(p.ins[j].aux), q = o / 8, r = o % 8;
                    std::string v = r == 0 ? w + std::to_string(q) + "_" : "(" + w + std::to_string(q) + "_ >> " + std::to_string(8 * r) + ")";
                    if (r + n > 8) v = "(" + v + " | (" + w + std::to_string(q + 1) + "_ << " + std::to_string(64 - 8 * r) + "))";
                    if (n < 8) v = "(" + v + " & 0x" + (n == 1 ? std::string("ffull") : n == 2 ? std::string("ffffull") : std::string("ffffffffull")) + ")";
                    E.line("        sp%u_%u_ = (%s)%s;", p.id, j, n == 8 ? "uint64_t" : "uint32_t", v.c_str());
                }
            };
            E.line("    { const uint32_t wo_ = %s - P;   // window of %u bytes for slots", addr(bb.first, (int32_t)lo).c_str(), 8 * words);
            if (xpf.on && p.id == xpf.prog && i == xpf.hp && bb.first == xpf.base && words == xpf.words) {
                E.line("      if (xc_ok_) {   // prefetched while the previous packet ran (analyze_xpf)");
                E.line("        xc_ok_ = 0u;");
                cut("xc");
                E.line("      } else");
            }
            E.line("      if ((uint64_t)wo_ + %uu <= L.M) {", 8 * words);
            for (uint32_t q = 0; q < words; q++)
                E.line("        const uint64_t w%u_ = %s(L.pkt + wo_ + %uu, 8u);", q, nt ? "ld_n_nt" : "ld_n", 8 * q);
            cut("w");
            E.line("      } else {");
            for (uint32_t j : js) emit_spec_one(p, j, "        ");
            E.line("      } }");
        }
    }

    void program(const ProgView &p) {
        if (p.n == 0) return;
        ctx_hints(p);
        cur_prog = p.id;
        if (proc) E.line("#undef PGID_\n#define PGID_ %uu", p.id);
        std::vector<uint32_t> L = leaders(p);
        for (int careful = 0; careful < (careful_copies ? 2 : 1); careful++) {
            for (size_t b = 0; b < L.size(); b++) {
                const uint32_t s = L[b], e = b + 1 < L.size() ? L[b + 1] : p.n;
                blk_start = s;
                if (!careful) {
                    E.line("  P%u_%u:", p.id, s);
                    if (careful_copies) E.line("    if (steps + %uu > kp.budget) goto C%u_%u;", e - s, p.id, s);
                    // Run(ctx) inside a long process (loops, calls): a block that crosses a multiple
                    // of 4096 steps reads the context again and stops before its first step once done
                    if (careful_copies && ctx_check)
                        E.line("    if (((steps + %uu) ^ steps) >> 12) { const uint32_t cz_ = ctx_done(kp, i); "
                               "if (cz_) TERM(MIMIC_ERR_CANCELED - 1u + cz_, %u); }", e - s, s);
                } else {
                    E.line("  C%u_%u:", p.id, s);
                }
                for (uint32_t i = s; i < e; i++) {
                    if (careful) E.line("    if (steps == kp.budget) TERM(MIMIC_ERR_STEP_LIMIT, %u);", i);
                    emit_spec(p, i);
                    if (!careful && i + 2 < e && fusable_inc(p, i)) {
                        emit_inc(p, i);
                        i += 2;
                        continue;
                    }
                    insn(p, i);
                }
                // falling off the end of the block
                const DInsn &last = p.ins[e - 1];
                if (!ends_block(last) || AUX_H(last.aux) == H_JCC ||
                    (AUX_H(last.aux) == H_CALL && (uint32_t)last.k == 12))
                    fall(p, e - 1);
            }
        }
    }

    // the branch prefix of a slow path: "else " (or an if's condition) gets [[unlikely]], so the
    // compiler lays the slow path out after the hot code (branch weights) instead of between its blocks
    std::string unl(const std::string &pre) const {
        if (!hint_knob) return pre;
        return pre.size() >= 5 && pre.compare(pre.size() - 5, 5, "else ") == 0 ? pre + "[[unlikely]] " : pre;
    }
    // the slow path of slot i of the program being emitted: a call (COLD_CALL) or a deferral
    std::string cold(const std::string &call, uint32_t i) const {
        if (defer_mode) return defer_text(i);
        return "COLD_CALL(" + call + ", " + std::to_string(i) + ");";
    }
    std::string defer_text(uint32_t i) const {
        const uint16_t m = defer_noregs == 1 || defer_noregs == 10 + (int)cur_prog ? 0 : live.at(cur_prog).at(i) | 1u | (1u << 10);
        std::string t = "{ DeferRec *dr_ = kp.defer + g;";
        for (uint32_t r = 0; r < 11; r++)
            if ((m >> r) & 1) t += " dr_->r[" + std::to_string(r) + "] = " + (defer_noregs == 2 && r ? "(uint32_t)" : "") + "r" + std::to_string(r) + ";";
        return t + " DFR(" + std::to_string(i) + "u, " + std::to_string(cur_prog) + "u); }";
    }
    // Registers live into each slot (backward dataflow over every program; a tail call continues
    // in any program's entry): what the interpreter may read when it resumes a process deferred
    // at that slot.  R0 is always live (every error stores it as the result), R10 too (the frame
    // pointer).  With BPF-to-BPF calls every register is taken as live.
    void analyze_live() {
        const uint16_t ALL = 0x7ff;
        live.assign(P.size(), {});
        for (auto &p : P) live[p.id].assign(p.n, any_local ? ALL : 0);
        if (any_local) return;
        auto bit = [](uint32_t r) -> uint16_t { return r <= 10 ? (uint16_t)(1u << r) : (uint16_t)0; };
        auto use_def = [&](const DInsn &x, uint16_t &use, uint16_t &def) {
            const uint32_t h = AUX_H(x.aux), d = insn_dst(x), sr = insn_src(x);
            const uint16_t xs = (x.aux & AUX_X) ? bit(sr) : 0;
            use = def = 0;
            switch (h) {
            case H_ALU64: case H_ALU32:
                use = ((insn_op(x) & 0xf0) == 0xb0 ? 0 : bit(d)) | xs;
                def = bit(d);
                break;
            case H_LDIMM: def = bit(d); break;
            case H_JCC: use = bit(d) | xs; break;
            case H_LDX: use = bit(sr); def = bit(d); break;
            case H_ST: use = bit(d); break;
            case H_STX: use = bit(d) | bit(sr); break;
            case H_EXIT: use = 1; break;
            case H_CALL:   // what the interpreter's helper reads (interp.hip H_CALL); helpers keep R1-R5 (Q8)
                switch ((uint32_t)x.k) {
                case 1: case 3: use = bit(1) | bit(2); break;
                case 2: use = bit(1) | bit(2) | bit(3); break;
                case 12: use = bit(2) | bit(3); break;
                case 65: use = bit(1); break;
                default: break;
                }
                break;
            case H_LDABS: use = bit(6) | xs; def = 0x3f; break;  // R0 loaded, R1-R5 zeroed
            case H_SLOW: case H_CALL_LOCAL: use = ALL; break;
            default: break;                                  // NOP, JA, ERR
            }
        };
        for (bool changed = true; changed;) {
            changed = false;
            uint16_t entry = 0;
            for (auto &p : P)
                if (p.n) entry |= live[p.id][0];
            for (auto &p : P) {
                for (int64_t i = (int64_t)p.n - 1; i >= 0; i--) {
                    const DInsn &x = p.ins[i];
                    const uint32_t h = AUX_H(x.aux);
                    uint16_t out = 0;
                    auto succ = [&](int64_t t) { if (t >= 0 && t < (int64_t)p.n) out |= live[p.id][t]; };
                    const bool fall = (x.aux & AUX_FALL_OK) != 0;
                    if (h == H_JA || h == H_JCC) {
                        if (h == H_JCC && fall) succ(i + 1);
                        if (x.aux & AUX_JT_OK) succ(jump_target(x, i));
                    } else if (h != H_EXIT && h != H_ERR) {
                        if (fall) succ(i + 1);
                        if (h == H_CALL && (uint32_t)x.k == 12) out |= entry;
                    }
                    uint16_t use, def;
                    use_def(x, use, def);
                    const uint16_t in = (uint16_t)(use | (out & ~def) | 1u);
                    if (in != live[p.id][i]) {
                        live[p.id][i] = in;
                        changed = true;
                    }
                }
            }
        }
    }

    // Counter increments.  `ldx rD, [rB + o]; add rD, k; stx [rB + o], rD` (4 or 8 bytes, one
    // basic block, rD dead after the store) on a map value is a read-modify-write of one word: its
    // load is a dependent memory round trip the lane waits for before the store can go.  When the
    // word lies in the value region the last lookup returned (the translation cache, where the
    // three slots' fast paths would go) it is one atomic add without return instead -- the lane
    // does not wait.  Equivalent for the lane's own sequence: a per-CPU row is touched by its lane
    // only; a shared map's word is raced by other vCPUs either way (processPool), and the add is
    // one of the interleavings.  Anything else (packet, stack, cached row, other entries,
    // unaligned) takes the three slots as they are.  MIMIC_JIT_INC=0: never.
    bool fusable_inc(const ProgView &p, uint32_t i) const {
        if (!inc_knob || !fast_paths || live.empty()) return false;
        const DInsn &ld = p.ins[i], &ad = p.ins[i + 1], &sx = p.ins[i + 2];
        if (AUX_H(ld.aux) != H_LDX || AUX_H(sx.aux) != H_STX) return false;
        const uint32_t n = AUX_SZ(ld.aux), d = insn_dst(ld), b = insn_src(ld);
        if ((n != 4 && n != 8) || d == 0 || d > 9 || b > 9 || b == d) return false;
        const uint32_t ah = AUX_H(ad.aux);
        if (!(ah == H_ALU64 || (ah == H_ALU32 && n == 4)) || (insn_op(ad) & 0xf8) != 0x00 || (ad.aux & AUX_X) ||
            insn_dst(ad) != d)
            return false;
        if (AUX_SZ(sx.aux) != n || insn_dst(sx) != b || insn_src(sx) != d || insn_off(sx) != insn_off(ld)) return false;
        if ((ld.aux & AUX_FALL_OK) == 0 || (ad.aux & AUX_FALL_OK) == 0) return false;
        if (i + 3 < p.n && (sx.aux & AUX_FALL_OK) && ((live[p.id][i + 3] >> d) & 1)) return false;
        if (spec_use.count({p.id, i}) || spec_at.count({p.id, i + 1}) || spec_at.count({p.id, i + 2})) return false;
        if (fwd_store.count({p.id, i + 2}) || elided.count({p.id, i + 2})) return false;
        return true;
    }
    void emit_inc(const ProgView &p, uint32_t i) {
        const DInsn &ld = p.ins[i], &ad = p.ins[i + 1];
        const uint32_t n = AUX_SZ(ld.aux), d = insn_dst(ld), b = insn_src(ld);
        const std::string N = std::to_string(n) + "u";
        const uint64_t k = AUX_H(ad.aux) == H_ALU32 ? (uint32_t)ad.k : ad.k;
        E.line("    // %u..%u: counter increment of r%u (dead after): one atomic add in the lookup's value region", i, i + 2, d);
        E.line("    ga_ = %s;", addr(b, insn_off(ld)).c_str());
        std::string cond = "(uint64_t)(uint32_t)(ga_ - L.t_lo) + " + N + " < L.t_n && !((uintptr_t)(L.t_ptr + (uint32_t)(ga_ - L.t_lo)) & (" + N + " - 1u))";
        if (vc_on && vc_lds) {
            // an aligned counter in the lane's LDS row: one LDS read-modify-write (the row is the
            // lane's own vCPU's: no other lane touches it)
            E.line("    if (vcv_ && (uint64_t)(uint32_t)(ga_ - vclo_) + %s <= vcb_ && !((ga_ - vclo_) & 3u)) { steps += 3u; lvc_add(lvt_, ga_ - vclo_, %s, %s); vcd_ = 1u; }",
                   N.c_str(), N.c_str(), imm(k).c_str());
            E.line("    else");
        }
        if (vc_on) cond = "!(vcv_ && (uint64_t)(uint32_t)(ga_ - vclo_) + " + N + " <= vcb_) && " + cond;
        if (spread_on) {
            // a counter of this packet's vCPU row in the spread map: into the block's table (or one
            // agent-scope add), any other word takes the three slots (resolve() guards them)
            if (n == spread_n) {
                cond = "L.t_lo == sbase_ && (uint64_t)(uint32_t)(ga_ - L.t_lo) + " + N + " < L.t_n && !((uint32_t)(ga_ - L.t_lo) & (" + N + " - 1u))";
                E.line("    if (%s) { steps += 3u; spread_add(%s); }", cond.c_str(), imm(k).c_str());
            } else {
                E.line("    if (false) { }");
            }
        } else
        E.line("    if (%s) { steps += 3u; CNT_ADD(L.t_ptr + (uint32_t)(ga_ - L.t_lo), %s, %s); }", cond.c_str(), N.c_str(), imm(k).c_str());
        E.line("    else {");
        insn(p, i);
        insn(p, i + 1);
        insn(p, i + 2);
        E.line("    }");
    }

    // PC+1 after slot i (vm.go:328-337)
    void fall(const ProgView &p, uint32_t i) {
        if (p.ins[i].aux & AUX_FALL_OK) E.line("    goto P%u_%u;", p.id, i + 1);
        else E.line("    TERM(MIMIC_ERR_PC_OOB, %u);", i);
    }

    // a taken jump / BPF-to-BPF call from slot i
    void jump(const ProgView &p, uint32_t i) {
        const DInsn &x = p.ins[i];
        const int64_t t = jump_target(x, i);
        if (x.aux & AUX_JT_OK) E.line("goto P%u_%u;", p.id, (uint32_t)t);
        else if (x.aux & AUX_JT_NEG)  // the next Step indexes Instructions[-x] (vm.go:300)
            E.line("{ if (steps == kp.budget) TERM(MIMIC_ERR_STEP_LIMIT, %" PRId64 "); steps++; TERM(MIMIC_PANIC_PC, %" PRId64 "); }", t, t);
        else E.line("TERM(MIMIC_ERR_PC_OOB, %u);", i);
    }

    static std::string reg(uint32_t r) { return "r" + std::to_string(r); }
    static std::string imm(uint64_t k) {
        char b[40];
        snprintf(b, sizeof b, "0x%" PRIx64 "ull", k);
        return b;
    }
    std::string xop(const DInsn &x) { return (x.aux & AUX_X) ? reg(insn_src(x)) : imm(x.k); }
    static std::string addr(uint32_t r, int32_t off) {
        return "(uint32_t)(" + reg(r) + " + " + imm((uint64_t)(int64_t)off) + ")";
    }

    // Memory access fast paths.  The base register hints which per-process entry the address
    // most likely falls in (r10: the stack; a copy of the entry r1: xdp_md; anything else: the
    // packet).  The fast path is taken only when the access lies inside that entry, where it is
    // exactly what GetEntry + VMMem.Load/Store would do.  Every other access (other entries, map
    // values, errors) goes through the generic resolve().  Hints never change results.
    enum Hint { HINT_PKT, HINT_STACK, HINT_CTX };
    Hint hint(uint32_t base) const {
        if (base == 10) return HINT_STACK;
        if (base < 11 && ctx_reg[base]) return HINT_CTX;
        return HINT_PKT;
    }
    bool ctx_reg[11] = {};

    // registers that only ever hold the context pointer: r1 (never written: helpers keep it,
    // Q8) and registers whose every write is `mov rX, r1`
    void ctx_hints(const ProgView &p) {
        bool written[11] = {}, other[11] = {};
        for (uint32_t i = 0; i < p.n; i++) {
            const DInsn &x = p.ins[i];
            const uint32_t h = AUX_H(x.aux), d = insn_dst(x), op = insn_op(x);
            bool writes = h == H_ALU64 || h == H_ALU32 || h == H_LDIMM || h == H_LDX || h == H_SLOW;
            if (h == H_CALL || h == H_CALL_LOCAL) { written[0] = other[0] = true; }
            if (h == H_CALL_LOCAL || h == H_LDABS) for (int r = 0; r <= 5; r++) written[r] = other[r] = true;
            if (!writes || d > 10) continue;
            written[d] = true;
            if (!(op == 0xbf && insn_src(x) == 1)) other[d] = true;
        }
        for (int r = 0; r < 11; r++) ctx_reg[r] = false;
        // after a tail call r1 is whatever the caller left there (usually the context): a wrong
        // hint only costs the fast path, the address check keeps every access exact
        ctx_reg[1] = !written[1];
        for (int r = 2; r < 10; r++) ctx_reg[r] = written[r] && !other[r];
    }

    // fast-path conditions and values for an access of n bytes at address ga_ (see hint())
    struct Fast {
        std::string cond, val, store;
        std::string scond = "";   // the store's condition when it differs from the load's
    };
    std::vector<Fast> fast_forms(uint32_t base, uint32_t n, const std::string &v) {
        std::vector<Fast> f;
        if (!fast_paths) return f;
        const std::string N = std::to_string(n) + "u";
        switch (hint(base)) {
        case HINT_STACK:
            f.push_back({"(uint64_t)(uint32_t)(ga_ - kp.static_next) + " + N + " <= kp.stack_size",
                         "stack_load(kp, L, ga_ - kp.static_next, " + N + ")",
                         "stack_store(kp, L, ga_ - kp.static_next, " + N + ", " + v + ")"});
            break;
        case HINT_CTX:
            if (ctx == CTX_XDP)
                f.push_back({"(uint64_t)(uint32_t)(ga_ - (P + L.M + 1)) + " + N + " <= MIMIC_XDP_MD_SIZE",
                             "xdp_load(kp, L, ga_ - (P + L.M + 1), " + N + ")",
                             "xdp_store(kp, L, ga_ - (P + L.M + 1), " + N + ", " + v + ")"});
            break;  // sk_buff fields: see skb_ctx_fast()
        default: {
            const std::string o = "(uint32_t)(ga_ - " + std::string(pa()) + ")";
            // sk_buff packets: the fast STORE covers the frame only -- a store into a head- or tailroom
            // takes the generic path, which marks the batch's rooms-clean word (runtime.h
            // skb_room_mark); the same test on the loads cost the cfg-5 chain 2 VGPRs, its second wave
            if (stage) {
                const std::string wo = "(uint32_t)(ga_ - " + std::string(pa()) + " - " + std::to_string(wb()) + "u)";
                f.push_back({"(uint64_t)" + wo + " + " + N + " <= W_", ord("win_load(pwin_, tl_, " + wo + ", " + N + ")", n), ""});
            }
            f.push_back({"(uint64_t)" + o + " + " + N + " <= L.M",
                         ord(std::string(nt ? "ld_n_nt" : "ld_n") + "(L.pkt + " + o + ", " + N + ")", n),
                         "{ PKT_ST(L.pkt + " + o + ", " + N + ", " + ord(v, n) + ");" +
                             (stage ? " win_store_rel(pwin_, tl_, W_, " + o + ", " + std::to_string(wb()) + "u, " + N + ", " + ord(v, n) + ");" : "") + " }",
                         ctx == CTX_SKB ? "(uint64_t)(uint32_t)(" + o + " - SKB_HEADROOM) + " + N + " <= (L.rec->len & ~SKB_LOAD_FAILED)" : ""});
            // the lane's cached per-CPU row (analyze_vc): every access inside the row while the
            // cache is valid is served here, so memory and registers never disagree
            if (vc_on && vc_lds)
                f.push_back({"vcv_ && (uint64_t)(uint32_t)(ga_ - vclo_) + " + N + " <= vcb_",
                             "lvc_load(lvt_, ga_ - vclo_, " + N + ")",
                             "{ lvc_store(lvt_, ga_ - vclo_, " + N + ", " + v + "); vcd_ = 1u; }"});
            else if (vc_on)
                f.push_back({"vcv_ && (uint64_t)(uint32_t)(ga_ - vclo_) + " + N + " <= vcb_",
                             "vc_load(vc0_, vc1_, vc2_, vc3_, ga_ - vclo_, " + N + ")",
                             "{ vc_store(vc0_, vc1_, vc2_, vc3_, ga_ - vclo_, " + N + ", " + v + "); vcd_ = 1u; }"});
            // the map value region the last lookup returned (translation cache, resolve()):
            // [t_lo, t_lo + t_n - 1] with GetEntry's inclusive end, t_n = 0 when empty.  Not in
            // spread kernels: there that region is per-CPU memory other lanes add to, reached by
            // fused increments only (an access the generator did not prove goes to resolve()).
            if (!spread_on) f.push_back({"(uint64_t)(uint32_t)(ga_ - L.t_lo) + " + N + " < L.t_n",
                         "ld_n(L.t_ptr + (uint32_t)(ga_ - L.t_lo), " + N + ")",
                         "st_n(L.t_ptr + (uint32_t)(ga_ - L.t_lo), " + N + ", " + v + ")"});
            break;
        }
        }
        return f;
    }

    // an sk_buff field access at a constant offset: convertAccess with the offset, size and
    // direction known, which the compiler folds to the one field's code
    bool skb_field_ok(int32_t off, uint32_t n) const {
        return skb_fields && off >= 0 && (uint32_t)off < 192 && (n == 1 || n == 2 || n == 4 || n == 8);
    }

    // sk_buff programs: does `base` hold the bpf_flow_keys (1) or bpf_sock (2) pointer, read from
    // the context earlier in this basic block (LDX from flow_keys / sk)?  0 otherwise.  The
    // generated code still compares the address, so a wrong guess only costs the fast path.
    int skb_ptr_kind(uint32_t i, uint32_t base) const {
        if (ctx != CTX_SKB || !skb_fields || base > 10) return 0;
        const ProgView *pv = nullptr;
        for (auto &q : P) if (q.id == cur_prog) pv = &q;
        if (!pv) return 0;
        for (int64_t j = (int64_t)i - 1; j >= (int64_t)blk_start; j--) {
            const DInsn &x = pv->ins[j];
            const uint32_t h = AUX_H(x.aux), d = insn_dst(x);
            if (h == H_CALL || h == H_LDABS || h == H_CALL_LOCAL) return 0;
            if ((h == H_ALU64 || h == H_ALU32 || h == H_LDIMM || h == H_SLOW || h == H_LDX) && d == base) {
                if (h != H_LDX || insn_src(x) > 10 || hint(insn_src(x)) != HINT_CTX) return 0;
                const int32_t o = insn_off(x);
                return (o == 144 || o == 148) ? 1 : (o == 168 || o == 172) ? 2 : 0;
            }
        }
        return 0;
    }
    // the inline bpf_flow_keys / bpf_sock field access for a base skb_ptr_kind() recognised
    void skb_ptr_fast(uint32_t i, uint32_t base, int32_t off, uint32_t n, bool load, const std::string &v, std::string &pre) {
        const int k = fast_paths ? skb_ptr_kind(i, base) : 0;
        if (!k || off < 0 || off > (k == 1 ? 40 : 80) || !(n == 1 || n == 2 || n == 4 || n == 8)) return;
        const char *fn = k == 1 ? "fk_convert_" : "sk_convert_";
        const char *at = k == 1 ? "L.ka + SKB_SK_SIZE + 1u + " : "L.ka + ";
        const char *cu = k == 1 ? "" : "(const mimic_skb_custom *)kp.skb_custom, ";   // sk_convert_ reads a user-given SK
        if (load)
            E.line("%sif (L.rec && ga_ == %s%uu) { uint64_t v_ = 0; const int s_ = %s(*L.rec, %s%uu, %uu, v_, true); if (s_) TERM(s_, %u); %s = v_; }",
                   pre.c_str(), at, (uint32_t)off, fn, cu, (uint32_t)off, n, i, v.c_str());
        else
            E.line("%sif (L.rec && ga_ == %s%uu) { uint64_t v_ = %s; const int s_ = %s(*L.rec, %s%uu, %uu, v_, false); if (s_) TERM(s_, %u); }",
                   pre.c_str(), at, (uint32_t)off, v.c_str(), fn, cu, (uint32_t)off, n, i);
        pre = "    else ";
    }

    void load(uint32_t i, uint32_t base, int32_t off, uint32_t n, const std::string &dst) {
        E.line("    ga_ = %s;", addr(base, off).c_str());
        std::string pre = "    ";
        bool sp = spec_use.count({cur_prog, i}) > 0;
        for (auto &f : fast_forms(base, n, "")) {   // the first form of a packet access is the packet
            if (sp) sp = false, E.line("%sif (spv_ && %s) %s = sp%u_%u_;", pre.c_str(), f.cond.c_str(), dst.c_str(), cur_prog, i);
            else E.line("%sif (%s) %s = %s;", pre.c_str(), f.cond.c_str(), dst.c_str(), f.val.c_str());
            pre = "    else ";
        }
        if (fast_paths && ctx == CTX_SKB && hint(base) == HINT_CTX) {  // __sk_buff field: convertAccess directly
            if (skb_field_ok(off, n)) {   // the field the instruction names, when base is the sk_buff
                E.line("%sif (ga_ == SK_ + %uu) { uint64_t v_ = 0; const int s_ = skb_convert_(*L.rec, (const mimic_skb_custom *)kp.skb_custom, kp.skb_ifindex, L.pa + SKB_HEADROOM, "
                       "L.pa + L.M - SKB_HEADROOM - SKB_TAILROOM, L.ka, L.ka + SKB_SK_SIZE + 1, %uu, %uu, v_, true); if (s_) TERM(s_, %u); %s = v_; }",
                       pre.c_str(), (uint32_t)off, (uint32_t)off, n, i, dst.c_str());
                pre = "    else ";
            }
            if (defer_mode)   // the generic convertAccess is a call: the resume kernel runs it
                E.line("%sif ((uint32_t)(ga_ - SK_) <= SKB_STRUCT_SIZE) %s", pre.c_str(), defer_text(i).c_str());
            else
                E.line("%sif ((uint32_t)(ga_ - SK_) <= SKB_STRUCT_SIZE) { const SkbRes o_ = skb_convert(L.rec, (const mimic_skb_custom *)kp.skb_custom, kp.skb_ifindex, "
                       "L.pa + SKB_HEADROOM, L.pa + L.M - SKB_HEADROOM - SKB_TAILROOM, L.ka, L.ka + SKB_SK_SIZE + 1, ga_ - SK_, %uu, 0, true);"
                       " if (o_.st) TERM(o_.st, %u); %s = o_.v; }", pre.c_str(), n, i, dst.c_str());
            pre = "    else ";
        }
        skb_ptr_fast(i, base, off, n, true, dst, pre);
        // generic GetEntry + Load (cold, out of line)
        E.line("%s{ %s %s = sp_.v; }", unl(pre).c_str(), cold("cold_load(kp, sp_, ga_, " + std::to_string(n) + "u)", i).c_str(), dst.c_str());
    }

    void store(uint32_t i, uint32_t base, int32_t off, uint32_t n, const std::string &val, bool deferred = false) {
        if (!deferred && fwd_store.count({cur_prog, i})) E.line("    fwd%u_%u_ = (uint32_t)(%s);", cur_prog, i, val.c_str());
        E.line("    ga_ = %s;", addr(base, off).c_str());
        if (!deferred && elided.count({cur_prog, i})) {   // the write happens in the lookup's cold path
            const auto f = fast_forms(base, n, val);
            E.line("    if (!(%s)) %s{ %s%s }", (f.at(0).scond.empty() ? f.at(0).cond : f.at(0).scond).c_str(), hint_knob ? "[[unlikely]] " : "", base == 10 && !spec_use.empty() ? "spv_ = 0u; " : "",
                   cold("cold_store(kp, sp_, ga_, " + std::to_string(n) + "u, " + val + ")", i).c_str());
            return;
        }
        std::string pre = "    ";
        for (auto &f : fast_forms(base, n, val)) {
            if (f.store.empty()) continue;
            E.line("%sif (%s) { %s; }", pre.c_str(), (f.scond.empty() ? f.cond : f.scond).c_str(), f.store.c_str());
            pre = "    else ";
        }
        if (fast_paths && ctx == CTX_SKB && hint(base) == HINT_CTX) {
            if (skb_field_ok(off, n)) {
                E.line("%sif (ga_ == SK_ + %uu) { uint64_t v_ = %s; const int s_ = skb_convert_(*L.rec, (const mimic_skb_custom *)kp.skb_custom, kp.skb_ifindex, L.pa + SKB_HEADROOM, "
                       "L.pa + L.M - SKB_HEADROOM - SKB_TAILROOM, L.ka, L.ka + SKB_SK_SIZE + 1, %uu, %uu, v_, false); if (s_) TERM(s_, %u); }",
                       pre.c_str(), (uint32_t)off, val.c_str(), (uint32_t)off, n, i);
                pre = "    else ";
            }
            if (defer_mode)
                E.line("%sif ((uint32_t)(ga_ - SK_) <= SKB_STRUCT_SIZE) %s", pre.c_str(), defer_text(i).c_str());
            else
                E.line("%sif ((uint32_t)(ga_ - SK_) <= SKB_STRUCT_SIZE) { const SkbRes o_ = skb_convert(L.rec, (const mimic_skb_custom *)kp.skb_custom, kp.skb_ifindex, "
                       "L.pa + SKB_HEADROOM, L.pa + L.M - SKB_HEADROOM - SKB_TAILROOM, L.ka, L.ka + SKB_SK_SIZE + 1, ga_ - SK_, %uu, %s, false);"
                       " if (o_.st) TERM(o_.st, %u); }", pre.c_str(), n, val.c_str(), i);
            pre = "    else ";
        }
        skb_ptr_fast(i, base, off, n, false, val, pre);
        // generic GetEntry + Store (cold); the stack / xdp_md state it may change comes back
        E.line("%s{ %s%s", unl(pre).c_str(), base == 10 && !spec_use.empty() ? "spv_ = 0u; " : "",
               cold("cold_store(kp, sp_, ga_, " + std::to_string(n) + "u, " + val + ")", i).c_str());
        if (stage)  // a store that reached the packet updates the window too
            E.line("      if (sp_.po) win_store_rel(pwin_, tl_, W_, sp_.po - 1u, %uu, %uu, %s); }", wb(), n, ord(val, n).c_str());
        else E.line("    }");
    }

    void insn(const ProgView &p, uint32_t i) {
        const DInsn &x = p.ins[i];
        const uint32_t op = insn_op(x), d = insn_dst(x), s = insn_src(x);
        const int32_t off = insn_off(x);
        const uint32_t h = AUX_H(x.aux);
        if (h == H_LDIMM) E.line("    // %u: op 0x%02x dst r%u src r%u (imm from the table)", i, op, d, s);
        else E.line("    // %u: op 0x%02x dst r%u src r%u off %d imm %" PRId64, i, op, d, s, off, (int64_t)x.k);
        E.line("    steps++;");
        switch (h) {
        case H_NOP:
            break;
        case H_ERR:
            E.line("    TERM(%u, %u);", AUX_ARG(x.aux), i);
            break;
        case H_ALU64:
        case H_ALU32:
            E.line("    %s = %s(0x%02xu, %s, %s);", reg(d).c_str(), h == H_ALU64 ? "alu64" : "alu32", op & 0xf0,
                   reg(d).c_str(), xop(x).c_str());
            break;
        case H_LDIMM:  // read from the table: map relocations do not change the kernel source
            E.line("    %s = cget(kp.insns, %uu).k;", reg(d).c_str(), p.base + i);
            break;
        case H_JA:
            E.s += "    ";
            jump(p, i);
            break;
        case H_JCC:
            E.s += "    if (jcond(";
            E.s += imm(AUX_ARG(x.aux)) + ", " + reg(d) + ", " + xop(x) + ((x.aux & AUX_W32) ? ", true)) " : ", false)) ");
            jump(p, i);
            break;
        case H_LDX:
            load(i, s, off, AUX_SZ(x.aux), reg(d));
            break;
        case H_ST:
        case H_STX:
            store(i, d, off, AUX_SZ(x.aux), h == H_STX ? reg(s) : imm(x.k));
            break;
        case H_EXIT:  // inst.go:277-296
            if (!any_local) {
                E.line("    TERM(MIMIC_OK, %d);", proc ? (int)i : -1);   // Step leaves PC on the exit
                break;
            }
            E.line("    if (L.nframes > 0) {");
            E.line("      L.nframes--;");
            E.line("      const uint32_t fq = kp.priv_frame_q + L.nframes * MIMIC_FRAME_QWORDS;");
            E.line("      const uint32_t spc = (uint32_t)priv_load(kp, L.lane, fq * 8, 8);");
            E.line("      r6 = priv_load(kp, L.lane, (fq + 1) * 8, 8);");
            E.line("      r7 = priv_load(kp, L.lane, (fq + 2) * 8, 8);");
            E.line("      r8 = priv_load(kp, L.lane, (fq + 3) * 8, 8);");
            E.line("      r9 = priv_load(kp, L.lane, (fq + 4) * 8, 8);");
            E.line("      r10 = r10 - kp.frame_size;");
            E.line("      if (%uu <= spc + 1) TERM(MIMIC_ERR_PC_OOB, %u);", p.n, i);
            E.line("      switch (spc + 1) {");
            for (uint32_t a = 1; a < p.n; a++) {
                const DInsn &c = p.ins[a - 1];
                if (all_leaders || AUX_H(c.aux) == H_CALL_LOCAL) E.line("      case %u: goto P%u_%u;", a, p.id, a);
            }
            E.line("      default: TERM(MIMIC_ERR_ENGINE_HELPER, %u);", i);
            E.line("      }");
            E.line("    }");
            E.line("    TERM(MIMIC_OK, %d);", proc ? (int)i : -1);
            break;
        case H_CALL_LOCAL:  // BPF-to-BPF, inst.go:244-258
            E.line("    if (L.nframes >= MIMIC_MAX_FRAMES) TERM(MIMIC_ERR_CALL_DEPTH, %u);", i);
            E.line("    { const uint32_t fq = kp.priv_frame_q + L.nframes * MIMIC_FRAME_QWORDS;");
            E.line("      priv_store(kp, L.lane, fq * 8, 8, %uull);", i);
            E.line("      priv_store(kp, L.lane, (fq + 1) * 8, 8, r6);");
            E.line("      priv_store(kp, L.lane, (fq + 2) * 8, 8, r7);");
            E.line("      priv_store(kp, L.lane, (fq + 3) * 8, 8, r8);");
            E.line("      priv_store(kp, L.lane, (fq + 4) * 8, 8, r9);");
            E.line("      L.nframes++;");
            E.line("      r10 = r10 + kp.frame_size; }");
            E.s += "    ";
            jump(p, i);
            break;
        case H_CALL:
            helper(p, i);
            break;
        case H_LDABS:
            ldabs(p, i);
            break;
        default:
            slow(p, i);
            break;
        }
    }

    // the LD_IMM64 slot whose constant R1 still holds at slot i (same basic block, R1 not
    // written in between; helpers keep R1, Q8), or -1
    int64_t r1_def(const ProgView &p, uint32_t i) const { return reg_def(p, i, 1); }
    // the LD_IMM64 slot whose constant register r still holds at slot i (same basic block, r not
    // written in between; helpers keep R1, Q8, any other register is taken as clobbered), or -1
    int64_t reg_def(const ProgView &p, uint32_t i, uint32_t r) const {
        for (int64_t j = (int64_t)i - 1; j >= (int64_t)blk_start; j--) {
            const DInsn &x = p.ins[j];
            const uint32_t h = AUX_H(x.aux), d = insn_dst(x);
            if (h == H_LDIMM && d == r) return j;
            if ((h == H_ALU64 || h == H_ALU32 || h == H_LDX || h == H_SLOW || h == H_LDIMM) && d == r) return -1;
            if (h == H_LDABS || h == H_CALL_LOCAL) return -1;
            if (h == H_CALL && r != 1) return -1;
        }
        return -1;
    }

    void helper(const ProgView &p, uint32_t i) {  // emulator_linux_.go:125-194
        const DInsn &x = p.ins[i];
        const uint32_t h = (uint32_t)x.k;
        switch (h) {
        case 1: {
            const int64_t j = fast_paths ? r1_def(p, i) : -1;
            if (j >= 0) {  // inline array lookup when R1 is the map object the LD_IMM64 hint names
                E.line("    { const uint32_t mh_ = AUX_MAPHINT(cget(kp.insns, %uu).aux);", p.base + (uint32_t)j);
                auto f = fwd_call.find({p.id, i});
                // array maps inline (with the key forwarded from its stack store when known); then
                // hash maps inline (the key read from the stack); then the generic helper
                const std::string hfast = hash_fast ? "mh_ && hash_lookup_fast(kp, L, mh_ - 1u, r1, r2, r0)" : "false";
                if (f != fwd_call.end()) {
                    E.line("      if (!(mh_ && lookup_fast_k(kp, L, mh_ - 1u, r1, r2, r0, true, fwd%u_%u_))) {", p.id, f->second);
                    if (elided.count({p.id, f->second})) {   // the deferred stack store first: the others read the key
                        const DInsn &sx = p.ins[f->second];
                        store(f->second, insn_dst(sx), insn_off(sx), AUX_SZ(sx.aux), "fwd" + std::to_string(p.id) + "_" + std::to_string(f->second) + "_", true);
                    }
                } else {
                    E.line("      if (!(mh_ && lookup_fast(kp, L, mh_ - 1u, r1, r2, r0))) {");
                }
                E.line("      if (!(%s)) %s%s } }", hfast.c_str(), hint_knob ? "[[unlikely]] " : "", cold("cold_lookup(kp, sp_)", i).c_str());
            } else {
                E.line("    %s", cold("cold_lookup(kp, sp_)", i).c_str());
            }
            break;
        }
        case 2:
            E.line("    %s", cold("cold_update(kp, sp_)", i).c_str());
            break;
        case 3:
            E.line("    %s", cold("cold_delete(kp, sp_)", i).c_str());
            break;
        case 8:
            E.line("    r0 = (uint64_t)(int64_t)L.cpu;");
            break;
        case 12: {
            // inline when R2 is a prog-array object named by an LD_IMM64 in this block
            const int64_t j = fast_paths && tail_inline ? reg_def(p, i, 2) : -1;
            auto jump_table = [&](const char *var) {
                E.line("        L.tailcalls++;");
            if (xpf.on) E.line("        xc_ok_ = 0u;");
                E.line("        switch (%s) {", var);
                if (dispatch_on()) {
                    E.line("%s", nonempty_cases().c_str());
                    E.line("          cur_ = (uint32_t)(%s); goto D_;", var);
                } else {
                    for (auto &q : P)
                        if (q.n) E.line("        case %u: goto P%u_0;", q.id, q.id);
                }
                if (proc)   // the interpreter's process is in the (empty) program it tail-called
                    E.line("        default: st_ = MIMIC_ERR_PC_OOB; epc_ = %d; pg_ = (uint32_t)(%s) < kp.nprogs ? (uint32_t)(%s) : PGID_; goto L_term;",
                           (int)i, var, var);
                else
                    E.line("        default: TERM(MIMIC_ERR_PC_OOB, %u);", i);   // empty or unknown program
                E.line("        }");
            };
            if (j >= 0) {
                E.line("    { const uint32_t th_ = AUX_MAPHINT(cget(kp.insns, %uu).aux);", p.base + (uint32_t)j);
                E.line("      const int np_ = th_ ? tail_fast(kp, L, th_ - 1u, r2, r3, r0) : -2;");
                E.line("      if (np_ >= 0) {");
                jump_table("np_");
                E.line("      } else if (np_ == -2) {");
                E.line("      %s", cold("cold_tailcall(kp, sp_)", i).c_str());
                E.line("      if (sp_.tail) {");
                jump_table("sp_.new_prog");
                E.line("      } } }");
            } else {
                E.line("    %s", cold("cold_tailcall(kp, sp_)", i).c_str());
                E.line("    {");
                E.line("      if (sp_.tail) {");
                jump_table("sp_.new_prog");
                E.line("      }");
                E.line("    }");
            }
            break;
        }
        default:  // 65: bpf_xdp_adjust_tail (emulator_linux_helpers.go:842-864)
            E.line("    %s", cold("cold_adjust_tail(kp, sp_)", i).c_str());
            break;
        }
    }

    // LD_ABS / LD_IND (emulator_linux_.go:198-288).  Fast path: R6 is this process's sk_buff
    // and the bytes lie in its packet memory -- then the generic answer is exactly a BigEndian
    // load at packet offset 32 + x (entries are disjoint, so nothing else can match first).
    void ldabs(const ProgView &p, uint32_t i) {
        const DInsn &x = p.ins[i];
        const uint32_t n = AUX_SZ(x.aux), s = insn_src(x);
        const bool ind = (x.aux & AUX_X) != 0;
        if (ind && s > 10) {  // Registers.Get panics (after the R6 check)
            if (defer_mode) E.line("    %s", defer_text(i).c_str());
            else E.line("    { SPILL(); cold_ldabs(kp, sp_, 0u, %uu, true); FILL(); TERM(sp_.st ? sp_.st : MIMIC_PANIC_BADREG, %u); }", n, i);
            return;
        }
        const std::string N = std::to_string(n) + "u";
        E.line("    ga_ = (uint32_t)%s%s;", imm(x.k).c_str(), ind ? (" + (uint32_t)" + reg(s)).c_str() : "");
        std::string pre = "    ";
        if (ctx == CTX_SKB && fast_paths) {
            E.line("    if ((uint32_t)r6 - SK_ <= SKB_STRUCT_SIZE && (uint64_t)(uint32_t)(%uu + ga_) + %s <= L.M) {", SKB_HEADROOM_J, N.c_str());
            if (stage)
                E.line("      if ((uint64_t)ga_ + %s <= W_) r0 = %s; else r0 = %s;", N.c_str(),
                       ord("win_load(pwin_, tl_, ga_, " + N + ")", n).c_str(),
                       ord("ld_n(L.pkt + (uint32_t)(" + std::to_string(SKB_HEADROOM_J) + "u + ga_), " + N + ")", n).c_str());
            else if (spec_use.count({cur_prog, i}))
                E.line("      r0 = spv_ ? %s : %s;", ord("sp" + std::to_string(cur_prog) + "_" + std::to_string(i) + "_", n).c_str(),
                       ord("ld_n(L.pkt + (uint32_t)(" + std::to_string(SKB_HEADROOM_J) + "u + ga_), " + N + ")", n).c_str());
            else
                E.line("      r0 = %s;", ord("ld_n(L.pkt + (uint32_t)(" + std::to_string(SKB_HEADROOM_J) + "u + ga_), " + N + ")", n).c_str());
            E.line("    }");
            pre = "    else ";
        }
        E.line("%s%s", pre.c_str(), cold("cold_ldabs(kp, sp_, ga_, " + N + ", false)", i).c_str());
        E.line("    r1 = 0; r2 = 0; r3 = 0; r4 = 0; r5 = 0;");
    }

    // the interpreter's H_SLOW forms, specialised: per-lane-ordered errors and END
    void slow(const ProgView &p, uint32_t i) {
        (void)p;
        const DInsn &x = p.ins[i];
        const uint32_t op = insn_op(x), d = insn_dst(x), s = insn_src(x), cls = op & 7, hi = op & 0xf0;
        const bool xsrc = (op & 0x08) != 0;
        const int32_t off = insn_off(x);
        if (cls == 1) {  // LDX with dst >= 10: the memory error comes first, inst.go:298-318
            static const uint32_t szs[4] = {4, 2, 1, 8};
            E.line("    %s", cold("cold_load(kp, sp_, " + addr(s, off) + ", " + std::to_string(szs[(op >> 3) & 3]) + "u)", i).c_str());
            E.line("    TERM(%s, %u);", d > 10 ? "MIMIC_PANIC_BADREG" : "MIMIC_ERR_R10_WRITE", i);
            return;
        }
        if (hi == 0xd0) {  // END, inst.go:138-198 (Q4)
            if (d > 10) {
                E.line("    TERM(MIMIC_PANIC_BADREG, %u);", i);
                return;
            }
            const std::string D = reg(d);
            std::string v = D;
            if (x.k == 16) v = xsrc ? "(" + D + " & 0xffffull)" : "(((" + D + " >> 8) & 0xffull) | ((" + D + " & 0xffull) << 8))";
            else if (x.k == 32) v = xsrc ? "(" + D + " & 0xffffffffull)" : "(uint64_t)__builtin_bswap32((uint32_t)" + D + ")";
            else if (x.k == 64) v = xsrc ? "(" + D + " >> 32)" : "(uint64_t)__builtin_bswap32((uint32_t)(" + D + " >> 32))";
            if (d == 10) E.line("    TERM(MIMIC_ERR_R10_WRITE, %u);", i);
            else E.line("    %s = %s;", D.c_str(), v.c_str());
            return;
        }
        // DIV / MOD with a register divisor (per-lane Go panic)
        const bool is64 = cls == 7;
        E.line("    if (%s == 0) TERM(MIMIC_PANIC_DIV0, %u);", is64 ? reg(s).c_str() : ("(uint32_t)" + reg(s)).c_str(), i);
        if (d == 10) E.line("    TERM(MIMIC_ERR_R10_WRITE, %u);", i);
        else E.line("    %s = %s(0x%02xu, %s, %s);", reg(d).c_str(), is64 ? "alu64" : "alu32", hi, reg(d).c_str(), reg(s).c_str());
    }
};

// 128-bit name of a kernel source (+ compile options) for the on-disk code-object cache
std::string cache_name(const std::string &src, const char *const *opts, int nopts) {
    uint64_t a = 1469598103934665603ull, b = 0x9e3779b97f4a7c15ull;
    auto mix = [&](const char *p, size_t n) {
        for (size_t i = 0; i < n; i++) {
            a = (a ^ (uint8_t)p[i]) * 1099511628211ull;
            b = (b + (uint8_t)p[i]) * 0xff51afd7ed558ccdull;
            b ^= b >> 29;
        }
    };
    mix(src.data(), src.size());
    for (int i = 0; i < nopts; i++) mix(opts[i], strlen(opts[i]) + 1);
    // the embedded runtime headers are part of every kernel: a changed header is a new kernel
    for (int i = 0; i < kJitHeaderCount; i++) mix(kJitHeaderSrc[i], strlen(kJitHeaderSrc[i]));
    int maj = 0, min = 0;
    hiprtcVersion(&maj, &min);
    char v[32];
    snprintf(v, sizeof v, "rtc%d.%d", maj, min);
    mix(v, strlen(v));
    char out[48];
    snprintf(out, sizeof out, "%016" PRIx64 "%016" PRIx64 ".hsaco", a, b);
    return out;
}

// MIMIC_JIT_CACHE=dir keeps compiled kernels across processes (unset or empty: no disk cache)
std::string cache_path(const std::string &name) {
    const char *d = getenv("MIMIC_JIT_CACHE");
    if (!d || !*d) return "";
    return std::string(d) + "/" + name;
}

bool read_file(const std::string &path, std::vector<char> &out) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n > 0 && fread(out.data(), 1, (size_t)n, f) == (size_t)n;
    fclose(f);
    return ok;
}

void write_file_atomic(const std::string &path, const std::vector<char> &data) {
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    fclose(f);
    if (ok) rename(tmp.c_str(), path.c_str());
    else remove(tmp.c_str());
}

const char *const kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label", "-Wno-unused-variable", "-Wno-c++20-extensions"};
const int kNOpts = (int)(sizeof kOpts / sizeof *kOpts);

// source -> gfx950 code object (hipRTC), through the disk cache when one is configured
int build_code(const std::string &src, std::vector<char> &code, std::string *log) {
    const std::string path = cache_path(cache_name(src, kOpts, kNOpts));
    if (!path.empty() && read_file(path, code)) return 0;
    // comgr's own compile cache does not see the embedded headers change; ours (keyed on the
    // source, the options and the headers) is the only one in use
    setenv("AMD_COMGR_CACHE", "0", 0);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "mimic_jit.hip", kJitHeaderCount, kJitHeaderSrc, kJitHeaderNames) !=
        HIPRTC_SUCCESS) {
        *log = "hiprtcCreateProgram failed";
        return -1;
    }
    const hiprtcResult rc = hiprtcCompileProgram(prog, kNOpts, kOpts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string lg(ls + 1, '\0');
    if (ls) hiprtcGetProgramLog(prog, &lg[0]);
    if (rc != HIPRTC_SUCCESS) {
        *log = "hipRTC: " + std::string(hiprtcGetErrorString(rc)) + "\n" + lg;
        hiprtcDestroyProgram(&prog);
        return -1;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    if (!path.empty()) write_file_atomic(path, code);
    return 0;
}

struct CacheKey {
    int device;
    std::string src;
    bool operator<(const CacheKey &o) const { return device != o.device ? device < o.device : src < o.src; }
};
std::mutex g_mu;
std::map<CacheKey, hipFunction_t> g_cache;

}  // namespace

std::string mimic_jit_source(const std::vector<DProg> &progs, const std::vector<DInsn> &all, uint32_t ctx_kind,
                             JitInfo *info, const std::vector<std::pair<uint32_t, uint32_t>> *vc_slots, bool no_early_loads,
                             const SpreadReq *spread, bool ctx_check, bool proc) {
    std::vector<ProgView> v;
    for (size_t p = 0; p < progs.size(); p++) v.push_back(ProgView{(uint32_t)p, progs[p].n, progs[p].base, all.data() + progs[p].base});
    Gen g(v, ctx_kind);
    if (vc_slots)
        for (auto &v : *vc_slots)
            if (v.second > 0 && v.second <= MIMIC_VC_MAX_ROW && !(v.second & 7)) g.vc_ok[v.first] = v.second;
    if (no_early_loads) g.speculate = 0;
    g.spread_req = spread;
    // (MIMIC_JIT_CTXCHECK=1: the context variant from every entry point -- CPU compile tests)
    static const bool ctx_env = getenv("MIMIC_JIT_CTXCHECK") && getenv("MIMIC_JIT_CTXCHECK")[0] == '1';
    g.ctx_check = ctx_check || ctx_env;
    g.proc = proc;
    if (proc) g.inc_knob = false;
    std::string src = g.source();
    if (info) {
        info->checks_budget = g.careful_copies;
        info->max_n = g.max_n;
        info->tail_calls = g.has_tail();
        info->early_loads = g.has_early_loads();
        info->cold_inline = g.cold_inline;
        info->defer = g.defer_mode;
        info->skb_walk = g.skb_walk;
        info->skb_fast = g.skb_fast;
        info->karg = g.karg != 0;
        info->spread = g.spread_on;
        info->spread_own = g.spread_own;
        info->hash_combine = g.hash_combine;
        info->hash_chunk = g.hash_chunk;
        info->proc = proc;
        info->proc_ok = proc && ctx_kind == CTX_XDP && !g.careful_copies && !g.defer_mode && !g.spread_on && !g.census;
        info->spread_map = g.spread_map;
        info->spread_n = g.spread_n;
        info->spread_roww = g.spread_n ? g.spread_row / g.spread_n : 0;
        info->spread_rows = g.spread_on && spread ? spread->lds_rows : 0;
    }
    return src;
}

uint64_t mimic_jit_step_bound(const JitInfo &info, uint32_t max_tail_calls) {
    if (info.checks_budget) return 0;
    // a jump to a negative PC counts one more Step than the slots executed
    return (info.tail_calls ? (uint64_t)max_tail_calls + 1 : 1) * ((uint64_t)info.max_n + 1);
}

int mimic_jit_compile(int device, const std::string &src, hipFunction_t *fn, std::string *log) {
    std::lock_guard<std::mutex> lk(g_mu);
    const CacheKey key{device, src};
    auto it = g_cache.find(key);
    if (it != g_cache.end()) {
        *fn = it->second;
        return 0;
    }
    std::vector<char> code;
    if (build_code(src, code, log)) return -1;
    hipModule_t mod;
    hipError_t e = hipModuleLoadData(&mod, code.data());
    if (e != hipSuccess) {
        *log = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
        return -1;
    }
    e = hipModuleGetFunction(fn, mod, "mimic_jit_kernel");
    if (e != hipSuccess) {
        *log = std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
        return -1;
    }
    g_cache[key] = *fn;  // modules live for the process (shared by every VM with these programs)
    return 0;
}

int mimic_jit_build_code(const std::string &src, std::vector<char> &code, std::string *log) {
    return build_code(src, code, log);
}

// compile into the disk cache only (no device): prewarming for later processes
int mimic_jit_prebuild_source(const std::string &src, std::string *log) {
    std::vector<char> code;
    return build_code(src, code, log);
}

int mimic_jit_launch(hipFunction_t fn, const JitInfo &info, const KParams *kp, const KParams *d_kp, hipStream_t st) {
    const uint32_t blocks = (kp->lanes + 255) / 256;
    if (blocks == 0) return 0;
    const KParams *p = d_kp;
    void *args[] = {info.karg ? (void *)kp : (void *)&p};   // by value (kernarg segment) or a device copy
    return hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, st, args, nullptr) == hipSuccess ? 0 : -1;
}

// compile only (no device needed): the hipRTC log, for build checks and tests
int mimic_jit_check_source(const std::string &src, std::string *log, size_t *code_size) {
    setenv("AMD_COMGR_CACHE", "0", 0);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "mimic_jit.hip", kJitHeaderCount, kJitHeaderSrc, kJitHeaderNames) !=
        HIPRTC_SUCCESS)
        return -1;
    const hiprtcResult rc = hiprtcCompileProgram(prog, kNOpts, kOpts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string lg(ls + 1, '\0');
    if (ls) hiprtcGetProgramLog(prog, &lg[0]);
    *log = lg;
    if (code_size) hiprtcGetCodeSize(prog, code_size);
    hiprtcDestroyProgram(&prog);
    return rc == HIPRTC_SUCCESS ? 0 : -1;
}
