"""JIT kernel generation and hipRTC compilation on the CPU host (no device needed).

The JIT turns the loaded programs into one HIP kernel. These tests check four things:
  * the generated source compiles for gfx950;
  * the source does not depend on map relocations (LD_IMM64 constants are read from the
    instruction table), so cached kernels are shared between VMs;
  * loop-free programs get no per-instruction budget checks;
  * programs with loops or calls do.
"""
import ctypes as C

import pytest

from mimic_amd import _lib
from mimic_amd import asm as A
from mimic_amd import workloads as W


def _source(raws, ctx: int = _lib.CTX_XDP):
    lib = _lib.load()
    bufs = [C.create_string_buffer(bytes(r), max(len(r), 1)) for r in raws]
    arr = (C.c_void_p * len(raws))(*[C.cast(b, C.c_void_p) for b in bufs])
    ns = (C.c_uint32 * len(raws))(*[len(r) // 8 for r in raws])
    n = lib.mimic_jit_source_for_ctx(arr, ns, len(raws), ctx, None, 0)
    assert n > 0
    buf = C.create_string_buffer(n + 1)
    assert lib.mimic_jit_source_for_ctx(arr, ns, len(raws), ctx, buf, n + 1) == n
    return buf.value.decode()


def _compiles(src):
    lib = _lib.load()
    log = C.create_string_buffer(1 << 16)
    cs = C.c_size_t()
    rc = lib.mimic_jit_check(src.encode(), log, 1 << 16, C.byref(cs))
    assert rc == 0, log.value.decode()[:4000]
    return cs.value


@pytest.mark.parametrize("fn", ["prog_pass8", "prog_classifier"])
def test_workload_kernels_compile(fn):
    p = getattr(W, fn)()
    assert _compiles(_source([p.raw])) > 0


def test_source_independent_of_relocated_constants():
    a = A.assemble([A.ld_map_fd(1, "m"), A.mov64_imm(0, 2), A.exit_()])[0]
    b = bytearray(a)
    b[4:8] = (0x12345).to_bytes(4, "little")  # what a relocation would write
    assert _source([a]) == _source([bytes(b)])


def test_loop_free_has_no_budget_checks_and_loops_do():
    straight = A.assemble([A.mov64_imm(0, 1), A.jmp("jeq", 0, 1, "x"), A.mov64_imm(0, 3), "x", A.exit_()])[0]
    loop = A.assemble([A.mov64_imm(0, 0), "top", A.alu64("add", 0, 1), A.jmp("jlt", 0, 10, "top"), A.exit_()])[0]
    s1, s2 = _source([straight]), _source([loop])
    assert "kp.budget" not in s1
    assert "kp.budget" in s2 and "MIMIC_ERR_STEP_LIMIT" in s2
    _compiles(s2)


def test_tail_calls_and_local_calls_compile():
    main = A.assemble([A.mov64_imm(1, 0), A.call_local("f"), A.ld_map_fd(2, "p"), A.mov64_imm(3, 0), A.call(12),
                       A.exit_(), "f", A.mov64_imm(0, 7), A.exit_()])[0]
    other = A.assemble([A.alu64("add", 0, 5), A.exit_()])[0]
    src = _source([main, other, b""])
    assert "case 1: goto P1_0;" in src and "MIMIC_ERR_PC_OOB" in src
    _compiles(src)


def test_skb_chain_kernel_compiles():
    """Config 5's tail-call chain as an sk_buff-context kernel: BigEndian packet fast paths and
    LD_ABS / LD_IND over the LDS window starting at skb->data."""
    progs, _, _ = W.skb_programs()
    src = _source([p.raw for p in progs], _lib.CTX_SKB)
    assert "#define MIMIC_CTX_FIXED 1" in src and "skb_load_lds(kp, L, i, r1," in src
    assert "bswap_n(" in src
    # a kernel this size defers its slow paths to the interpreter's resume kernel (no calls)
    assert "DFR(" in src and "L_defer:" in src and "COLD_CALL(cold" not in src
    assert _compiles(src) > 0


def test_skb_chain_register_budget():
    """cfg 5's five-program chain with deferred slow paths: no call left in the kernel, so no
    scratch (the Spill record and the call ABI's saves were 240 bytes per lane) and at least two
    waves per SIMD (it was 380 VGPRs + AGPRs at one wave with called slow paths)."""
    from mimic_amd import jit as J

    progs, maps, _ = W.skb_programs()
    r = _resources([p.raw for p in progs], _lib.CTX_SKB)
    assert r["vgpr_total"] <= 256 and r["waves_per_simd"] >= 2, r
    assert r["scratch"] == 0 and r["vgpr_spill"] == 0 and r["agpr"] == 0, r
    # the kernel the cfg-5 bench runs (the per-CPU stats row in the LDS value cache): it sits at the
    # edge -- one more live value spills into AGPRs and halves the waves (0.22 -> 0.36 ms)
    vc = J.vc_slots([(p.raw, p.relocs) for p in progs], maps)
    r = _resources([p.raw for p in progs], _lib.CTX_SKB, vc)
    assert r["vgpr_total"] <= 256 and r["waves_per_simd"] >= 2 and r["agpr"] == 0, r


def test_defer_sites_store_live_registers_only():
    """A deferred slot stores the registers the interpreter can read from it on (plus R0, every
    result's value, and R10): after `mov r6, r1` at slot 0 of the chain's entry, slot 1 (a load
    through r6) needs r0, r6 and r10 only."""
    progs, _, _ = W.skb_programs()
    src = _source([p.raw for p in progs], _lib.CTX_SKB)
    site = [l for l in src.splitlines() if "DFR(1u, 0u)" in l][0]
    stored = sorted(int(x) for x in __import__("re").findall(r"dr_->r\[(\d+)\]", site))
    assert stored == [0, 6, 10], site


def test_skb_and_xdp_kernels_differ_only_in_context():
    p = W.prog_classifier()
    x, s = _source([p.raw]), _source([p.raw], _lib.CTX_SKB)
    assert "#define MIMIC_CTX_FIXED 0" in x and "#define MIMIC_CTX_FIXED 1" in s
    _compiles(s)


# ---------------------------------------------------------------------------------------------
# register budget of the generated kernels (code-object metadata of the hipRTC build): the
# kernels are latency-bound, so occupancy is what hides the per-packet HBM round trips
# ---------------------------------------------------------------------------------------------
def _resources(raws, ctx=_lib.CTX_XDP, vc=()):
    from mimic_amd import jit as J

    return J.kernel_resources(J.code_object(J.kernel_source(raws, ctx, vc)))


@pytest.mark.parametrize("fn,vgprs,waves", [("prog_classifier", 120, 4), ("prog_parse5", 120, 4)])
def test_hot_kernels_register_budget(fn, vgprs, waves):
    """cfg 2 / cfg 3 kernels as the bench's VM generates them (the classifier with its lane value
    cache): unified VGPRs within budget, no VGPR spills, no scratch.  A few SGPRs may spill (into
    VGPR lanes): keeping the per-packet result pointers in SGPRs measured faster than reloading
    them (jit.cpp, MIMIC_JIT_KQ); the generic lookup's fallback to h_find for keys over 32 bytes
    (hashmap.h h_find_ro, inlined into every kernel's cold lookup) costs the classifier 8 more.  parse5's early packet loads (jit.cpp, analyze_spec)
    cost it the fifth wave and measured faster anyway: 1.155 vs 1.193 ms per launch; forcing 5
    waves (MIMIC_JIT_WAVES=5) measured 1.47 ms.  The classifier's deferred key store
    (analyze_elide) costs it the fifth wave too and measured 29.1 vs 32.4 us per launch; its lane
    value cache (analyze_vc, 115 VGPRs) measured 25.5 vs 28.1 us."""
    from mimic_amd import jit as J

    p = getattr(W, fn)()
    r = _resources([p.raw], vc=J.vc_slots([(p.raw, p.relocs)], p.maps))
    assert r["vgpr_total"] <= vgprs and r["waves_per_simd"] >= waves, r
    assert r["vgpr_spill"] == 0 and r["sgpr_spill"] <= 12 and r["scratch"] == 0, r


def test_lane_value_cache_selection():
    """The lane value cache is generated for per-CPU arrays whose row is a multiple of 8 bytes: up
    to 32 bytes in four registers, up to 128 bytes in an LDS slot per lane."""
    from mimic_amd import jit as J

    p = W.prog_classifier()
    assert J.vc_slots([(p.raw, p.relocs)], p.maps) == [(0, 27, 32)]
    src = J.kernel_source([p.raw], 0, [(0, 27, 32)])
    assert "vc_open" in src and "lvc_open" not in src
    assert "vc_open" not in J.kernel_source([p.raw], 0, [])
    lsrc = J.kernel_source([p.raw], 0, [(0, 27, 64)])
    assert "constexpr uint32_t vcb_ = 64u;" in lsrc and "lvc_open(kp, cget(kp.maps, mh_ - 1u), L.cpu, vcb_," in lsrc and "__shared__ uint32_t lvc_[(64u / 4u + 2u) * 256u]" in lsrc
    for E, S, ok in [(4, 8, True), (2, 16, True), (1, 8, True), (5, 4, False), (8, 8, True), (16, 8, True), (17, 8, False),
                     (3, 4, False)]:
        m = dict(p.maps[0], max_entries=E, value_size=S)
        assert (J.vc_slots([(p.raw, p.relocs)], [m]) != []) == ok
    assert J.vc_slots([(p.raw, p.relocs)], [dict(p.maps[0], type=2)]) == []   # a plain array: shared by every lane


def test_small_kernel_resources():
    r = _resources([W.prog_pass8().raw])
    assert r["waves_per_simd"] == 8 and r["lds"] == 0 and r["scratch"] == 0, r


def test_cfg4_kernel_register_budget():
    """cfg 4 (hash insert) kernel: built for 4 waves per SIMD like every kernel that inlines its
    slow paths (jit.cpp), so the 262 144 lanes run in one round.  That spills about 40 VGPRs of
    its slow paths to scratch and measured faster anyway: 0.137 vs 0.172 ms per launch at its
    natural 169 VGPRs / 2 waves.  Its LDS stack window is there too, and the block
    combiner of its freelist reservations (hashmap.h h_comb_reserve: 4 x 272 bytes) and the block's
    chunk of positions (h_chunk_fill: 64 bytes)."""
    r = _resources([W.prog_flowtrack().raw])
    assert r["vgpr_total"] <= 128 and r["waves_per_simd"] >= 4 and r["lds"] == 16 * 256 * 8 + 4 * 272 + 64, r
    assert r["vgpr_spill"] <= 64, r


def test_lds_stack_window_selection():
    """The LDS stack window is generated when a stack store is made for real: not for the
    classifier (its one key store is deferred into the lookup's cold path) and not for sk_buff
    kernels (their LDS holds the SkbRec slots)."""
    from mimic_amd import jit as J

    assert "MIMIC_LDS_STACK_Q 16" in J.kernel_source([W.prog_flowtrack().raw])
    assert "MIMIC_LDS_STACK_Q" not in J.kernel_source([W.prog_classifier().raw])
    progs, _, _ = W.skb_programs()
    assert "MIMIC_LDS_STACK_Q" not in J.kernel_source([p.raw for p in progs], _lib.CTX_SKB)


def test_every_gpu_test_kernel_generates():
    """Kernel source generation (host C++: leaders, forwarding, early loads, deferred stores) for
    every program set the GPU suite compiles, so a crash in the generator shows up on the CPU."""
    import importlib

    from mimic_amd import jit as J

    count = 0
    for name in ("test_gpu_kat", "test_gpu_skb", "test_gpu_parity", "test_gpu_hash", "test_gpu_fastpaths", "test_gpu_vc"):
        mod = importlib.import_module(name)
        for k in mod.jit_kernels():
            assert "mimic_jit_kernel" in J.kernel_source(*k)
            count += 1
    assert count > 20


def test_context_variant_compiles():
    """The Run(ctx) variant (launches given contexts): a check before each process's first step,
    and in kernels with loops one at every block start that crosses a multiple of 4096 steps.
    Generated in a child process with MIMIC_JIT_CTXCHECK=1 (the knob is read once per process)."""
    import json
    import os
    import subprocess
    import sys

    loop = A.assemble([A.mov64_imm(0, 0), "top", A.alu64("add", 0, 1), A.jmp("jlt", 0, 10, "top"), A.exit_()])[0]
    straight = W.prog_classifier().raw
    code = ("import sys, json; sys.path.insert(0, 'tests'); import test_jit_cpu as t; "
            f"print(json.dumps([t._source([bytes.fromhex('{loop.hex()}')]), t._source([bytes.fromhex('{straight.hex()}')])]))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                         env=dict(os.environ, MIMIC_JIT_CTXCHECK="1"), check=True).stdout
    s_loop, s_straight = json.loads(out.strip().splitlines()[-1])
    assert s_loop.count("ctx_done(") >= 2 and ">> 12" in s_loop
    assert s_straight.count("ctx_done(") == 1
    assert "ctx_done(" not in _source([loop])
    _compiles(s_loop)
    _compiles(s_straight)
