#!/usr/bin/env python3
"""Known-answer vectors for the reference's Process.Run semantics -> tests/golden/kat.json.

The reference (Go, /root/reference) cannot be compiled or imported in this image, so its
instruction semantics are pinned here by hand: every expected value below is derived from the
cited Go line by reasoning about Go's integer semantics (conversions, unmasked shifts, panics),
written as literal numbers where a quirk is involved and as small Go-equivalent Python
expressions for the ALU matrix.  This file is independent of the C oracle (oracle/) and of the
engine; tests check both against the fixture it writes.

Run:  python tests/golden/make_golden.py   (rewrites kat.json)
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from mimic_amd import asm as A  # noqa: E402

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

# status names (shared numbering, include/mimic_amd.h)
OK, PC_OOB, UNSUP, UNRES, NOTVMMEM, BOUNDS, NOTDATASEC, R10W = 0, 1, 2, 3, 4, 5, 6, 7
MAP_PTR, KEY, VALUE, MAP_OP, TAILCALL, H_UNIMPL, H_CANT, LDABS = 8, 9, 10, 11, 12, 13, 14, 15
DIV0, SHIFT, BADREG, CALLX, PANIC_PC, HELPER_NEG, STEP_LIMIT, CALL_DEPTH, ENGINE_HELPER = (
    16, 17, 18, 19, 20, 21, 22, 23, 24)

CASES = []


def case(name, items, expect, ref, packet=b"\x00" * 64, vcpus=1, maps=(), map_init=(), prog_array=(),
         extra_progs=(), cpu=0, headroom=0, tailroom=0, ingress=0, rxq=0, egress=0, step_budget=0,
         max_tail_calls=33):
    raw, rel = A.assemble(items)
    progs = [dict(name="main", raw=raw.hex(), relocs=rel)]
    for nm, it in extra_progs:
        r2, rl2 = A.assemble(it)
        progs.append(dict(name=nm, raw=r2.hex(), relocs=rl2))
    CASES.append(dict(name=name, ref=ref, progs=progs, packet=bytes(packet).hex(), vcpus=vcpus,
                      maps=list(maps), map_init=[[m, k.hex(), v.hex(), c] for m, k, v, c in map_init],
                      prog_array=list(prog_array), cpu=cpu, headroom=headroom, tailroom=tailroom,
                      ingress=ingress, rxq=rxq, egress=egress, step_budget=step_budget,
                      max_tail_calls=max_tail_calls, expect=expect))


def e(r0=None, status=OK, steps=None, err_pc=-1):
    d = {"status": status, "err_pc": err_pc}
    if r0 is not None:
        d["r0"] = r0 & M64
    if steps is not None:
        d["steps"] = steps
    return d


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


# ------------------------------------------------------------------------------------------
# ALU matrix: r1 = a, r2 = b (LD_IMM64), then `r1 op= r2` (X) or `r1 op= imm` (K), r0 = r1
# Go expressions restated (inst_gen.go:7-225):
#   ALU32: uint64(uint32(dst) OP uint32(x));  ALU64: dst OP x, x = uint64(Constant) for K
#   shifts: Go yields 0 for counts >= width (no masking); DIV/MOD by 0 panic
# ------------------------------------------------------------------------------------------

def go_alu(op, is64, a, x):
    if is64:
        a &= M64
        x &= M64
        if op == "add": return (a + x) & M64
        if op == "sub": return (a - x) & M64
        if op == "mul": return (a * x) & M64
        if op == "div": return None if x == 0 else a // x
        if op == "mod": return None if x == 0 else a % x
        if op == "or": return a | x
        if op == "and": return a & x
        if op == "xor": return a ^ x
        if op == "lsh": return 0 if x >= 64 else (a << x) & M64
        if op == "rsh": return 0 if x >= 64 else a >> x
    else:
        a &= M32
        x &= M32
        if op == "add": return (a + x) & M32
        if op == "sub": return (a - x) & M32
        if op == "mul": return (a * x) & M32
        if op == "div": return None if x == 0 else a // x
        if op == "mod": return None if x == 0 else a % x
        if op == "or": return a | x
        if op == "and": return a & x
        if op == "xor": return a ^ x
        if op == "lsh": return 0 if x >= 32 else (a << x) & M32
        if op == "rsh": return 0 if x >= 32 else a >> x
    raise ValueError(op)


VALS = [0, 1, 5, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 0x1_0000_0001, 0x8000_0000_0000_0000, M64, 0x1234_5678_9ABC_DEF0,
        31, 32, 63, 64, 65]
IMMS = [0, 1, -1, 3, 31, 32, 63, 64, -0x80000000, 0x7FFFFFFF, 0x12345678]

for op in ("add", "sub", "mul", "div", "mod", "or", "and", "xor", "lsh", "rsh"):
    for is64 in (True, False):
        w = "alu64" if is64 else "alu32"
        for ai, a in enumerate(VALS[:10]):
            # register source
            for b in (VALS[2], VALS[7], VALS[10 + (ai % 5)], 0 if ai % 3 == 0 else VALS[ai]):
                r = go_alu(op, is64, a, b)
                items = [A.ld_imm64(1, a), A.ld_imm64(2, b),
                         (A.alu64 if is64 else A.alu32)(op, 1, 2, reg=True), A.mov64_reg(0, 1), A.exit_()]
                exp = e(r0=r, steps=7) if r is not None else e(status=DIV0, steps=5, err_pc=4)
                case(f"{w}_{op}_x_{a:x}_{b:x}", items, exp, "inst_gen.go:7-225")
            # immediate source: Constant = int64(int32(imm)); ALU64 uses uint64(Constant)
            imm = IMMS[ai % len(IMMS)]
            x = imm & M64 if is64 else imm & M32
            r = go_alu(op, is64, a, x)
            items = [A.ld_imm64(1, a), (A.alu64 if is64 else A.alu32)(op, 1, imm), A.mov64_reg(0, 1), A.exit_()]
            exp = e(r0=r, steps=5) if r is not None else e(status=DIV0, steps=3, err_pc=2)
            case(f"{w}_{op}_k_{a:x}_{imm & M32:x}", items, exp, "inst_gen.go:7-225")

# ------------------------------------------------------------------------------------------
# quirk ledger, literal expectations
# ------------------------------------------------------------------------------------------
# Q6: ALU32 NEG / ARSH sign-extend (inst.go:86-89, 116-125)
case("neg32_one", [A.mov64_imm(0, 1), A.alu32("neg", 0, 0), A.exit_()], e(r0=0xFFFFFFFFFFFFFFFF, steps=3), "inst.go:86-89")
case("neg32_min", [A.ld_imm64(0, 0x80000000), A.alu32("neg", 0, 0), A.exit_()], e(r0=0xFFFFFFFF80000000, steps=4), "inst.go:86-89")
case("neg32_hi_bits", [A.ld_imm64(0, 0xABCD_0000_0000_0002), A.alu32("neg", 0, 0), A.exit_()], e(r0=0xFFFFFFFFFFFFFFFE, steps=4), "inst.go:86-89")
case("neg64", [A.mov64_imm(0, 5), A.alu64("neg", 0, 0), A.exit_()], e(r0=-5, steps=3), "inst.go:91-94")
case("neg64_regform_0x8f", [A.mov64_imm(0, 7), A.raw(0x8F, 0, 3), A.exit_()], e(r0=-7, steps=3), "inst.go:28")
case("arsh32_k", [A.ld_imm64(0, 0x80000000), A.alu32("arsh", 0, 4), A.exit_()], e(r0=0xFFFFFFFFF8000000, steps=4), "inst.go:116-119")
case("arsh32_k_ge32", [A.ld_imm64(0, 0x80000000), A.alu32("arsh", 0, 40), A.exit_()], e(r0=M64, steps=4), "inst.go:118")
case("arsh32_k_pos_ge32", [A.mov64_imm(0, 0x7FFF), A.alu32("arsh", 0, 33), A.exit_()], e(r0=0, steps=3), "inst.go:118")
case("arsh32_x_hi_count", [A.ld_imm64(0, 0x80000000), A.ld_imm64(2, 0x1_0000_0001), A.alu32("arsh", 0, 2, reg=True), A.exit_()],
     e(r0=M64, steps=6), "inst.go:121-125 (64-bit shift count is not truncated)")
case("arsh64_k", [A.ld_imm64(0, 0x8000_0000_0000_0000), A.alu64("arsh", 0, 60), A.exit_()], e(r0=0xFFFFFFFFFFFFFFF8, steps=4), "inst.go:127-130")
case("arsh64_x_70", [A.ld_imm64(0, 0x8000_0000_0000_0000), A.mov64_imm(2, 70), A.alu64("arsh", 0, 2, reg=True), A.exit_()],
     e(r0=M64, steps=5), "inst.go:132-136")
# Q5: negative ARSH immediate panics (Go: negative shift amount)
case("arsh64_k_negative_panics", [A.mov64_imm(0, 1), A.alu64("arsh", 0, -1), A.exit_()], e(status=SHIFT, steps=2, err_pc=1), "inst.go:129")
case("arsh32_k_negative_panics", [A.mov64_imm(0, 1), A.alu32("arsh", 0, -3), A.exit_()], e(status=SHIFT, steps=2, err_pc=1), "inst.go:118")
# Q5: unmasked shifts
case("lsh64_by_64", [A.mov64_imm(0, 1), A.alu64("lsh", 0, 64), A.exit_()], e(r0=0, steps=3), "inst_gen.go:144-147")
case("lsh32_x_hi_count", [A.mov64_imm(0, 1), A.ld_imm64(2, 0x1_0000_0001), A.alu32("lsh", 0, 2, reg=True), A.exit_()],
     e(r0=2, steps=5), "inst_gen.go:149-153 (uint32(src))")
case("rsh64_neg_imm", [A.mov64_imm(0, -1), A.alu64("rsh", 0, -1), A.exit_()], e(r0=0, steps=3), "inst_gen.go:166-169 (uint64(-1) >= 64)")
# MOV (inst.go:96-114)
case("mov32_imm_neg", [A.mov32_imm(0, -1), A.exit_()], e(r0=0xFFFFFFFF, steps=2), "inst.go:96-99")
case("mov64_imm_neg", [A.mov64_imm(0, -1), A.exit_()], e(r0=M64, steps=2), "inst.go:107-109")
case("mov32_reg_trunc", [A.ld_imm64(2, 0x1234_5678_9ABC_DEF0), A.alu32("mov", 0, 2, reg=True), A.exit_()], e(r0=0x9ABCDEF0, steps=4), "inst.go:101-105")
# Q4: END (inst.go:138-198); 0xd4 = to-LE, 0xdc = to-BE, ALU32 class only
V = 0x1122_3344_AABB_CCDD
for imm, le, be in ((16, 0xDDCC, 0xCCDD), (32, 0xDDCCBBAA, 0xAABBCCDD), (64, 0x44332211, 0x11223344), (8, V, V)):
    case(f"end_le_{imm}", [A.ld_imm64(0, V), A.raw(0xD4, 0, 0, 0, imm), A.exit_()], e(r0=le, steps=4), "inst.go:138-167")
    case(f"end_be_{imm}", [A.ld_imm64(0, V), A.raw(0xDC, 0, 0, 0, imm), A.exit_()], e(r0=be, steps=4), "inst.go:169-198")
case("end64_class_unsupported", [A.ld_imm64(0, V), A.raw(0xD7, 0, 0, 0, 16), A.exit_()], e(status=UNSUP, steps=3, err_pc=2), "inst.go:45-46 (only ALU32 slots)")
case("end_r10_write", [A.raw(0xD4, 10, 0, 0, 16), A.exit_()], e(status=R10W, steps=1, err_pc=0), "vm.go:459-460")

# jumps: taken => PC += Offset, then Step's PC++ (inst_gen.go:227-605)
def jcase(name, a, b, ins, taken, ref):
    items = [A.ld_imm64(1, a), A.ld_imm64(2, b), A.mov64_imm(0, 0), ins, A.exit_(), A.mov64_imm(0, 1), A.exit_()]
    case(name, items, e(r0=1 if taken else 0, steps=8 if taken else 7), ref)


# Q1: JMP register forms compare the low 32 bits
jcase("jeq_x_low32", 0x1_0000_0005, 5, A.jmp("jeq", 1, 2, 1, reg=True), True, "inst_gen.go:618,245-253 (Q1)")
jcase("jgt_x_low32", 0x1_0000_0000, 5, A.jmp("jgt", 1, 2, 1, reg=True), False, "inst_gen.go:626 (Q1)")
jcase("jsgt_x_int32", 0x0000_0000_8000_0000, 1, A.jmp("jsgt", 1, 2, 1, reg=True), False, "inst_gen.go:654 (Q1: int32 view)")
jcase("jslt_x_int32", 0xFFFF_FFFF, 0, A.jmp("jslt", 1, 2, 1, reg=True), True, "inst_gen.go:683 (Q1)")
jcase("jne_x_low32", 0xAAAA_0000_0000_0007, 0xBBBB_0000_0000_0007, A.jmp("jne", 1, 2, 1, reg=True), False, "inst_gen.go:646 (Q1)")
# immediate forms are 64-bit with the sign-extended constant
jcase("jeq_k_64", 0x1_0000_0005, 5, A.jmp("jeq", 1, 5, 1), False, "inst_gen.go:613,236-243")
jcase("jeq_k_signext", M64, 0, A.jmp("jeq", 1, -1, 1), True, "inst_gen.go:238 (uint64(Constant))")
jcase("jgt_k_unsigned", M64, 0, A.jmp("jgt", 1, 5, 1), True, "inst_gen.go:621")
jcase("jsgt_k_signed", M64, 0, A.jmp("jsgt", 1, 5, 1), False, "inst_gen.go:649")
jcase("jlt_k", 3, 0, A.jmp("jlt", 1, 5, 1), True, "inst_gen.go:669")
jcase("jsle_k", s64(-7) & M64, 0, A.jmp("jsle", 1, -7, 1), True, "inst_gen.go:684")
# JMP32 immediate: 32-bit views
jcase("jeq32_k", 0x1_0000_0005, 0, A.jmp32("jeq", 1, 5, 1), True, "inst_gen.go:614,227-234")
jcase("jsgt32_k", 0x7FFF_FFFF, 0, A.jmp32("jsgt", 1, -1, 1), True, "inst_gen.go:650")
jcase("jlt32_k", 0x1_0000_0000, 0, A.jmp32("jlt", 1, 1, 1), True, "inst_gen.go:670")
# Q3: JSET taken when (dst & x) == 0 (inst.go:205-241)
jcase("jset_k_inverted_set", 1, 0, A.jmp("jset", 1, 1, 1), False, "inst.go:214-221 (Q3)")
jcase("jset_k_inverted_clear", 2, 0, A.jmp("jset", 1, 1, 1), True, "inst.go:214-221 (Q3)")
jcase("jset_x_64bit", 0x1_0000_0000, 0x1_0000_0000, A.jmp("jset", 1, 2, 1, reg=True), False, "inst.go:53,233-241")
jcase("jset32_k", 0x1_0000_0000, 0, A.jmp32("jset", 1, 0x1, 1), True, "inst.go:50,205-212")
jcase("jset32_x", 0x1_0000_0001, 0x2_0000_0001, A.jmp32("jset", 1, 2, 1, reg=True), False, "inst.go:51,223-231")
# 0xff slot = instJump64JSLEReg (last write of initGen, inst_gen.go:686)
jcase("slot_0xff_is_jsle64_reg", M64, 0, A.raw(0xFF, 1, 2, 1), True, "inst_gen.go:686 (Appendix A)")
jcase("slot_0xff_not_taken", 5, 3, A.raw(0xFF, 1, 2, 1), False, "inst_gen.go:686")
# Q2: JMP32 register forms are nil -> CustomInstruction -> unsupported
case("jeq32_x_unsupported", [A.mov64_imm(0, 0), A.jmp32("jeq", 0, 0, 1, reg=True), A.exit_(), A.exit_()],
     e(status=UNSUP, steps=2, err_pc=1), "inst_gen.go:618 keys JumpClass, emulator_linux_.go:287 (Q2)")
case("ja32_unsupported", [A.raw(0x06, 0, 0, 1), A.exit_(), A.exit_()], e(status=UNSUP, steps=1, err_pc=0), "inst.go:48 (JA only in JumpClass)")
case("ja", [A.mov64_imm(0, 4), A.ja(1), A.mov64_imm(0, 9), A.exit_()], e(r0=4, steps=3), "inst.go:200-203")
# PC bounds (vm.go:327-334, 297-300)
case("jump_past_end", [A.mov64_imm(0, 1), A.ja(5), A.exit_()], e(r0=1, status=PC_OOB, steps=2, err_pc=1), "vm.go:327-334")
case("fall_off_end", [A.mov64_imm(0, 1)], e(r0=1, status=PC_OOB, steps=1, err_pc=0), "vm.go:327-334")
case("empty_program", [], e(r0=0, status=PC_OOB, steps=1, err_pc=0), "vm.go:297-299")
case("negative_pc_panics", [A.mov64_imm(0, 1), A.ja(-3), A.exit_()], e(r0=1, status=PANIC_PC, steps=3, err_pc=-1), "vm.go:297-300 (Q14)")
case("backward_loop_budget", [A.mov64_imm(0, 0), A.alu64("add", 0, 1), A.ja(-2)], e(r0=50, status=STEP_LIMIT, steps=100, err_pc=2),
     "vm.go:343-360 (deadline as a step budget)", step_budget=100)
# registers (vm.go:407-466)
case("write_r10", [A.mov64_imm(10, 1), A.exit_()], e(status=R10W, steps=1, err_pc=0), "vm.go:459-460 (Q15)")
case("read_bad_register", [A.mov64_reg(0, 11), A.exit_()], e(status=BADREG, steps=1, err_pc=0), "vm.go:431-432 (Q15)")
case("write_bad_register", [A.mov64_imm(12, 1), A.exit_()], e(status=BADREG, steps=1, err_pc=0), "vm.go:461-462")
case("ldx_mem_error_before_badreg", [A.ldx(4, 11, 10, -300), A.exit_()], e(status=UNRES, steps=1, err_pc=0), "inst.go:298-317 (r10-300 < 0x10000)")
case("ldx_badreg_after_load", [A.ldx(4, 11, 10, -8), A.exit_()], e(status=BADREG, steps=1, err_pc=0), "inst.go:317, vm.go:461")
case("ldx_into_r10", [A.ldx(4, 10, 10, -8), A.exit_()], e(status=R10W, steps=1, err_pc=0), "inst.go:317, vm.go:459")
# Q7: division by zero panics
case("div64_x_zero", [A.mov64_imm(0, 9), A.mov64_imm(2, 0), A.alu64("div", 0, 2, reg=True), A.exit_()], e(r0=9, status=DIV0, steps=3, err_pc=2), "inst_gen.go:89-93")
case("div32_x_truncated_zero", [A.mov64_imm(0, 9), A.ld_imm64(2, 0x1_0000_0000), A.alu32("div", 0, 2, reg=True), A.exit_()],
     e(r0=9, status=DIV0, steps=4, err_pc=3), "inst_gen.go:83-87 (uint32(src) == 0)")
case("mod64_k_zero", [A.mov64_imm(0, 9), A.alu64("mod", 0, 0), A.exit_()], e(r0=9, status=DIV0, steps=2, err_pc=1), "inst_gen.go:188-191")
case("div_r10_dst_zero_divisor", [A.mov64_imm(2, 0), A.alu64("div", 10, 2, reg=True), A.exit_()], e(status=DIV0, steps=2, err_pc=1), "inst_gen.go:89-93 (panic before Set)")
case("div_r10_dst", [A.mov64_imm(2, 3), A.alu64("div", 10, 2, reg=True), A.exit_()], e(status=R10W, steps=2, err_pc=1), "vm.go:459")
# unsupported / unimplemented (emulator_linux_.go:198-288)
case("atomic_add_unsupported", [A.raw(0xDB, 10, 0, -8, 0), A.exit_()], e(status=UNSUP, steps=1, err_pc=0), "inst.go:77 (TODO atomics)")
case("ld_abs_on_xdp", [A.raw(0x30, 0, 0, 0, 12), A.exit_()], e(status=LDABS, steps=1, err_pc=0), "emulator_linux_.go:200-213")
case("ld_ind_on_xdp", [A.raw(0x50, 0, 1, 0, 12), A.exit_()], e(status=LDABS, steps=1, err_pc=0), "emulator_linux_.go:243-256")
case("callx_panics", [A.raw(0x8D, 0, 0, 0, 1), A.exit_()], e(status=CALLX, steps=1, err_pc=0), "inst.go:270-273")
case("exit_regform_unsupported", [A.raw(0x9D)], e(status=UNSUP, steps=1, err_pc=0), "inst.go:58")
case("ldx_memsx_unsupported", [A.raw(0x81, 0, 10, -8), A.exit_()], e(status=UNSUP, steps=1, err_pc=0), "inst.go:62-65")
# helpers (emulator_linux_.go:125-194)
case("helper_unimplemented", [A.call(6), A.exit_()], e(status=H_UNIMPL, steps=1, err_pc=0), "emulator_linux_helpers.go:28-204 (trace_printk nil)")
case("helper_beyond_table", [A.call(176), A.exit_()], e(status=H_UNIMPL, steps=1, err_pc=0), "emulator_linux_.go:184-186")
case("helper_cant_emulate", [A.call(14), A.exit_()], e(status=H_CANT, steps=1, err_pc=0), "emulator_linux_helpers.go:473-475")
case("helper_negative_panics", [A.call(-1), A.exit_()], e(status=HELPER_NEG, steps=1, err_pc=0), "emulator_linux_.go:126")
case("helper_ktime_engine", [A.call(5), A.exit_()], e(status=ENGINE_HELPER, steps=1, err_pc=0), "emulator_linux_helpers.go:588-594 (non-deterministic, not emulated by the engine)")
# Q8: helpers leave R1-R5 alone; get_smp_processor_id (emulator_linux_helpers.go:603-606)
case("smp_id_cpu3_keeps_r1_r5", [A.mov64_imm(3, 77), A.call(8), A.alu64("add", 0, 3, reg=True), A.exit_()],
     e(r0=80, steps=4), "emulator_linux_helpers.go:603-606 (Q8)", vcpus=4, cpu=3)
# Q11: xdp_adjust_tail needs a 20-byte ctx: always -EINVAL on the 24-byte xdp_md
case("xdp_adjust_tail_einval", [A.mov64_imm(2, -4), A.call(65), A.exit_()], e(r0=-22, steps=3), "emulator_linux_helpers.go:861-864 (Q11)")
# Q12: BPF-to-BPF call executes target-1 first (fixup imm = sym-i-1; PC += imm-1; PC++)
case("bpf2bpf_lands_at_target_minus_1",
     [A.mov64_imm(0, 1), A.Insn(A.JMP | A.CALL, 0, 1, 0, 2), A.exit_(), A.alu64("add", 0, 10), A.alu64("add", 0, 100), A.exit_()],
     e(r0=111, steps=6), "vm.go:163-169, inst.go:253, vm.go:337 (Q12)")
case("bpf2bpf_frame_restores_r6_r9_and_r10",
     [A.mov64_imm(6, 5), A.mov64_reg(7, 10), A.Insn(A.JMP | A.CALL, 0, 1, 0, 5),
      A.mov64_reg(0, 10), A.alu64("sub", 0, 7, reg=True), A.alu64("add", 0, 6, reg=True), A.exit_(),
      A.mov64_imm(6, 1000), A.mov64_reg(1, 10), A.alu64("sub", 1, 7, reg=True), A.exit_()],
     e(r0=5, steps=11), "inst.go:243-258, 277-296")
case("bpf2bpf_r10_moves_by_frame", [A.Insn(A.JMP | A.CALL, 0, 1, 0, 3), A.exit_(), A.exit_(), A.mov64_reg(0, 10), A.exit_()],
     e(r0=0x10009 + 256 + 256, steps=4), "inst.go:255 (R10 += StackFrameSize); stack at 0x10009")

# memory layout (memory_controller.go:58-112, vm.go:218-224, context_xdp_md.go:66-112)
# one program, no maps: prog @0x10000 (size 8) -> stack @0x10009, R10 = 0x10109,
# packet @0x10009+2049 = 0x1080A, xdp_md @ packet + (H+L+T) + 1
case("layout_r10", [A.mov64_reg(0, 10), A.exit_()], e(r0=0x10109, steps=2), "vm.go:218-224")
case("layout_r1_xdp_md", [A.mov64_reg(0, 1), A.exit_()], e(r0=0x1080A + 64 + 1, steps=2), "context_xdp_md.go:107-112")
case("layout_r1_headroom_tailroom", [A.mov64_reg(0, 1), A.exit_()], e(r0=0x1080A + 16 + 64 + 8 + 1, steps=2),
     "context_xdp_md.go:52-112", headroom=16, tailroom=8)
case("xdp_md_data", [A.ldx(4, 0, 1, 0), A.exit_()], e(r0=0x1080A + 16, steps=2), "context_xdp_md.go:71-75", headroom=16)
case("xdp_md_data_end", [A.ldx(4, 0, 1, 4), A.exit_()], e(r0=0x1080A + 16 + 64, steps=2), "context_xdp_md.go:77-81", headroom=16)
case("xdp_md_data_meta", [A.ldx(4, 0, 1, 8), A.exit_()], e(r0=0x1080A + 16, steps=2), "context_xdp_md.go:83-87", headroom=16)
case("xdp_md_ifindex_fields", [A.ldx(4, 0, 1, 12), A.ldx(4, 2, 1, 16), A.alu64("lsh", 2, 16), A.alu64("or", 0, 2, reg=True),
                               A.ldx(4, 2, 1, 20), A.alu64("lsh", 2, 32), A.alu64("or", 0, 2, reg=True), A.exit_()],
     e(r0=3 | (2 << 16) | (0xFFFFFFFF << 32), steps=8), "context_xdp_md.go:89-105", ingress=3, rxq=2, egress=-1)
case("xdp_md_u64_load", [A.ldx(8, 0, 1, 0), A.exit_()], e(r0=(0x1080A + 64) << 32 | 0x1080A, steps=2), "memory_plain.go:47-48")
case("xdp_md_store_then_load", [A.st(4, 1, 12, 99), A.ldx(4, 0, 1, 12), A.exit_()], e(r0=99, steps=3), "memory_plain.go:55-87")
case("xdp_md_bounds", [A.ldx(8, 0, 1, 20), A.exit_()], e(status=BOUNDS, steps=1, err_pc=0), "memory_plain.go:27")
case("xdp_md_end_inclusive", [A.ldx(1, 0, 1, 24), A.exit_()], e(status=BOUNDS, steps=1, err_pc=0), "memory_controller.go:137 (Q13)")
case("beyond_last_entry", [A.ldx(1, 0, 1, 25), A.exit_()], e(status=UNRES, steps=1, err_pc=0), "memory_controller.go:117-145")
case("below_mem_start", [A.mov64_imm(2, 0xFFFF), A.ldx(1, 0, 2, 0), A.exit_()], e(status=UNRES, steps=2, err_pc=1), "memory_controller.go:55")
case("stack_end_inclusive_bounds", [A.ldx(1, 0, 10, 1792), A.exit_()], e(status=BOUNDS, steps=1, err_pc=0), "memory_controller.go:137, memory_plain.go:27 (Q13)")
case("stack_below_is_program_object", [A.ldx(1, 0, 10, -257), A.exit_()], e(status=NOTVMMEM, steps=1, err_pc=0), "inst.go:307-310 (*ebpf.ProgramSpec at 0x10000..0x10008)")
case("stack_zeroed", [A.ldx(8, 0, 10, -8), A.exit_()], e(r0=0, steps=2), "vm.go:208-210 (fresh zeroed stack)")
case("stack_store_load", [A.ld_imm64(2, 0x1122334455667788), A.stx(8, 10, -16, 2), A.ldx(4, 0, 10, -12), A.exit_()],
     e(r0=0x11223344, steps=5), "memory_plain.go (native little endian)")
case("stack_unaligned_across_words", [A.ld_imm64(2, 0x1122334455667788), A.stx(8, 10, -13, 2), A.ldx(8, 0, 10, -14), A.exit_()],
     e(r0=0x2233445566778800, steps=5), "memory_plain.go:25-87 (byte addressed)")
case("stack_st_imm_signext", [A.st(8, 10, -8, -2), A.ldx(8, 0, 10, -8), A.exit_()], e(r0=-2, steps=3), "inst.go:334 (uint64(Constant))")
case("packet_load_be_field", [A.ldx(4, 2, 1, 0), A.ldx(2, 0, 2, 12), A.exit_()], e(r0=0x0008, steps=3), "memory_plain.go:43-44 (native LE)",
     packet=b"\x00" * 12 + b"\x08\x00" + b"\x00" * 50)
case("packet_store_visible", [A.ldx(4, 2, 1, 0), A.st(4, 2, 60, 0x01020304), A.ldx(1, 0, 2, 63), A.exit_()], e(r0=1, steps=4), "memory_plain.go:55-87")
case("packet_bounds", [A.ldx(4, 2, 1, 0), A.ldx(4, 0, 2, 62), A.exit_()], e(status=BOUNDS, steps=2, err_pc=1), "memory_plain.go:27-34")
case("packet_zero_length", [A.ldx(4, 2, 1, 0), A.ldx(1, 0, 2, 0), A.exit_()], e(status=BOUNDS, steps=2, err_pc=1), "context_xdp_md.go:52-66", packet=b"")
case("headroom_is_zero", [A.ldx(4, 2, 1, 0), A.ldx(8, 0, 2, -8), A.exit_()], e(r0=0, steps=3), "context_xdp_md.go:52-64", headroom=8,
     packet=b"\xff" * 64)

# maps: array (emulator_linux_map_array.go), reference tests + quirks
ARR = dict(name="arr", type=2, key_size=4, value_size=4, max_entries=5)
k = lambda i: i.to_bytes(4, "little")  # noqa: E731
lookup_prog = [A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "arr"),
               A.call(1), A.jmp("jeq", 0, 0, 1), A.ldx(4, 0, 0, 0), A.exit_()]
case("ref_TestLinuxHelperLookup_m1_eq_2", lookup_prog, e(r0=2, steps=9), "emulator_linux_helpers_test.go:11-113",
     maps=[ARR], map_init=[("arr", k(1), k(2), 0)])
case("array_lookup_address", lookup_prog[:6] + [A.exit_()], e(r0=0x10009 + 4, steps=8),
     "emulator_linux_map_array.go:30-54, 78-94 (obj @0x10000, values @0x10009)", maps=[ARR])
case("array_lookup_oob_null", [A.st(4, 10, -4, 5), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "arr"),
                               A.call(1), A.exit_()], e(r0=0, steps=7), "emulator_linux_map_array.go:87-90", maps=[ARR])
case("array_update_e2big_positive", [A.st(4, 10, -4, 9), A.st(4, 10, -8, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4),
                                     A.mov64_reg(3, 10), A.alu64("add", 3, -8), A.ld_map_fd(1, "arr"), A.mov64_imm(4, 0),
                                     A.call(2), A.exit_()], e(r0=7, steps=11), "emulator_linux_map_array.go:107-110, helpers.go:549 (Q9)",
     maps=[ARR])
case("array_update_flags_ignored", [A.st(4, 10, -4, 1), A.st(4, 10, -8, 42), A.mov64_reg(2, 10), A.alu64("add", 2, -4),
                                    A.mov64_reg(3, 10), A.alu64("add", 3, -8), A.ld_map_fd(1, "arr"), A.mov64_imm(4, 1),
                                    A.call(2), A.mov64_reg(6, 0), A.st(4, 10, -4, 1), A.mov64_reg(2, 10),
                                    A.alu64("add", 2, -4), A.ld_map_fd(1, "arr"), A.call(1), A.ldx(4, 0, 0, 0),
                                    A.alu64("add", 0, 6, reg=True), A.exit_()],
     e(r0=42, steps=20), "emulator_linux_map_array.go:97-113 (Q10)", maps=[ARR], map_init=[("arr", k(1), k(5), 0)])
case("array_delete_not_deleter", [A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "arr"),
                                  A.call(3), A.exit_()], e(status=MAP_OP, steps=6, err_pc=5), "emulator_linux_helpers.go:565-568", maps=[ARR])
case("array_direct_load_not_datasec", [A.ld_map_fd(1, "arr"), A.ldx(4, 0, 1, 0), A.exit_()], e(status=NOTDATASEC, steps=3, err_pc=2),
     "emulator_linux_map_array.go:136-138", maps=[ARR])
case("lookup_bad_map_pointer", [A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.mov64_imm(1, 5),
                                A.call(1), A.exit_()], e(status=MAP_PTR, steps=5, err_pc=4), "emulator_linux_helpers.go:415-420", maps=[ARR])
case("lookup_key_deref_error", [A.mov64_imm(2, 3), A.ld_map_fd(1, "arr"), A.call(1), A.exit_()], e(status=KEY, steps=4, err_pc=3),
     "emulator_linux_helpers.go:449-456", maps=[ARR])
case("lookup_double_map_pointer", [A.ld_map_fd(3, "arr"), A.stx(4, 10, -16, 3), A.mov64_reg(1, 10), A.alu64("add", 1, -16),
                                   A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.call(1),
                                   A.ldx(4, 0, 0, 0), A.exit_()],
     e(r0=2, steps=11), "emulator_linux_helpers.go:422-440 (map-in-map double pointer)", maps=[ARR], map_init=[("arr", k(1), k(2), 0)])
DS = dict(name="ds", type=2, key_size=4, value_size=8, max_entries=2, datasec=True)
case("datasec_pseudo_map_value_offset", [A.ld_map_value(1, "ds", 4), A.ldx(4, 0, 1, 0), A.exit_()], e(r0=0x11223344, steps=4),
     "emulator_linux_.go:328-331 (Q16), emulator_linux_map_array.go:134-150", maps=[DS],
     map_init=[("ds", k(0), bytes.fromhex("ddccbbaa44332211"), 0)])
case("datasec_store_then_lookup", [A.ld_map_value(1, "ds"), A.st(4, 1, 8, 77), A.st(4, 10, -4, 1), A.mov64_reg(2, 10),
                                   A.alu64("add", 2, -4), A.ld_map_fd(1, "ds"), A.call(1), A.ldx(4, 0, 0, 0), A.exit_()],
     e(r0=77, steps=11), "emulator_linux_map_array.go:143-150", maps=[DS])
# per-CPU array (emulator_linux_map_array.go:177-250; reference test emulator_linux_map_array_test.go:10-103)
PCA = dict(name="pca", type=6, key_size=4, value_size=4, max_entries=5)
pc_prog = [A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "pca"),
           A.call(1), A.jmp("jeq", 0, 0, 1), A.ldx(4, 0, 0, 0), A.exit_()]
for cpu, val in ((0, 2), (1, 3)):
    case(f"ref_TestLinuxPerCPUArray_cpu{cpu}", pc_prog, e(r0=val, steps=9), "emulator_linux_map_array_test.go:10-103",
         vcpus=2, maps=[PCA], map_init=[("pca", k(1), k(2), 0), ("pca", k(1), k(3), 1)], cpu=cpu)
for cpu in (0, 1):
    case(f"percpu_lookup_address_cpu{cpu}", pc_prog[:5] + [A.exit_()], e(r0=0x10009 + 9 + cpu * 30 + 4, steps=7),
         "emulator_linux_map_array.go:185-215 (sub-arrays at 0x10009 + c*(E*S+10))", vcpus=2, maps=[PCA], cpu=cpu)
case("percpu_counter_increment", [A.st(4, 10, -4, 2), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "pca"),
                                  A.call(1), A.jmp("jeq", 0, 0, 4), A.ldx(4, 1, 0, 0), A.alu64("add", 1, 1), A.stx(4, 0, 0, 1),
                                  A.ldx(4, 0, 0, 0), A.exit_()], e(r0=41, steps=12), "emulator_linux_map_array.go:235-241",
     vcpus=3, maps=[PCA], map_init=[("pca", k(2), k(40), 2)], cpu=2)
case("percpu_via_sub_array_object", [A.ld_map_fd(1, "pca"), A.alu64("add", 1, 9 + 30), A.st(4, 10, -4, 1), A.mov64_reg(2, 10),
                                     A.alu64("add", 2, -4), A.call(1), A.ldx(4, 0, 0, 0), A.exit_()],
     e(r0=3, steps=9), "emulator_linux_map_array.go:202-208 (sub-array object is a LinuxArrayMap)", vcpus=2, maps=[PCA],
     map_init=[("pca", k(1), k(2), 0), ("pca", k(1), k(3), 1)], cpu=0)
# ref test TestLinuxHelperGetSmpProcessorID (emulator_linux_helpers_test.go:185-220)
for cpu in (0, 1):
    case(f"ref_TestLinuxHelperGetSmpProcessorID_cpu{cpu}", [A.call(8), A.exit_()], e(r0=cpu, steps=2),
         "emulator_linux_helpers_test.go:185-220", vcpus=2, cpu=cpu)
# tail calls (emulator_linux_helpers.go:649-738)
PA = dict(name="progs", type=3, key_size=4, value_size=4, max_entries=4)
tc_main = [A.mov64_imm(0, 1), A.ld_map_fd(2, "progs"), A.mov64_imm(3, 0), A.call(12), A.alu64("add", 0, 1000), A.exit_()]
tc_target = [A.alu64("add", 0, 5), A.exit_()]
case("tailcall_switches_program", tc_main, e(r0=6, steps=7), "emulator_linux_helpers.go:649-738",
     maps=[PA], extra_progs=[("t", tc_target)], prog_array=[("progs", 0, 1)])
case("tailcall_empty_slot_einval", tc_main[:2] + [A.mov64_imm(3, 2)] + tc_main[3:], e(r0=-22 + 1000, steps=7),
     "emulator_linux_helpers.go:713-718", maps=[PA], extra_progs=[("t", tc_target)], prog_array=[("progs", 0, 1)])
case("tailcall_key_oob_einval", tc_main[:2] + [A.mov64_imm(3, 9)] + tc_main[3:], e(r0=-22 + 1000, steps=7),
     "emulator_linux_map_array.go:87-90 -> helpers.go:694-699", maps=[PA], extra_progs=[("t", tc_target)])
tc_loop = [A.alu64("add", 0, 1), A.ld_map_fd(2, "progs"), A.mov64_imm(3, 0), A.call(12), A.exit_()]
case("tailcall_max_33_eperm", tc_loop, e(r0=-1, steps=34 * 5 + 1), "emulator_linux_helpers.go:663-666 (MaxTailCalls 33)",
     maps=[PA], prog_array=[("progs", 0, 0)])
case("tailcall_max_custom_3", tc_loop, e(r0=-1, steps=4 * 5 + 1), "emulator_linux_.go:40-44 (OptMaxTailCalls)",
     maps=[PA], prog_array=[("progs", 0, 0)], max_tail_calls=3)
case("tailcall_not_prog_array", [A.ld_map_fd(2, "arr"), A.mov64_imm(3, 0), A.call(12), A.exit_()], e(status=TAILCALL, steps=4, err_pc=3),
     "emulator_linux_helpers.go:674-676", maps=[ARR])
case("tailcall_into_empty_program", tc_main, e(r0=1, status=PC_OOB, steps=5, err_pc=4), "vm.go:327-334 after PC = -1",
     maps=[PA], extra_progs=[("empty", [])], prog_array=[("progs", 0, 1)])


# hash maps (emulator_linux_map_hash.go): obj (8) | keys (E*K) | values (E*S); per-CPU hash:
# V x values (E*S) | obj | keys.  A new key takes the freelist head (slots 0..E-1 initially,
# :56-64, :179-186); Delete pushes the slot to the tail (:244-250); a full freelist is E2BIG.
# Straight-line programs: steps = slots executed (the LD_IMM64 pad Nop counts, inst.go:82-84).
H3 = dict(name="h", type=1, key_size=4, value_size=8, max_entries=3)
H_KEYS, H_VALS = 0x10009, 0x10009 + 12 + 1


def h_upd(key, val, m="h"):
    return [A.st(4, 10, -4, key), A.st(8, 10, -16, val), A.mov64_reg(2, 10), A.alu64("add", 2, -4),
            A.mov64_reg(3, 10), A.alu64("add", 3, -16), A.ld_map_fd(1, m), A.mov64_imm(4, 0), A.call(2)]


def h_look(key, m="h"):
    return [A.st(4, 10, -4, key), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, m), A.call(1)]


def h_del(key, m="h"):
    return [A.st(4, 10, -4, key), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, m), A.call(3)]


def straight(name, items, r0, ref, **kw):
    items = items + [A.exit_()]
    case(name, items, e(r0=r0, steps=len(A.assemble(items)[0]) // 8), ref, **kw)


straight("hash_lookup_absent_null", h_look(7), 0, "emulator_linux_map_hash.go:145-149", maps=[H3])
straight("hash_update_returns_zero", h_upd(7, 100), 0, "emulator_linux_map_hash.go:158-203", maps=[H3])
straight("hash_first_slot_address", h_upd(7, 100) + h_look(7), H_VALS,
         "emulator_linux_map_hash.go:43-97 (obj @0x10000, keys @0x10009, values @0x10016), :152-154", maps=[H3])
straight("hash_value_readback", h_upd(7, 100) + h_look(7) + [A.ldx(8, 0, 0, 0)], 100,
         "emulator_linux_map_hash.go:196-200", maps=[H3])
fifo = h_upd(1, 11) + h_upd(2, 22) + h_del(1) + h_upd(3, 33) + h_upd(4, 44)
straight("hash_fifo_reuse_tail", fifo + h_look(4), H_VALS + 0,
         "emulator_linux_map_hash.go:179-186, 244-250 (slot 0 returns to the tail)", maps=[H3])
straight("hash_fifo_head_order", fifo + h_look(3), H_VALS + 16,
         "emulator_linux_map_hash.go:61-64 (freelist 0,1,2 in order)", maps=[H3])
straight("hash_fifo_value", fifo + h_look(4) + [A.ldx(8, 0, 0, 0)], 44, "emulator_linux_map_hash.go:196-200", maps=[H3])
straight("hash_e2big_positive", h_upd(1, 1) + h_upd(2, 2) + h_upd(3, 3) + h_upd(4, 4), 7,
         "emulator_linux_map_hash.go:181-184, helpers.go:549 (Q9)", maps=[H3])
straight("hash_update_existing_keeps_slot",
         h_upd(1, 1) + h_upd(2, 2) + h_upd(1, 5) + h_upd(3, 3) + h_look(1) + [A.ldx(8, 0, 0, 0)], 5,
         "emulator_linux_map_hash.go:170-177 (found: same slot, no freelist pop)", maps=[H3])
straight("hash_update_existing_then_full", h_upd(1, 1) + h_upd(2, 2) + h_upd(1, 5) + h_upd(3, 3) + h_upd(4, 4), 7,
         "emulator_linux_map_hash.go:170-186", maps=[H3])
straight("hash_delete_absent_zero", h_del(9), 0, "emulator_linux_map_hash.go:233-237", maps=[H3])
straight("hash_delete_then_lookup_null", h_upd(1, 1) + h_del(1) + h_look(1), 0,
         "emulator_linux_map_hash.go:239-244", maps=[H3])
straight("hash_keys_backing_visible", h_upd(0x11223344, 1) + [A.ld_imm64(1, H_KEYS), A.ldx(4, 0, 1, 0)], 0x11223344,
         "emulator_linux_map_hash.go:188-193 (keys PlainMemory is VM memory)", maps=[H3])
straight("hash_keys_backing_second_slot",
         h_upd(5, 1) + h_upd(0x0a0b0c0d, 2) + [A.ld_imm64(1, H_KEYS + 4), A.ldx(4, 0, 1, 0)], 0x0a0b0c0d,
         "emulator_linux_map_hash.go:188-193", maps=[H3])
straight("hash_host_update_then_lookup", h_look(5) + [A.ldx(8, 0, 0, 0)], 77, "emulator_linux_map_hash.go:158-203 (host Update)",
         maps=[H3], map_init=[("h", k(5), (77).to_bytes(8, "little"), 0)])
case("hash_object_not_vmmem", [A.ld_map_fd(1, "h"), A.ldx(4, 0, 1, 0), A.exit_()], e(status=NOTVMMEM, steps=3, err_pc=2),
     "inst.go:308-311 (LinuxHashMap is not VMMem)", maps=[H3])
case("hash_lookup_key_unresolved", [A.mov64_imm(2, 3), A.ld_map_fd(1, "h"), A.call(1), A.exit_()],
     e(status=KEY, steps=4, err_pc=3), "emulator_linux_helpers.go:449-456", maps=[H3])
case("hash_update_value_unresolved", [A.st(4, 10, -4, 1), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.mov64_imm(3, 3),
                                      A.ld_map_fd(1, "h"), A.call(2), A.exit_()],
     e(status=VALUE, steps=7, err_pc=6), "emulator_linux_helpers.go:525-530", maps=[H3])
case("hash_delete_key_unresolved", [A.mov64_imm(2, 3), A.ld_map_fd(1, "h"), A.call(3), A.exit_()],
     e(status=KEY, steps=4, err_pc=3), "emulator_linux_helpers.go:570-574", maps=[H3])
case("hash_key_partly_outside_stack", [A.mov64_reg(2, 10), A.alu64("add", 2, -2), A.ld_map_fd(1, "h"), A.call(1), A.exit_()],
     e(status=OK, r0=0, steps=6), "memory_plain.go:27-34 (4 key bytes at r10-2 are inside the 2 KiB stack)", maps=[H3])
# 13-byte 5-tuple keys (K not a multiple of 8): keys backing 52 B, values @0x10009 + 53
H13 = dict(name="h13", type=1, key_size=13, value_size=8, max_entries=4)
H13_VALS = 0x10009 + 52 + 1


def k13(last):
    return [A.st(8, 10, -16, 0x01020304), A.st(4, 10, -8, 0x0a0b0c0d), A.st(1, 10, -4, last)]


def h13_upd(last, val):
    return k13(last) + [A.st(8, 10, -24, val), A.mov64_reg(2, 10), A.alu64("add", 2, -16), A.mov64_reg(3, 10),
                        A.alu64("add", 3, -24), A.ld_map_fd(1, "h13"), A.mov64_imm(4, 0), A.call(2)]


def h13_look(last):
    return k13(last) + [A.mov64_reg(2, 10), A.alu64("add", 2, -16), A.ld_map_fd(1, "h13"), A.call(1)]


straight("hash_key13_first_slot", h13_upd(0x55, 9) + h13_look(0x55), H13_VALS, "emulator_linux_map_hash.go:43-97, 152-154",
         maps=[H13])
straight("hash_key13_last_byte_distinguishes", h13_upd(0x55, 9) + h13_upd(0x56, 10) + h13_look(0x56) + [A.ldx(8, 0, 0, 0)],
         10, "emulator_linux_map_hash.go:134-155 (exact key bytes)", maps=[H13])
straight("hash_key13_miss", h13_upd(0x55, 9) + h13_look(0x57), 0, "emulator_linux_map_hash.go:145-149", maps=[H13])
# per-CPU hash: values of cpu c @0x10000 + c*(E*S+1), obj after them, keys after the obj
PH = dict(name="ph", type=5, key_size=4, value_size=4, max_entries=2)
for cpu in (0, 1):
    straight(f"percpu_hash_address_cpu{cpu}", h_upd(5, 3, "ph") + h_look(5, "ph"), 0x10000 + cpu * 9,
             "emulator_linux_map_hash.go:439-500 (values per cpu first), :537-561", vcpus=2, maps=[PH], cpu=cpu)
for cpu, val in ((0, 9), (1, 0)):
    straight(f"percpu_hash_value_cpu{cpu}", h_look(5, "ph") + [A.ldx(4, 0, 0, 0)], val,
             "emulator_linux_map_hash.go:564-612 (shared key table, per-cpu values)", vcpus=2, maps=[PH], cpu=cpu,
             map_init=[("ph", k(5), k(9), 0)])
straight("percpu_hash_keys_backing", h_upd(0x01020304, 3, "ph") + [A.ld_imm64(1, 0x10012 + 9), A.ldx(4, 0, 1, 0)], 0x01020304,
         "emulator_linux_map_hash.go:484-494 (keys after the map object)", vcpus=2, maps=[PH], cpu=1)
case("percpu_hash_object_not_vmmem", [A.ld_map_fd(1, "ph"), A.ldx(4, 0, 1, 0), A.exit_()], e(status=NOTVMMEM, steps=3, err_pc=2),
     "inst.go:308-311", vcpus=2, maps=[PH])
straight("percpu_hash_e2big", h_upd(1, 1, "ph") + h_upd(2, 2, "ph") + h_upd(3, 3, "ph"), 7,
         "emulator_linux_map_hash.go:584-590", vcpus=2, maps=[PH])

def main():
    out = os.path.join(HERE, "kat.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": CASES}, f, indent=0)
    print(f"wrote {len(CASES)} cases to {out}")


if __name__ == "__main__":
    main()
