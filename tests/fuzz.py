"""Random eBPF program generator for differential testing (oracle vs GPU engine)."""
from __future__ import annotations

import numpy as np

from mimic_amd import asm as A

EDGE_IMMS = [0, 1, -1, 2, 7, 8, 15, 16, 31, 32, 33, 63, 64, 65, 255, 0x7FFFFFFF, -0x80000000, 0x12345678, -2, 3]


def _imm(rng):
    if rng.random() < 0.5:
        return int(rng.choice(EDGE_IMMS))
    return int(rng.integers(-2**31, 2**31))


def _reg(rng, allow_bad=0.0, allow_r10=0.0):
    x = rng.random()
    if x < allow_bad:
        return int(rng.integers(11, 16))
    if x < allow_bad + allow_r10:
        return 10
    return int(rng.integers(0, 10))


def random_program(rng, n_body: int = 40, map_name=None, allow_errors: bool = True, packet_len: int = 64,
                   allow_backjump: bool = False):
    """Returns (raw bytes, relocs).  r6 = ctx, r2/r3 = data/data_end, r7 = r10 copy at entry."""
    bad = 0.01 if allow_errors else 0.0
    r10p = 0.01 if allow_errors else 0.0
    items = [A.mov64_reg(6, 1), A.ldx(4, 2, 6, 0), A.ldx(4, 3, 6, 4), A.mov64_reg(7, 10)]
    labels = [f"L{i}" for i in range(n_body + 1)]
    for i in range(n_body):
        items.append(labels[i])
        kind = rng.random()
        if kind < 0.40:   # ALU
            cls = A.ALU64 if rng.random() < 0.5 else A.ALU
            op = int(rng.choice([A.ADD, A.SUB, A.MUL, A.DIV, A.OR, A.AND, A.LSH, A.RSH, A.NEG, A.MOD, A.XOR,
                                 A.MOV, A.ARSH]))
            x = rng.random() < 0.5
            if op in (A.DIV, A.MOD) and not allow_errors:
                x = False
            imm = _imm(rng)
            if op in (A.DIV, A.MOD) and (not allow_errors or rng.random() < 0.8) and imm == 0:
                imm = 3
            if op == A.ARSH and not x and (not allow_errors or rng.random() < 0.8):
                imm = abs(imm) % 70
            dst = _reg(rng, bad, r10p)
            src = _reg(rng, bad)
            if op in (A.DIV, A.MOD) and x and not allow_errors:
                x = False
            items.append(A.Insn(cls | op | (A.X if x else A.K), dst, src if x else 0, 0, 0 if x else imm))
        elif kind < 0.45:  # END
            to_be = rng.random() < 0.5
            width = int(rng.choice([16, 32, 64, 8]))
            items.append(A.Insn(A.ALU | A.END | (A.X if to_be else A.K), _reg(rng, bad, r10p), 0, 0, width))
        elif kind < 0.62:  # conditional / unconditional jumps (forward)
            target = int(rng.integers(i + 1, n_body + 1))
            if allow_backjump and rng.random() < 0.1:
                target = int(rng.integers(0, i + 1))
            jcls = A.JMP if rng.random() < 0.6 else A.JMP32
            op = int(rng.choice([A.JEQ, A.JGT, A.JGE, A.JSET, A.JNE, A.JSGT, A.JSGE, A.JLT, A.JLE, A.JSLT, A.JSLE]))
            if rng.random() < 0.1:
                items.append(A.ja(labels[target]))
                continue
            x = rng.random() < 0.5
            if jcls == A.JMP32 and x and not allow_errors and op != A.JSET:
                x = False
            items.append(A.Insn(jcls | op | (A.X if x else A.K), _reg(rng, bad), _reg(rng, bad) if x else 0,
                                labels[target], 0 if x else _imm(rng)))
        elif kind < 0.75:  # stack memory via r10 / r7
            size = int(rng.choice([1, 2, 4, 8]))
            off = -int(rng.integers(1, 64)) if rng.random() < 0.9 else -int(rng.integers(1, 2100))
            base = 10 if rng.random() < 0.7 else 7
            r = rng.random()
            if r < 0.4:
                items.append(A.ldx(size, _reg(rng, bad, r10p), base, off))
            elif r < 0.7:
                items.append(A.stx(size, base, off, _reg(rng, bad)))
            else:
                items.append(A.st(size, base, off, _imm(rng)))
        elif kind < 0.85:  # packet / ctx memory
            size = int(rng.choice([1, 2, 4, 8]))
            if rng.random() < 0.8:
                off = int(rng.integers(0, packet_len + 4))
                base = 2
            else:
                off = int(rng.integers(0, 30))
                base = 6
            if rng.random() < 0.7:
                items.append(A.ldx(size, _reg(rng, bad, r10p), base, off))
            else:
                items.append(A.stx(size, base, off, int(rng.integers(0, 10))))
        elif kind < 0.90 and map_name is not None:  # map lookup/update with a stack key
            key = int(rng.integers(0, 6))
            items += [A.st(4, 10, -8, key), A.mov64_reg(2, 10), A.alu64("add", 2, -8), A.ld_map_fd(1, map_name)]
            if rng.random() < 0.6:
                items += [A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, 3), A.ldx(8, 4, 0, 0),
                          A.alu64("add", 4, int(rng.integers(1, 100))), A.stx(8, 0, 0, 4)]
            else:
                items += [A.st(8, 10, -16, _imm(rng)), A.mov64_reg(3, 10), A.alu64("add", 3, -16),
                          A.mov64_imm(4, 0), A.call(A.FN_MAP_UPDATE_ELEM)]
            # the helpers leave r1-r5 as they are (Q8); restore data pointers
            items += [A.ldx(4, 2, 6, 0), A.ldx(4, 3, 6, 4)]
        elif kind < 0.93:
            items.append(A.call(int(rng.choice([8, 8, 8, 5, 7, 4, 6, 200, 12]))))
        elif allow_errors and kind < 0.95:
            items.append(A.raw(int(rng.integers(0, 256)), _reg(rng), _reg(rng), int(rng.integers(-3, 4)), _imm(rng)))
        else:
            items.append(A.mov64_imm(int(rng.integers(0, 10)), _imm(rng)))
    items.append(labels[n_body])
    if rng.random() < 0.5:
        items.append(A.mov64_reg(0, int(rng.integers(0, 10))))
    items.append(A.exit_())
    return A.assemble(items)
