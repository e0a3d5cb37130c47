"""Random programs over the sk_buff context for differential testing (oracle vs GPU engine):
__sk_buff / bpf_sock / bpf_flow_keys loads and stores at field and off-field offsets, direct
packet access through skb->data (BigEndian memory), LD_ABS / LD_IND, all mixed into r9."""
from __future__ import annotations

import numpy as np

from mimic_amd import asm as A

SKB_OFFS = sorted(set(A.SKB.values()) | {9, 50, 64, 92, 95, 99, 100, 113, 115, 116, 131, 190, 192})
SOCK_OFFS = sorted(set(A.SOCK.values()) | {26, 43, 54, 60, 68, 70, 71, 80})
FK_OFFS = list(range(0, 41))
WRITABLE = [A.SKB[k] for k in ("mark", "queue_mapping", "priority", "tc_index", "tc_classid", "tstamp")] + [52, 0]


def _size(rng):
    return int(rng.choice([1, 2, 4, 8], p=[0.2, 0.2, 0.45, 0.15]))


def random_skb_program(rng, n_ops: int = 10):
    items = [A.mov64_reg(6, 1), A.mov64_imm(9, 0), A.mov64_imm(8, int(rng.integers(0, 40)))]
    for _ in range(n_ops):
        k = rng.random()
        sz = _size(rng)
        if k < 0.25:     # __sk_buff load
            items += [A.ldx(sz, 7, 6, int(rng.choice(SKB_OFFS))), A.alu64("xor", 9, 7, reg=True)]
        elif k < 0.35:   # __sk_buff store (writable or read-only field)
            off = int(rng.choice(WRITABLE)) if rng.random() < 0.8 else int(rng.choice(SKB_OFFS))
            items += [A.stx(sz, 6, off, 9)]
        elif k < 0.45:   # bpf_sock
            items += [A.ldx(4, 2, 6, A.SKB["sk"])]
            if rng.random() < 0.2:
                items += [A.st(4, 2, int(rng.choice(SOCK_OFFS)), int(rng.integers(0, 1000)))]
            items += [A.ldx(sz, 7, 2, int(rng.choice(SOCK_OFFS))), A.alu64("xor", 9, 7, reg=True)]
        elif k < 0.55:   # bpf_flow_keys
            items += [A.ldx(4, 2, 6, A.SKB["flow_keys"])]
            off = int(rng.choice(FK_OFFS))
            if rng.random() < 0.5:
                items += [A.stx(sz, 2, off, 9)]
            items += [A.ldx(sz, 7, 2, int(rng.choice(FK_OFFS))), A.alu64("xor", 9, 7, reg=True)]
        elif k < 0.75:   # packet through skb->data, sometimes guarded by data_end
            items += [A.ldx(4, 2, 6, A.SKB["data"])]
            off = int(rng.integers(-40, 140))
            if rng.random() < 0.3:
                items += [A.stx(sz, 2, off, 9)]
            items += [A.ldx(sz, 7, 2, off), A.alu64("xor", 9, 7, reg=True)]
        elif k < 0.9:    # LD_ABS
            items += [A.ld_abs(sz, int(rng.integers(-8, 120))), A.alu64("xor", 9, 0, reg=True)]
        else:            # LD_IND
            items += [A.ld_ind(sz, 8, int(rng.integers(-4, 60))), A.alu64("xor", 9, 0, reg=True)]
    items += [A.mov64_reg(0, 9), A.exit_()]
    return A.assemble(items)
