"""Minimal eBPF assembler: builds raw little-endian instruction slots.

The reference loads programs through cilium/ebpf (``asm.Instruction``, go.mod: cilium/ebpf
v0.9.0); this image has no BPF-capable clang, so tests, fixtures and benchmarks assemble
bytecode by hand with these helpers.  Opcode values follow the Linux BPF ISA, which is
what cilium's ``asm`` constants encode (``asm.ALUClass`` = 0x04, ``asm.RegSource`` = 0x08, ...).

An instruction is an ``Insn``; ``assemble()`` turns a list of them (and string labels)
into ``bytes``.  ``LD_IMM64`` occupies two slots, exactly like the reference's Nop padding
(vm.go:102-112).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple, Union

# classes
LD, LDX, ST, STX, ALU, JMP, JMP32, ALU64 = 0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07
# sources
K, X = 0x00, 0x08
# sizes
W, H, B, DW = 0x00, 0x08, 0x10, 0x18
SIZE_BYTES = {1: B, 2: H, 4: W, 8: DW}
# modes
IMM, ABS, IND, MEM = 0x00, 0x20, 0x40, 0x60
# alu ops
ADD, SUB, MUL, DIV, OR, AND, LSH, RSH, NEG, MOD, XOR, MOV, ARSH, END = (
    0x00, 0x10, 0x20, 0x30, 0x40, 0x50, 0x60, 0x70, 0x80, 0x90, 0xA0, 0xB0, 0xC0, 0xD0)
# jump ops
JA, JEQ, JGT, JGE, JSET, JNE, JSGT, JSGE, CALL, EXIT, JLT, JLE, JSLT, JSLE = (
    0x00, 0x10, 0x20, 0x30, 0x40, 0x50, 0x60, 0x70, 0x80, 0x90, 0xA0, 0xB0, 0xC0, 0xD0)

ALU_OPS = {"add": ADD, "sub": SUB, "mul": MUL, "div": DIV, "or": OR, "and": AND, "lsh": LSH,
           "rsh": RSH, "mod": MOD, "xor": XOR, "mov": MOV, "arsh": ARSH, "neg": NEG}
JMP_OPS = {"jeq": JEQ, "jgt": JGT, "jge": JGE, "jset": JSET, "jne": JNE, "jsgt": JSGT,
           "jsge": JSGE, "jlt": JLT, "jle": JLE, "jslt": JSLT, "jsle": JSLE}

PSEUDO_MAP_FD = 1
PSEUDO_MAP_VALUE = 2
PSEUDO_CALL = 1

# helper ids (Linux uapi numbering; asm.FnMapLookupElem ...)
FN_MAP_LOOKUP_ELEM = 1
FN_MAP_UPDATE_ELEM = 2
FN_MAP_DELETE_ELEM = 3
FN_GET_SMP_PROCESSOR_ID = 8
FN_TAIL_CALL = 12
FN_XDP_ADJUST_TAIL = 65

XDP_ABORTED, XDP_DROP, XDP_PASS, XDP_TX, XDP_REDIRECT = range(5)
TC_ACT_OK, TC_ACT_SHOT = 0, 2

# __sk_buff field offsets (include/uapi/linux/bpf.h; SKBuff.convertAccess, emulator_linux_sk_buff.go:295-676)
SKB = dict(len=0, pkt_type=4, mark=8, queue_mapping=12, protocol=16, vlan_present=20, vlan_tci=24, vlan_proto=28,
           priority=32, ingress_ifindex=36, ifindex=40, tc_index=44, cb=48, hash=68, tc_classid=72, data=76,
           data_end=80, napi_id=84, family=88, remote_ip4=92, local_ip4=96, remote_ip6=100, local_ip6=116,
           remote_port=132, local_port=136, data_meta=140, flow_keys=144, tstamp=152, wire_len=160, gso_segs=164,
           sk=168, gso_size=176, hwtstamp=184)
# struct bpf_sock (SK.convertAccess :772-918) and struct bpf_flow_keys (:1031-1175)
SOCK = dict(bound_dev_if=0, family=4, type=8, protocol=12, mark=16, priority=20, src_ip4=24, src_ip6=28,
            src_port=44, dst_port=48, dst_ip4=52, dst_ip6=56, state=72, rx_queue_mapping=76)
FLOW_KEYS = dict(nhoff=0, thoff=2, addr_proto=4, is_frag=6, is_first_frag=7, is_encap=8, ip_proto=9, n_proto=10,
                 sport=12, dport=14, ipv4_src=16, ipv4_dst=20, ipv6_src=16, flags=32, flow_label=36)


@dataclass
class Insn:
    op: int
    dst: int = 0
    src: int = 0
    off: Union[int, str] = 0
    imm: Union[int, str] = 0
    imm64: Optional[int] = None     # set for LD_IMM64 (two slots)
    map_ref: Optional[str] = None   # symbolic map reference for relocation

    @property
    def slots(self) -> int:
        return 2 if self.op == (LD | IMM | DW) else 1


Item = Union[Insn, str]  # a str is a label


def _s16(v: int) -> int:
    if not -0x8000 <= v <= 0x7FFF:
        raise ValueError(f"offset {v} does not fit int16")
    return v


def _u32(v: int) -> int:
    return v & 0xFFFFFFFF


def encode(op: int, dst: int = 0, src: int = 0, off: int = 0, imm: int = 0) -> bytes:
    return struct.pack("<BBhI", op & 0xFF, (dst & 0xF) | ((src & 0xF) << 4), _s16(off), _u32(imm))


def assemble(items: Sequence[Item]) -> Tuple[bytes, List[Tuple[int, str]]]:
    """Assemble ``items`` -> (raw bytes, [(slot, map_name)] relocations).

    String items are labels; an ``Insn`` whose ``off`` is a label string jumps to it
    (offset = target - (slot + 1)); a CALL with ``imm`` as a label is a BPF-to-BPF call
    (imm = target - slot - 1, the value cilium's fixupJumpsAndCalls writes, vm.go:168)."""
    labels = {}
    slot = 0
    for it in items:
        if isinstance(it, str):
            if it in labels:
                raise ValueError(f"duplicate label {it}")
            labels[it] = slot
        else:
            slot += it.slots
    out = bytearray()
    relocs: List[Tuple[int, str]] = []
    slot = 0
    for it in items:
        if isinstance(it, str):
            continue
        off = it.off
        if isinstance(off, str):
            off = labels[off] - (slot + 1)
        imm = it.imm
        if isinstance(imm, str):
            imm = labels[imm] - slot - 1
        if it.slots == 2:
            v = it.imm64 if it.imm64 is not None else imm
            v &= 0xFFFFFFFFFFFFFFFF
            out += encode(it.op, it.dst, it.src, off, v & 0xFFFFFFFF)
            out += struct.pack("<BBhI", 0, 0, 0, v >> 32)
            if it.map_ref is not None:
                relocs.append((slot, it.map_ref))
        else:
            out += encode(it.op, it.dst, it.src, off, imm)
        slot += it.slots
    return bytes(out), relocs


# --- convenience constructors ------------------------------------------------------------

def alu64(op: str, dst: int, src_or_imm: int, reg: bool = False) -> Insn:
    return Insn(ALU64 | ALU_OPS[op] | (X if reg else K), dst, src_or_imm if reg else 0, 0,
                0 if reg else src_or_imm)


def alu32(op: str, dst: int, src_or_imm: int, reg: bool = False) -> Insn:
    return Insn(ALU | ALU_OPS[op] | (X if reg else K), dst, src_or_imm if reg else 0, 0,
                0 if reg else src_or_imm)


def mov64_imm(dst: int, imm: int) -> Insn:
    return alu64("mov", dst, imm)


def mov64_reg(dst: int, src: int) -> Insn:
    return alu64("mov", dst, src, reg=True)


def mov32_imm(dst: int, imm: int) -> Insn:
    return alu32("mov", dst, imm)


def ld_imm64(dst: int, value: int) -> Insn:
    return Insn(LD | IMM | DW, dst, 0, 0, 0, imm64=value)


def ld_map_fd(dst: int, map_name: str) -> Insn:
    return Insn(LD | IMM | DW, dst, PSEUDO_MAP_FD, 0, 0, imm64=0, map_ref=map_name)


def ld_map_value(dst: int, map_name: str, off: int = 0) -> Insn:
    return Insn(LD | IMM | DW, dst, PSEUDO_MAP_VALUE, off, 0, imm64=0, map_ref=map_name)


def ldx(size: int, dst: int, src: int, off: int) -> Insn:
    return Insn(LDX | MEM | SIZE_BYTES[size], dst, src, off, 0)


def stx(size: int, dst: int, off: int, src: int) -> Insn:
    return Insn(STX | MEM | SIZE_BYTES[size], dst, src, off, 0)


def st(size: int, dst: int, off: int, imm: int) -> Insn:
    return Insn(ST | MEM | SIZE_BYTES[size], dst, 0, off, imm)


def jmp(op: str, dst: int, src_or_imm: int, off: Union[int, str], reg: bool = False) -> Insn:
    return Insn(JMP | JMP_OPS[op] | (X if reg else K), dst, src_or_imm if reg else 0, off,
                0 if reg else src_or_imm)


def jmp32(op: str, dst: int, src_or_imm: int, off: Union[int, str], reg: bool = False) -> Insn:
    return Insn(JMP32 | JMP_OPS[op] | (X if reg else K), dst, src_or_imm if reg else 0, off,
                0 if reg else src_or_imm)


def ld_abs(size: int, imm: int) -> Insn:
    """LD_ABS: R0 = ntoh(*(size *)(skb->data + imm)), R1-R5 clobbered (emulator_linux_.go:200-238)."""
    return Insn(LD | ABS | SIZE_BYTES[size], 0, 0, 0, imm)


def ld_ind(size: int, src: int, imm: int) -> Insn:
    """LD_IND: R0 = ntoh(*(size *)(skb->data + src + imm)) (emulator_linux_.go:240-284)."""
    return Insn(LD | IND | SIZE_BYTES[size], 0, src, 0, imm)


def ja(off: Union[int, str]) -> Insn:
    return Insn(JMP | JA, 0, 0, off, 0)


def call(helper: int) -> Insn:
    return Insn(JMP | CALL, 0, 0, 0, helper)


def call_local(label: str) -> Insn:
    return Insn(JMP | CALL, 0, PSEUDO_CALL, 0, label)


def exit_() -> Insn:
    return Insn(JMP | EXIT)


def raw(op: int, dst: int = 0, src: int = 0, off: int = 0, imm: int = 0) -> Insn:
    return Insn(op, dst, src, off, imm)


def slots(raw_bytes: bytes) -> int:
    return len(raw_bytes) // 8
