"""Tiny eBPF disassembler for debugging (raw slots -> text)."""
import struct, sys

ALU = {0x00: "add", 0x10: "sub", 0x20: "mul", 0x30: "div", 0x40: "or", 0x50: "and", 0x60: "lsh", 0x70: "rsh",
       0x80: "neg", 0x90: "mod", 0xa0: "xor", 0xb0: "mov", 0xc0: "arsh", 0xd0: "end"}
JMP = {0x00: "ja", 0x10: "jeq", 0x20: "jgt", 0x30: "jge", 0x40: "jset", 0x50: "jne", 0x60: "jsgt", 0x70: "jsge",
       0x80: "call", 0x90: "exit", 0xa0: "jlt", 0xb0: "jle", 0xc0: "jslt", 0xd0: "jsle"}
SZ = {0x00: "u32", 0x08: "u16", 0x10: "u8", 0x18: "u64"}


def disasm(raw: bytes):
    out = []
    for i in range(len(raw) // 8):
        op, regs, off, imm = struct.unpack_from("<BBhi", raw, 8 * i)
        dst, src = regs & 0xF, regs >> 4
        cls = op & 7
        x = op & 8
        if cls in (4, 7):
            n = ALU.get(op & 0xF0, "?") + ("64" if cls == 7 else "32")
            t = f"{n} r{dst}, " + (f"r{src}" if x else f"{imm}")
        elif cls in (5, 6):
            n = JMP.get(op & 0xF0, "?") + ("32" if cls == 6 else "")
            t = f"{n} r{dst}, " + (f"r{src}" if x else f"{imm}") + f", {off:+d} -> {i + off + 1}"
        elif cls == 1:
            t = f"r{dst} = *({SZ[op & 0x18]}*)(r{src}{off:+d})"
        elif cls == 3:
            t = f"*({SZ[op & 0x18]}*)(r{dst}{off:+d}) = r{src}"
        elif cls == 2:
            t = f"*({SZ[op & 0x18]}*)(r{dst}{off:+d}) = {imm}"
        else:
            t = f"ld op={op:#x} r{dst} src={src} imm={imm}"
        out.append(f"{i:4d}: {op:02x} {t}")
    return "\n".join(out)
