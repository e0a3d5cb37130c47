"""The hand assembler produces the Linux BPF encoding cilium/ebpf decodes."""
import struct

from mimic_amd import asm as A


def test_encoding_fields():
    raw = A.encode(0x07, 3, 5, -2, -1)
    op, regs, off, imm = struct.unpack("<BBhi", raw)
    assert (op, regs & 0xF, regs >> 4, off, imm) == (0x07, 3, 5, -2, -1)


def test_ld_imm64_two_slots_and_labels():
    raw, rel = A.assemble([A.ld_imm64(1, 0x1122334455667788), "x", A.ja("x"), A.ld_map_fd(2, "m"), A.exit_()])
    assert len(raw) == 8 * 6
    assert raw[0] == 0x18 and struct.unpack_from("<I", raw, 4)[0] == 0x55667788
    assert raw[8:12] == b"\x00" * 4 and struct.unpack_from("<I", raw, 12)[0] == 0x11223344
    assert struct.unpack_from("<h", raw, 16 + 2)[0] == -1  # ja x: x is slot 2, the ja itself
    assert rel == [(3, "m")]
    assert raw[8 * 3 + 1] >> 4 == A.PSEUDO_MAP_FD


def test_call_local_offset():
    raw, _ = A.assemble([A.call_local("f"), A.exit_(), "f", A.exit_()])
    assert struct.unpack_from("<i", raw, 4)[0] == 1  # target - slot - 1 (vm.go:168)
    assert raw[1] >> 4 == A.PSEUDO_CALL
