"""pcap ingest (mimic_amd.pcap): round trips in both timestamp resolutions and byte orders, the
batch layout it produces, and the oracle run over a pcap-sourced batch equal to the same
frames laid out directly."""
import struct

import numpy as np
import pytest

from harness import Scenario, packets_to_buffer, run_oracle
from mimic_amd import pcap
from mimic_amd import workloads as W


def _frames(n=50, seed=1):
    buf, off, lens = W.make_packets(n, **W.IMIX, seed=seed)
    return pcap.batch_to_frames(buf, off, lens)


@pytest.mark.parametrize("nanos", [False, True])
def test_round_trip(nanos):
    fr = _frames()
    ts = [1_700_000_000_123_456_789 + 1000 * i for i in range(len(fr))]
    data = pcap.write_pcap(fr, ts, nanos=nanos)
    buf, off, lens, t, lt = pcap.read_pcap(data, headroom=8, tailroom=4)
    assert lt == pcap.LINKTYPE_ETHERNET and len(lens) == len(fr)
    assert pcap.batch_to_frames(buf, off, lens, 8) == fr
    want = np.array(ts, np.uint64) if nanos else np.array(ts, np.uint64) // 1000 * 1000
    assert np.array_equal(t, want)
    assert all(int(o) % 64 == 0 for o in off)
    for o, n in zip(off, lens):       # room bytes are zero
        assert not buf[int(o):int(o) + 8].any() and not buf[int(o) + 8 + int(n):int(o) + 12 + int(n)].any()


def test_big_endian_and_errors():
    fr = _frames(5)
    le = pcap.write_pcap(fr)
    be = bytearray(struct.pack(">IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
    p = 24
    while p < len(le):
        sec, us, incl, orig = struct.unpack_from("<IIII", le, p)
        be += struct.pack(">IIII", sec, us, incl, orig) + le[p + 16:p + 16 + incl]
        p += 16 + incl
    assert pcap.batch_to_frames(*pcap.read_pcap(bytes(be))[:3]) == fr
    with pytest.raises(ValueError):
        pcap.read_pcap(b"\x0a\x0d\x0d\x0a" + bytes(40))       # pcapng
    with pytest.raises(ValueError):
        pcap.read_pcap(le[:-3])


def test_oracle_over_pcap_batch():
    fr = _frames(200, seed=4)
    p = W.prog_parse5()
    sc = Scenario(vcpus=8, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])
    b1, o1, l1, _, _ = pcap.read_pcap(pcap.write_pcap(fr))
    b2, o2, l2 = packets_to_buffer(fr)
    cpu = W.schedule_cpu(len(fr), 8, "chunked")
    r1, r2 = run_oracle(sc, b1, o1, l1, cpu), run_oracle(sc, b2, o2, l2, cpu)
    for k in ("r0", "status", "steps"):
        assert np.array_equal(r1[k], r2[k])
    assert r1["maps"] == r2["maps"]
