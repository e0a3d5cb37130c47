"""Run(ctx) on the CPU (vm.go:343-360): the native context object (cancel, deadline timer, the
first reason kept) and the oracle's restatement of the check before every step -- a process whose
context is done when Run starts takes no step and returns ctx.Err(), after NewProcess has loaded its
context (xdp_md rooms zeroed, sk_buff entries leaked), and leaves every map untouched."""
import time

import numpy as np
import pytest

import mimic_amd as M
from harness import Scenario, run_oracle, run_oracle_skb, packets_to_buffer, skb_packets_to_buffer
from mimic_amd import _lib
from mimic_amd import asm as A
from mimic_amd import workloads as W

CANCELED, DEADLINE = _lib.STATUS["ERR_CANCELED"], _lib.STATUS["ERR_DEADLINE"]


def test_status_codes():
    assert (CANCELED, DEADLINE) == (29, 30)


def test_native_cancel_keeps_the_first_reason():
    lib = _lib.load()
    c = M.WithCancel()
    h = c.native()
    assert c.Err() is None and lib.mimic_ctx_err(h) == 0 and not c.Done()
    c.Cancel()
    assert c.Err() == "context canceled" and lib.mimic_ctx_err(h) == 1
    c.Cancel()
    assert lib.mimic_ctx_err(h) == 1
    d = M.WithTimeout(0.02)
    hd = d.native()
    time.sleep(0.1)
    assert lib.mimic_ctx_err(hd) == 2 and d.Err() == "context deadline exceeded"
    d.Cancel()   # cancel after the deadline: Err() stays DeadlineExceeded (context.go)
    assert lib.mimic_ctx_err(hd) == 2
    c.close()
    d.close()


def test_free_with_a_pending_timer_returns_at_once():
    import ctypes as C

    lib = _lib.load()
    h = C.c_void_p()
    assert lib.mimic_ctx_new(int(60e9), C.byref(h)) == 0
    t = time.monotonic()
    lib.mimic_ctx_free(h)
    assert time.monotonic() - t < 1.0


def test_python_deadline_before_the_handle():
    c = M.WithTimeout(0.0)
    assert c.Err() == "context deadline exceeded"
    assert M.Background().Err() is None
    with pytest.raises(M.MimicError):
        M.vm._ctx_args(M.WithCancel(), [None], 1)


def _count_prog():
    """c[0] += 1 (per-CPU), r0 = data_end - data, and one byte written into the packet."""
    raw, rel = A.assemble([A.mov64_reg(6, 1), A.ldx(4, 7, 6, 0), A.ldx(4, 8, 6, 4), A.st(1, 7, 0, 0x5a),
                           A.st(4, 10, -4, 0), A.mov64_reg(2, 10), A.alu64("add", 2, -4), A.ld_map_fd(1, "c"),
                           A.call(A.FN_MAP_LOOKUP_ELEM), A.jmp("jeq", 0, 0, "out"), A.ldx(8, 3, 0, 0),
                           A.alu64("add", 3, 1), A.stx(8, 0, 0, 3), "out", A.mov64_reg(0, 8),
                           A.alu64("sub", 0, 7, reg=True), A.exit_()])
    return Scenario(vcpus=4, maps=[dict(name="c", type=6, key_size=4, value_size=8, max_entries=1)],
                    progs=[("cnt", raw, rel)])


def test_oracle_done_contexts_take_no_step():
    sc = _count_prog()
    rng = np.random.default_rng(5)
    pkts = [bytes(rng.integers(1, 255, int(L), dtype=np.uint8)) for L in rng.integers(14, 200, 64)]
    buf, off, lens = packets_to_buffer(pkts, headroom=8, tailroom=8)
    buf[:] = np.where(buf == 0, 0x77, buf)   # rooms non-zero: Load zeroes them
    cpu = (np.arange(64) % 4).astype(np.int32)
    done = rng.choice([0, 0, 1, 2], 64).astype(np.uint8)
    o = run_oracle(sc, buf, off, lens, cpu, headroom=8, tailroom=8, ctx_done=done)
    live = done == 0
    assert (o["status"][~live] == 28 + done[~live]).all()
    assert (o["steps"][~live] == 0).all() and (o["r0"][~live] == 0).all() and (o["err_pc"][~live] == 0).all()
    assert (o["status"][live] == 0).all() and (o["r0"][live] == lens[live]).all()
    # the per-CPU counters saw only the live processes
    per_cpu = [int(np.frombuffer(v, np.uint64)[0]) for v in o["maps"]["c"]]
    assert per_cpu == [int((live & (cpu == c)).sum()) for c in range(4)]
    # a done process's packet memory: its rooms zeroed by Load, its packet bytes untouched
    for i in np.nonzero(~live)[0]:
        a, L = int(off[i]), int(lens[i])
        mem = o["pkt"][a:a + 16 + L]
        assert not mem[:8].any() and not mem[8 + L:].any()
        assert mem[8] == buf[a + 8]
    # the same as a batch of the live packets only
    keep = np.nonzero(live)[0]
    b2, o2, l2 = packets_to_buffer([pkts[i] for i in keep], headroom=8, tailroom=8)
    r = run_oracle(sc, b2, o2, l2, cpu[keep], headroom=8, tailroom=8)
    assert (r["r0"] == o["r0"][keep]).all() and (r["steps"] == o["steps"][keep]).all()
    assert r["maps"] == o["maps"]


def test_oracle_skb_done_contexts_still_load():
    """sk_buff: a done context's process has loaded (its entries leak), so the next processes'
    addresses are those of a run where nothing was canceled."""
    raw, _ = A.assemble([A.ldx(4, 0, 1, A.SKB["data"]), A.exit_()])
    sc = Scenario(vcpus=4, progs=[("d", raw, [])])
    buf, off, lens = W.make_skb_packets(200, sizes=(60, 300), weights=(2, 1), variety=0.2)
    cpu = W.schedule_cpu(len(lens), 4, "chunked")
    done = np.zeros(len(lens), np.uint8)
    done[::3] = 1
    done[1::7] = 2
    a = run_oracle_skb(sc, buf, off, lens, cpu)
    b = run_oracle_skb(sc, buf, off, lens, cpu, ctx_done=done)
    loaded = a["status"] != _lib.STATUS["ERR_CTX_LOAD"]
    live = (done == 0) & loaded
    assert (b["r0"][live] == a["r0"][live]).all()
    assert (b["status"][(done > 0) & loaded] == 28 + done[(done > 0) & loaded]).all()
    assert (b["status"][~loaded] == _lib.STATUS["ERR_CTX_LOAD"]).all()   # Load fails before Run
