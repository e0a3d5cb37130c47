"""GPU parity for the sk_buff context (config 5): the HIP engine vs the CPU oracle, bit-exact,
through the C ABI (mimic_run_skb).  Covers the hand-derived vectors of kat_skb.json, random
programs over header variants, the config-5 tail-call chain with hash / per-CPU maps, the
leaked-entry address layout across batches, and the API rules around it."""
import numpy as np
import pytest

import kat_skb
from fuzz_skb import random_skb_program
from harness import (Scenario, assert_same, assert_same_sequence, build_engine, kernel_of, run_engine_skb, run_oracle_skb,
                     run_sequence_engine, run_sequence_oracle)
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu

CASES = kat_skb.load_cases()
GROUPS = kat_skb.jit_groups(CASES)


def _fuzz(seed):
    rng = np.random.default_rng(7000 + seed)
    raw, rel = random_skb_program(rng, n_ops=int(rng.integers(3, 16)))
    return Scenario(vcpus=8, progs=[("fz", raw, rel)]), rng


def jit_kernels():
    ks = [kernel_of(sc, 1) for sc, _, _ in GROUPS] + [kernel_of(_fuzz(s)[0], 1) for s in range(24)]
    progs, _, _ = W.skb_programs()
    from mimic_amd import asm as A
    return ks + [([p.raw for p in progs], 1), ([A.assemble([A.ldx(4, 0, 1, A.SKB["data"]), A.exit_()])[0]], 1),
                 ([A.assemble([A.ldx(4, 0, 1, A.SKB["sk"]), A.exit_()])[0]], 1)]


def _skb_kat(c, exec_mode):
    sc = kat_skb.scenario(c)
    inp = kat_skb.inputs(c)
    e = run_engine_skb(sc, inp["buf"], inp["off"], inp["lens"], inp["cpu"], ifindex=inp["ifindex"], exec_mode=exec_mode,
                       custom=inp["custom"])
    kat_skb.check(c, e)
    o = run_oracle_skb(sc, inp["buf"], inp["off"], inp["lens"], inp["cpu"], ifindex=inp["ifindex"], custom=inp["custom"])
    assert_same(o, e)


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_skb_kat_interp(gpu, c):
    _skb_kat(c, "interp")


@pytest.mark.parametrize("g", range(len(GROUPS)))
def test_skb_kat_jit_chunk(gpu, g):
    """The vectors' programs in chunks, one JIT kernel per chunk, against the oracle running the
    same batch sequence on the same VM layout."""
    sc, runs, _ = GROUPS[g]
    e = run_sequence_engine(sc, runs, exec_mode="jit")
    assert_same_sequence(run_sequence_oracle(sc, runs), e, tag=f"skb chunk {g}")
    assert any(r["last_exec"] == "jit" for r in e[0])


@pytest.mark.parametrize("seed", range(24))
def test_skb_fuzz(gpu, seed):
    sc, rng = _fuzz(seed)
    buf, off, lens = W.make_skb_packets(96, sizes=(14, 40, 64, 128, 576), weights=(1, 1, 3, 2, 1), seed=seed,
                                        variety=0.6)
    cpu = rng.integers(0, 8, len(lens)).astype(np.int32)
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=3, step_budget=5000)
    e = run_engine_skb(sc, buf, off, lens, cpu, ifindex=3, step_budget=5000)
    assert_same(o, e)


def _cfg5(vcpus: int, buf, off, lens):
    progs, maps, pa = W.skb_programs()
    init = [("flows", k, v, 0) for k, v in W.skb_flow_keys(buf, off, lens)]
    return Scenario(vcpus=vcpus, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa,
                    map_init=init)


@pytest.mark.parametrize("variety", [0.0, 0.3])
def test_cfg5_chain_small(gpu, variety):
    buf, off, lens = W.make_skb_packets(4096, **W.IMIX, variety=variety)
    sc = _cfg5(64, buf, off, lens)
    cpu = W.schedule_cpu(len(lens), 64, "chunked")
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=2)
    e = run_engine_skb(sc, buf, off, lens, cpu, ifindex=2)
    assert_same(o, e)
    ok = o["status"] == 0
    assert ok.mean() > 0.5
    assert set(np.unique(o["r0"][ok])) <= {0, 1, 2}


def test_cfg5_multi_batch_leaks(gpu):
    """Three batches on one VM: the leaked sock / flow-keys / packet entries of earlier batches
    move every later process's addresses (data, data_end, sk, flow_keys)."""
    buf, off, lens = W.make_skb_packets(3000, **W.IMIX, variety=0.2)
    sc = _cfg5(32, buf, off, lens)
    cpu = W.schedule_cpu(len(lens), 32, "interleaved")
    o = run_oracle_skb(sc, buf, off, lens, cpu, splits=[1000, 2100])
    e = run_engine_skb(sc, buf, off, lens, cpu, splits=[1000, 2100])
    assert_same(o, e)


def test_leaked_addresses_across_batches(gpu):
    """r0 = skb->data for every packet, in two batches on one VM."""
    from mimic_amd import asm as A

    raw, _ = A.assemble([A.ldx(4, 0, 1, A.SKB["data"]), A.exit_()])
    sc = Scenario(vcpus=4, progs=[("d", raw, [])])
    buf, off, lens = W.make_skb_packets(500, sizes=(60, 300, 1500), weights=(2, 1, 1), variety=0.3)
    cpu = W.schedule_cpu(len(lens), 4, "chunked")
    o = run_oracle_skb(sc, buf, off, lens, cpu, splits=[233])
    e = run_engine_skb(sc, buf, off, lens, cpu, splits=[233])
    assert_same(o, e)
    ok = o["status"] == 0
    assert len(np.unique(o["r0"][ok])) == ok.sum()   # every process got a fresh packet entry


def test_leak_prefix_large_batches(gpu):
    """r0 = skb->data over two batches of ~150 K packets (1 172 prep blocks in all, so the block
    offsets kernel scans two sums per thread): the first 1 000 processes equal the oracle's, and
    every process's packet entry follows the previous one's by its leak footprint 219 + L
    (context_sk_buff.go:73-95: sock 80+1, flow keys 40+1, packet 32+L+64+1), across the batch
    boundary too.  A size-independent check of the two-part leak prefix (skb.hip)."""
    from mimic_amd import asm as A

    raw, _ = A.assemble([A.ldx(4, 0, 1, A.SKB["data"]), A.exit_()])
    sc = Scenario(vcpus=1024, progs=[("d", raw, [])])
    n = 300_001
    buf, off, lens = W.make_skb_packets(n, sizes=(60, 64, 200), weights=(2, 3, 1), variety=0.05)
    cpu = W.schedule_cpu(n, 1024, "interleaved")
    e = run_engine_skb(sc, buf, off, lens, cpu, splits=[150_001])
    m = 1000
    o = run_oracle_skb(sc, buf, off[:m], lens[:m], cpu[:m])
    assert_same(o, e, check_pkt=False, n=m)
    ok = np.asarray(e["status"]) == 0
    assert ok.mean() > 0.9
    d = np.asarray(e["r0"], dtype=np.int64)[ok]
    L = np.asarray(lens, dtype=np.int64)[ok]
    assert np.array_equal(np.diff(d), 219 + L[:-1])


@pytest.mark.slow
def test_cfg5_large(gpu):
    """Config 5 shape at 65 536 IMIX packets, 16 384 vCPUs: exact against the oracle.  (The
    oracle's time grows with the square of the batch: every process leaks three memory-controller
    entries and AddEntry's first-fit scan walks them all, memory_controller.go:58-112.)"""
    n, V = 1 << 16, 1 << 14
    buf, off, lens = W.make_skb_packets(n, **W.IMIX, variety=0.05)
    sc = _cfg5(V, buf, off, lens)
    cpu = W.schedule_cpu(n, V, "chunked")
    o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=1)
    e = run_engine_skb(sc, buf, off, lens, cpu, ifindex=1)
    assert_same(o, e)


def test_skb_api_rules(gpu):
    """xdp_md batches, new maps and new programs are refused while sk_buff leaks exist (first
    fit would place them in the freed stack / sk_buff hole); SKBRelease resets the VM's layout."""
    import mimic_amd as M
    from mimic_amd import asm as A

    raw, _ = A.assemble([A.mov64_imm(0, 2), A.exit_()])
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(2))
    pid = vm.AddProgram(M.ProgramSpec("p", raw, []))
    sb = M.SKBBatch.from_packets([bytes(64)] * 4, device="cuda:0")
    r = vm.RunSKBBatch(pid, sb)
    assert r.numpy(4)["r0"].tolist() == [2] * 4
    xb = M.XDPBatch.from_packets([bytes(64)], device="cuda:0")
    with pytest.raises(M.MimicError):
        vm.RunXDPBatch(pid, xb)
    with pytest.raises(M.MimicError):
        vm.AddProgram(M.ProgramSpec("q", raw, []))
    vm.SKBRelease()
    assert vm.RunXDPBatch(pid, xb).numpy(1)["r0"].tolist() == [2]
    vm.close()


def test_process_run_skb(gpu):
    """Process.Run with a LinuxContextSKBuff: one process at a time, leaks accumulate like the
    reference's (the second process's skb->sk is 219 + L above the first's)."""
    import mimic_amd as M
    from mimic_amd import asm as A

    raw, _ = A.assemble([A.ldx(4, 0, 1, A.SKB["sk"]), A.exit_()])
    emu = M.NewLinuxEmulator()
    vm = M.NewVM(M.VMOptEmulator(emu), M.VMOptSetvCPUs(1))
    pid = vm.AddProgram(M.ProgramSpec("p", raw, []))
    got = []
    for L in (64, 100):
        p = vm.NewProcess(pid, M.LinuxContextSKBuff(Packet=bytes(L), Dev=M.NetDev(3)))
        p.SetCPUID(0)
        p.Run()
        got.append(p.Registers.R0)
    assert got[1] - got[0] == 219 + 64
    ctx = M.UnmarshalContextJSON('{"name": "x", "type": "sk_buff", "ctx": {"packet": "AAAA", "dev": {"ifIndex": 4}}}')
    assert isinstance(ctx, M.LinuxContextSKBuff) and ctx.Dev.IFIndex == 4 and ctx.Packet == b"\0\0\0"
    vm.close()


@pytest.mark.parametrize("name", ["sock_family", "sock_ip4_16_bytes", "sock_rxq_u64", "fk_user_flow_label", "sock_and_fk",
                                  "sock_nil_ips", "fk_user_store"])
def test_process_with_user_sock_and_flow_keys(gpu, name):
    """NewProcess over an sk_buff context with a user-given sock / flow keys
    (mimic_process_new_skb_ctx, context_sk_buff.go:53-66), run to the end: the vector's answer."""
    import mimic_amd as M
    from mimic_amd import vm as V

    c = next(c for c in CASES if c["name"] == name)
    table = kat_skb.custom_table(c["contexts"])
    vm = M.NewVM(M.VMOptEmulator(M.NewLinuxEmulator()), M.VMOptSetvCPUs(1))
    pid = vm.AddProgram(M.ProgramSpec("main", bytes.fromhex(c["raw"])))
    for k, (pkt, ex) in enumerate(zip(c["packets"], c["expect"])):
        cj = c["contexts"][k] or {}
        sk = M.SK.FromJSON(cj["sock"]) if cj.get("sock") is not None else None
        if sk is not None and cj.get("nilIPs"):
            sk.ips = None
        fk = M.FlowKeys.FromJSON(cj["flowKeys"]) if cj.get("flowKeys") is not None else None
        ctx = M.LinuxContextSKBuff(Packet=bytes.fromhex(pkt), SK=sk, FlowKeys=fk, Dev=M.NetDev(c["ifindex"]))
        assert V.skb_custom_record(ctx).tobytes() == table[k].tobytes()
        p = vm.NewProcess(pid, ctx)
        p.SetCPUID(0)
        try:
            p.Run()
        except M.MimicError:
            pass
        assert p.Status == ex["status"], (name, k, p.Status)
        if "r0" in ex and ex["status"] == 0:
            assert p.Registers.R0 == ex["r0"], (name, k, hex(p.Registers.R0))
        p.Cleanup()
    vm.close()


@pytest.mark.parametrize("exec_mode", ["jit", "interp"])
def test_rooms_clean_word(gpu, exec_mode):
    """mimic_skb_batch.rooms_state: one batch launched three times.  A program that reads a headroom
    and a tailroom byte (R0 = tail << 8 | head) and then writes them must see zero rooms every time
    (Load hands over zeroed rooms, context_sk_buff.go:42-107): its room stores set the word back to
    0, so the next launch's prep reads the rooms and the chain zeroes them.  A program that never
    touches a room leaves the word at 1 (the next prep reads no room) and stays exact.  A program that
    stores into the frame only keeps the word at 1 on the JIT (its frame-only fast store) and sets it
    to 0 on the interpreter (whose every packet store marks, runtime.h skb_room_mark): both exact."""
    import mimic_amd as M
    from mimic_amd import asm as A

    S = A.SKB
    rooms_rw, _ = A.assemble([
        A.ldx(4, 2, 1, S["data"]), A.ldx(4, 3, 1, S["len"]), A.mov64_reg(4, 2), A.alu64("add", 4, 3, reg=True),
        A.ldx(1, 5, 2, -1), A.ldx(1, 6, 4, 3),                  # headroom byte, tailroom byte
        A.mov64_reg(0, 6), A.alu64("lsh", 0, 8), A.alu64("or", 0, 5, reg=True),
        A.alu64("add", 5, 1), A.stx(1, 2, -1, 5), A.alu64("add", 6, 2), A.stx(1, 4, 3, 6),
        A.exit_()])
    quiet, _ = A.assemble([A.ldx(4, 2, 1, S["data"]), A.ldx(1, 0, 2, 0), A.exit_()])
    frame_w, _ = A.assemble([A.ldx(4, 2, 1, S["data"]), A.mov64_imm(3, 0x5A), A.stx(1, 2, 0, 3),
                             A.mov64_imm(0, 7), A.exit_()])   # the frame's first byte := 0x5A
    buf, off, lens = W.make_skb_packets(3000, sizes=(60, 300, 1500), weights=(2, 1, 1), seed=41)
    for name, raw, touches in (("rooms_rw", rooms_rw, True), ("quiet", quiet, False),
                               ("frame_w", frame_w, exec_mode == "interp")):
        sc = Scenario(vcpus=8, progs=[(name, raw, [])])
        cpu = W.schedule_cpu(len(lens), 8, "chunked")
        o = run_oracle_skb(sc, buf, off, lens, cpu, ifindex=1)
        assert (o["status"] == 0).all() and (o["r0"] == 0).all() if name == "rooms_rw" else True
        vm, maps, pids = build_engine(sc, ctx=1, exec_mode=exec_mode)
        batch = M.SKBBatch.from_numpy(buf, off, lens, device="cuda:0", ifindex=1, schedule=M.SCHED_EXPLICIT, cpu=cpu)
        for k in range(3):
            e = vm.RunSKBBatch(pids[0], batch).numpy(len(lens))
            for f in ("r0", "status", "steps"):
                assert np.array_equal(np.asarray(o[f]).astype(np.int64), np.asarray(e[f]).astype(np.int64)), (name, k, f)
            assert int(batch.rooms_state.item()) == (0 if touches else 1), (name, k)
            vm.SKBRelease()
        assert np.array_equal(o["pkt"], batch.pkt_data.cpu().numpy()), name
        vm.close()
