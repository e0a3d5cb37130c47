"""Shared test harness: build the same VM (maps, programs, prog-array entries) on the CPU
oracle and on the GPU engine, run one xdp_md batch on both, compare everything."""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from mimic_amd import asm as A  # noqa: E402


@dataclass
class Scenario:
    vcpus: int = 4
    maps: List[dict] = field(default_factory=list)          # name,type,key_size,value_size,max_entries[,datasec]
    progs: List[Tuple[str, bytes, List[Tuple[int, str]]]] = field(default_factory=list)
    prog_array: List[Tuple[str, int, int]] = field(default_factory=list)  # (map, key, prog index)
    map_init: List[Tuple[str, bytes, bytes, int]] = field(default_factory=list)  # (map, key, value, cpu)
    max_tail_calls: int = 33


HASH_TYPES = (1, 13, 18, 19, 24, 25, 26, 28, 29)
PERCPU_HASH_TYPES = (5, 21)


def ncpus(sc: Scenario, m: dict) -> int:
    return sc.vcpus if m["type"] in (5, 6, 21) else 1


def is_hash(m: dict) -> bool:
    return m["type"] in HASH_TYPES + PERCPU_HASH_TYPES


def build_oracle(sc: Scenario):
    import oracle

    vm = oracle.OracleVM(sc.vcpus, 256, 8, sc.max_tail_calls)
    mids = {}
    for m in sc.maps:
        mids[m["name"]] = vm.map_create(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"],
                                        m.get("datasec", False))
    pids = []
    for name, raw, rel in sc.progs:
        pids.append(vm.prog_load(name, raw, [(s, mids[n]) for s, n in rel]))
    for mname, key, pi in sc.prog_array:
        rc = vm.map_update(mids[mname], key.to_bytes(4, "little"), vm.prog_addr(pids[pi]).to_bytes(4, "little"))
        assert rc == 0
    for mname, key, val, cpu in sc.map_init:
        assert vm.map_update(mids[mname], key, val, 0, cpu) == 0
    return vm, mids, pids


def kernel_of(sc: Scenario, ctx: int = 0):
    """The JIT kernel a scenario's VM runs: (raw programs in load order, batch context, the
    LD_IMM64 slots the lane value cache may use) -- what a test module's jit_kernels() lists for
    the session prewarm (conftest.py)."""
    from mimic_amd import jit as J

    return [raw for _, raw, _ in sc.progs], ctx, J.vc_slots([(raw, rel) for _, raw, rel in sc.progs], sc.maps)


def spread_kernel_of(sc: Scenario, own: bool = False):
    """The spread kernel a scenario's VM builds (jit.spread_spec; own: its owned form): for the
    session prewarm."""
    from mimic_amd import jit as J

    progs = [(raw, rel) for _, raw, rel in sc.progs]
    return [raw for _, raw, _ in sc.progs], 0, (), J.spread_spec(progs, sc.maps, sc.vcpus, own=own)


def build_engine(sc: Scenario, device: int = 0, shard=None, ctx: int = 0, exec_mode: Optional[str] = None,
                 spread: Optional[int] = None):
    import mimic_amd as M

    emu = M.NewLinuxEmulator(M.OptMaxTailCalls(sc.max_tail_calls))
    opts = [M.VMOptEmulator(emu), M.VMOptSetvCPUs(sc.vcpus), M.VMOptDevice(device)]
    if shard is not None:
        opts.append(M.VMOptShard(*shard))
    if exec_mode is not None:
        opts.append(M.VMOptExecMode(exec_mode))
    if spread is not None:
        opts.append(M.VMOptSpread(spread))
    vm = M.NewVM(*opts)
    maps = {}
    for m in sc.maps:
        mm = M.MapSpecToLinuxMap(M.MapSpec(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"],
                                           m.get("datasec", False)))
        emu.AddMap(m["name"], mm)
        maps[m["name"]] = mm
    pids = [vm.AddProgram(M.ProgramSpec(name, raw, list(rel))) for name, raw, rel in sc.progs]
    for mname, key, pi in sc.prog_array:
        assert maps[mname].UpdateProgram(key.to_bytes(4, "little"), pids[pi]) == 0
    for mname, key, val, cpu in sc.map_init:
        assert maps[mname].Update(key, val, 0, cpu) == 0
    return vm, maps, pids


def packets_to_buffer(packets: Sequence[bytes], headroom=0, tailroom=0, align: int = 64):
    import mimic_amd as M

    lens = np.array([len(p) for p in packets], dtype=np.uint32)
    off, total = M.XDPBatch.layout(lens, headroom, tailroom, align)
    buf = np.zeros(max(total, 1), dtype=np.uint8)
    for i, p in enumerate(packets):
        h = headroom if np.isscalar(headroom) else int(headroom[i])
        buf[int(off[i]) + h:int(off[i]) + h + len(p)] = np.frombuffer(bytes(p), np.uint8)
    return buf, off, lens


def run_oracle(sc: Scenario, buf, off, lens, cpu, entry: int = 0, headroom=0, tailroom=0, ingress=None,
               rxq=None, egress=None, step_budget=0, ctx_done=None, ctx_done_step=None):
    """ctx_done: per packet, the state of its Run's context (0 not done, 1 canceled, 2 deadline)."""
    vm, mids, pids = build_oracle(sc)
    out = vm.run_xdp_batch(pids[entry], buf.copy(), off, lens, cpu, headroom, tailroom, ingress, rxq, egress,
                           step_budget, ctx_done=ctx_done, ctx_done_step=ctx_done_step)
    out["maps"] = {}
    out["hash"] = {}
    for m in sc.maps:
        vals = [vm.map_values(mids[m["name"]], c) for c in range(ncpus(sc, m))]
        out["maps"][m["name"]] = vals
        if is_hash(m):
            S = m["value_size"]
            out["hash"][m["name"]] = {k: [v[s * S:(s + 1) * S] for v in vals]
                                      for k, s in vm.map_entries(mids[m["name"]])}
    vm.close()
    return out


def run_engine(sc: Scenario, buf, off, lens, cpu=None, entry: int = 0, headroom=0, tailroom=0, ingress=0, rxq=0,
               egress=0, step_budget=0, schedule=None, device: int = 0, exec_mode: Optional[str] = None,
               spread: Optional[int] = None, ctx=None, ctx_per_packet=None):
    import mimic_amd as M

    vm, maps, pids = build_engine(sc, device, exec_mode=exec_mode, spread=spread)
    if schedule is None:
        schedule = M.SCHED_EXPLICIT
    batch = M.XDPBatch.from_numpy(buf, off, lens, device=f"cuda:{device}", headroom=headroom, tailroom=tailroom,
                                  ingress=ingress, rxq=rxq, egress=egress, schedule=schedule, cpu=cpu,
                                  step_budget=step_budget)
    res = vm.RunXDPBatch(pids[entry], batch, ctx=ctx, ctx_per_packet=ctx_per_packet)
    out = res.numpy(len(lens))
    out["pkt"] = batch.pkt_data.cpu().numpy()
    out["maps"] = {}
    out["hash"] = {}
    for m in sc.maps:
        out["maps"][m["name"]] = [maps[m["name"]].Values(c) for c in range(ncpus(sc, m))]
        if is_hash(m):
            out["hash"][m["name"]] = maps[m["name"]].Contents()
    out["steps_total"] = vm.LastSteps()
    out["last_exec"] = vm.LastExec()
    vm.close()
    return out


def assert_same(o, e, check_pkt: bool = True, n: Optional[int] = None, hash_exact: bool = True,
                check_steps: bool = True):
    """hash_exact=False: compare hash maps by key (the slot a key gets depends on the order in
    which concurrent vCPUs insert; the reference's processPool is no different).
    check_steps=False: a packet's path (found vs inserted) may depend on that order too."""
    for k in ("r0", "status", "steps", "err_pc"):
        if k == "steps" and not check_steps:
            continue
        a = np.asarray(o[k])
        b = np.asarray(e[k])
        if n is not None:
            a, b = a[:n], b[:n]
        a = a.astype(np.uint64) if k == "r0" else a.astype(np.int64)
        b = b.astype(np.uint64) if k == "r0" else b.astype(np.int64)
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{k} differs at {bad[:8]}: oracle={a[bad[:8]]} engine={b[bad[:8]]}"
    if check_pkt:
        assert np.array_equal(o["pkt"][:len(e["pkt"])], e["pkt"][:len(o["pkt"])]), "packet memory differs"
    for name, vals in o["maps"].items():
        if name in o.get("hash", {}):
            oh, eh = o["hash"][name], e["hash"][name]
            assert sorted(oh) == sorted(eh), f"hash map {name}: key sets differ ({len(oh)} vs {len(eh)} keys)"
            for key in oh:
                assert oh[key] == eh[key], f"hash map {name} key {key.hex()}: values differ"
            if not hash_exact:
                continue
        for c, v in enumerate(vals):
            assert v == e["maps"][name][c], f"map {name} cpu {c} differs"


def single(sc: Scenario, packet: bytes = b"\x00" * 64, cpu: int = 0, **kw):
    buf, off, lens = packets_to_buffer([packet], kw.pop("headroom", 0), kw.pop("tailroom", 0))
    return buf, off, lens, np.array([cpu], dtype=np.int32)


# ---------------------------------------------------------------------------------------------
# sk_buff batches (LinuxContextSKBuff): packet memory i = 32 + L + 64 bytes at off[i]
# ---------------------------------------------------------------------------------------------
SKB_ROOM = (32, 64)


def skb_packets_to_buffer(packets: Sequence[bytes], align: int = 64):
    return packets_to_buffer(packets, SKB_ROOM[0], SKB_ROOM[1], align)


def _splits(n: int, splits):
    if not splits:
        return [(0, n)]
    cuts = [0] + [int(s) for s in splits] + [n]
    return [(cuts[k], cuts[k + 1]) for k in range(len(cuts) - 1)]


def _map_readout(sc, read_values, read_hash):
    maps, hashes = {}, {}
    for m in sc.maps:
        vals = [read_values(m["name"], c) for c in range(ncpus(sc, m))]
        maps[m["name"]] = vals
        if is_hash(m):
            hashes[m["name"]] = read_hash(m, vals)
    return maps, hashes


def run_oracle_skb(sc: Scenario, buf, off, lens, cpu, entry: int = 0, ifindex: int = 0, step_budget: int = 0,
                   splits=None, custom=None, ctx_done=None):
    """Sequential reference semantics; `splits` = indices where a new batch (same VM) starts;
    custom = the contexts' mimic_skb_custom table (numpy) or None; ctx_done as in run_oracle."""
    vm, mids, pids = build_oracle(sc)
    buf = np.array(buf, dtype=np.uint8, copy=True)
    parts = []
    for a, b in _splits(len(lens), splits):
        parts.append(vm.run_skb_batch(pids[entry], buf, off[a:b], lens[a:b], cpu[a:b], ifindex, step_budget,
                                      custom=None if custom is None else custom[a:b],
                                      ctx_done=None if ctx_done is None else np.asarray(ctx_done)[a:b]))
    out = {k: np.concatenate([p[k] for p in parts]) for k in ("r0", "status", "steps", "err_pc")}
    out["pkt"] = buf

    def hread(m, vals):
        S = m["value_size"]
        return {k: [v[s * S:(s + 1) * S] for v in vals] for k, s in vm.map_entries(mids[m["name"]])}

    out["maps"], out["hash"] = _map_readout(sc, lambda name, c: vm.map_values(mids[name], c), hread)
    vm.close()
    return out


def run_engine_skb(sc: Scenario, buf, off, lens, cpu=None, entry: int = 0, ifindex: int = 0, step_budget: int = 0,
                   schedule=None, splits=None, device: int = 0, exec_mode: Optional[str] = None, custom=None,
                   ctx_per_packet=None):
    import torch

    import mimic_amd as M

    vm, maps, pids = build_engine(sc, device, ctx=1, exec_mode=exec_mode)
    if schedule is None:
        schedule = M.SCHED_EXPLICIT
    dev = f"cuda:{device}"
    full = M.SKBBatch.from_numpy(buf, off, lens, device=dev, ifindex=ifindex, custom=custom)
    CS = 136   # sizeof(mimic_skb_custom)
    parts = []
    for a, b in _splits(len(lens), splits):
        sub = M.SKBBatch(full.pkt_data, full.pkt_off[a:b], full.pkt_len[a:b], ifindex, schedule,
                         None if cpu is None else np.asarray(cpu)[a:b], step_budget,
                         None if full.custom is None else full.custom[a * CS:b * CS])
        parts.append(vm.RunSKBBatch(pids[entry], sub, ctx_per_packet=None if ctx_per_packet is None
                                    else ctx_per_packet[a:b]).numpy(b - a))
    out = {k: np.concatenate([p[k] for p in parts]) for k in ("r0", "status", "steps", "err_pc")}
    torch.cuda.synchronize(device)
    out["pkt"] = full.pkt_data.cpu().numpy()
    out["maps"], out["hash"] = _map_readout(sc, lambda name, c: maps[name].Values(c),
                                            lambda m, vals: maps[m["name"]].Contents())
    out["steps_total"] = vm.LastSteps()
    out["last_exec"] = vm.LastExec()
    vm.close()
    return out


# ---------------------------------------------------------------------------------------------
# sequences: many single batches, each with its own entry program, on ONE VM (one JIT kernel
# for all its programs).  The oracle runs the same sequence on the same layout.
# ---------------------------------------------------------------------------------------------
def _maps_out(sc, read_values, read_hash):
    maps, hashes = {}, {}
    for m in sc.maps:
        vals = [read_values(m["name"], c) for c in range(ncpus(sc, m))]
        maps[m["name"]] = vals
        if is_hash(m):
            hashes[m["name"]] = read_hash(m, vals)
    return maps, hashes


def run_sequence_oracle(sc: Scenario, runs):
    vm, mids, pids = build_oracle(sc)
    outs = []
    for r in runs:
        if r.get("skb"):
            b = np.array(r["buf"], dtype=np.uint8, copy=True)
            o = vm.run_skb_batch(pids[r["entry"]], b, r["off"], r["lens"], r["cpu"], r.get("ifindex", 0),
                                 r.get("step_budget", 0), custom=r.get("custom"))
            o["pkt"] = b
            outs.append(o)
            continue
        o = vm.run_xdp_batch(pids[r["entry"]], r["buf"].copy(), r["off"], r["lens"], r["cpu"], r.get("headroom", 0),
                             r.get("tailroom", 0), r.get("ingress"), r.get("rxq"), r.get("egress"),
                             r.get("step_budget", 0))
        outs.append(o)

    def hread(m, vals):
        S = m["value_size"]
        return {k: [v[s * S:(s + 1) * S] for v in vals] for k, s in vm.map_entries(mids[m["name"]])}

    maps, hashes = _maps_out(sc, lambda name, c: vm.map_values(mids[name], c), hread)
    vm.close()
    return outs, maps, hashes


def run_sequence_engine(sc: Scenario, runs, exec_mode: Optional[str] = None, device: int = 0):
    import mimic_amd as M

    vm, maps, pids = build_engine(sc, device, ctx=1 if runs and runs[0].get("skb") else 0, exec_mode=exec_mode)
    outs = []
    for r in runs:
        if r.get("skb"):
            sb = M.SKBBatch.from_numpy(r["buf"], r["off"], r["lens"], f"cuda:{device}", r.get("ifindex", 0),
                                       M.SCHED_EXPLICIT, r["cpu"], r.get("step_budget", 0), r.get("custom"))
            o = vm.RunSKBBatch(pids[r["entry"]], sb).numpy(len(r["lens"]))
            o["pkt"] = sb.pkt_data.cpu().numpy()
            o["last_exec"] = vm.LastExec()
            outs.append(o)
            continue
        zero = np.zeros(len(r["lens"]), np.int32)
        batch = M.XDPBatch.from_numpy(r["buf"], r["off"], r["lens"], device=f"cuda:{device}",
                                      headroom=r.get("headroom", 0), tailroom=r.get("tailroom", 0),
                                      ingress=r.get("ingress", zero), rxq=r.get("rxq", zero),
                                      egress=r.get("egress", zero), schedule=M.SCHED_EXPLICIT, cpu=r["cpu"],
                                      step_budget=r.get("step_budget", 0))
        o = vm.RunXDPBatch(pids[r["entry"]], batch).numpy(len(r["lens"]))
        o["pkt"] = batch.pkt_data.cpu().numpy()
        o["last_exec"] = vm.LastExec()
        outs.append(o)
    mp, hs = _maps_out(sc, lambda name, c: maps[name].Values(c), lambda m, vals: maps[m["name"]].Contents())
    vm.close()
    return outs, mp, hs


def assert_same_sequence(o, e, tag=""):
    oo, om, oh = o
    eo, em, eh = e
    assert len(oo) == len(eo)
    for k, (a, b) in enumerate(zip(oo, eo)):
        try:
            assert_same(dict(a, maps={}, hash={}), dict(b, maps={}, hash={}))
        except AssertionError as ex:
            raise AssertionError(f"{tag} run {k}: {ex}") from None
    if oo:  # final map contents
        assert_same(dict(oo[-1], maps=om, hash=oh), dict(eo[-1], maps=em, hash=eh), check_pkt=False)
