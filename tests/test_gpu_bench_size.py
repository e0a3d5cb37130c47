"""Every BASELINE.json config at the size bench.py measures it, against the oracle.

The inputs are bench.py's own `Workload` objects (same programs, maps, map contents, seeded
packets, vCPU count and schedule), so a green run here is parity for exactly the batches the
bench line times:

  cfg 2  classifier, 1 048 576 x 64 B, V = 262 144          (test_gpu_parity.py, full size)
  cfg 3  parse5, 16 777 216 IMIX, V = 262 144, interleaved   exact: per packet + every (cpu, key)
  cfg 4  flowtrack shard, 2 097 152 IMIX, E = 131 072, V = 262 144, interleaved
         per packet r0 / status exact, key -> value map exact (slots and the found / inserted
         path of a packet depend on which vCPU of a flow ran first, as in processPool)
  cfg 5  sk_buff 5-program tail-call chain, 1 048 576 IMIX, V = 131 072, interleaved
         exact: per packet r0 / status / steps / err_pc, packet memory, every map

Per-CPU maps make vCPUs independent, so the cfg-3 oracle runs in host threads, each one a VM
with the full V-vCPU layout running the packets of its own vCPU range in order
(vm.go:548-573: one worker per vCPU, its jobs in order).
"""
import os
import sys
import threading

import numpy as np
import pytest

from harness import Scenario, build_engine, build_oracle, kernel_of

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _scenario(wl, V) -> Scenario:
    return Scenario(vcpus=V, maps=list(wl.maps), progs=[(p.name, p.raw, p.relocs) for p in wl.progs],
                    prog_array=list(wl.prog_array), map_init=[(m, k, v, 0) for m, k, v in wl.map_init])


def jit_kernels():
    import bench

    out = []
    for name in ("parse5", "flowtrack", "skb"):
        cfg = bench.CONFIGS[name]
        from mimic_amd import workloads as W

        if cfg.get("kind") == "skb":
            progs, maps, pa = W.skb_programs()
            sc = Scenario(vcpus=1, maps=maps, progs=[(p.name, p.raw, p.relocs) for p in progs], prog_array=pa)
            out.append(kernel_of(sc, 1))
        else:
            p = getattr(W, cfg["prog"])()
            out.append(kernel_of(Scenario(vcpus=1, maps=p.maps, progs=[(p.name, p.raw, p.relocs)]), 0))
    return out


def _workload(name):
    import bench
    from mimic_amd import workloads as W

    cfg = bench.CONFIGS[name]
    n = cfg["packets"]
    return bench.Workload(name, n, W.SEED), n, cfg["vcpus"]


def _host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def _oracle_percpu_threads(sc, buf, off, lens, cpu, V, threads):
    """The oracle over vCPU ranges in parallel threads (valid when every map the programs write is
    per-CPU).  Returns per-packet results and, per per-CPU map, its (V, E*S) value rows."""
    n = len(lens)
    res = {"r0": np.zeros(n, np.uint64), "status": np.zeros(n, np.uint8), "steps": np.zeros(n, np.uint32),
           "err_pc": np.zeros(n, np.int32)}
    rows = {m["name"]: np.zeros((V, m["max_entries"] * m["value_size"]), np.uint8) for m in sc.maps if m["type"] == 6}
    shared = {}
    cuts = [V * t // threads for t in range(threads + 1)]
    errs = []

    def work(t):
        try:
            c0, c1 = cuts[t], cuts[t + 1]
            vm, mids, pids = build_oracle(sc)
            sel = np.nonzero((cpu >= c0) & (cpu < c1))[0]
            o = vm.run_xdp_batch(pids[0], buf, off[sel], lens[sel], cpu[sel], write_back=False)
            for k in res:
                res[k][sel] = o[k]
            for m in sc.maps:
                if m["type"] == 6:
                    for c in range(c0, c1):
                        rows[m["name"]][c] = np.frombuffer(vm.map_values(mids[m["name"]], c), np.uint8)
                else:
                    shared.setdefault(m["name"], []).append(vm.map_values(mids[m["name"]], 0))
            vm.close()
        except Exception as ex:  # surfaced below
            errs.append(ex)

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs, errs
    for name, vals in shared.items():   # read-only shared maps end equal on every thread
        assert all(v == vals[0] for v in vals), name
    return res, rows


def _engine_run(sc, wl, n, V, ctx=0):
    import torch

    import mimic_amd as M

    vm, maps, pids = build_engine(sc, 0, ctx=ctx)
    if ctx:
        batch = M.SKBBatch.from_numpy(wl.buf, wl.off, wl.lens, device="cuda:0", ifindex=1,
                                      schedule=M.SCHED_INTERLEAVED)
        res = vm.RunSKBBatch(pids[0], batch)
    else:
        batch = M.XDPBatch.from_numpy(wl.buf, wl.off, wl.lens, device="cuda:0", ingress=1,
                                      schedule=M.SCHED_INTERLEAVED)
        res = vm.RunXDPBatch(pids[0], batch)
    out = res.numpy(n)
    torch.cuda.synchronize()
    out["steps_total"] = vm.LastSteps()
    out["last_exec"] = vm.LastExec()
    return vm, maps, batch, out


def _same(o, e, keys=("r0", "status", "steps", "err_pc")):
    for k in keys:
        a = np.asarray(o[k]).astype(np.uint64 if k == "r0" else np.int64)
        b = np.asarray(e[k]).astype(np.uint64 if k == "r0" else np.int64)
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"{k} differs at {len(bad)} packets, first {bad[:6]}: oracle {a[bad[:6]]} engine {b[bad[:6]]}"


def test_cfg3_parse5_bench_size_exact(gpu):
    wl, n, V = _workload("parse5")
    assert n == 1 << 24 and V == 1 << 18
    sc = _scenario(wl, V)
    from mimic_amd import workloads as W

    cpu = W.schedule_cpu(n, V, "interleaved")
    vm, maps, batch, e = _engine_run(sc, wl, n, V)
    assert e["last_exec"] == "spread_own"   # the owned spread form, as the bench runs it (Q = 4)
    del batch
    erows = maps["flows"].ValuesRange(0, V)
    vm.close()
    o, orows = _oracle_percpu_threads(sc, wl.buf, wl.off, wl.lens, cpu, V, _host_threads())
    _same(o, e)
    assert np.array_equal(orows["flows"], erows), "per-CPU map rows differ"
    assert e["steps_total"] == int(o["steps"].astype(np.int64).sum())
    # size-independent property: every packet counted once in its own vCPU's row
    assert int(erows.view(np.uint64).sum()) == n
    assert set(np.unique(e["r0"]).tolist()) <= {1, 2}


def test_cfg4_flowtrack_bench_size_per_key_exact(gpu):
    wl, n, V = _workload("flowtrack")
    assert n == 1 << 21 and V == 1 << 18 and wl.maps[0]["max_entries"] == 131072
    sc = _scenario(wl, V)
    from mimic_amd import workloads as W

    cpu = W.schedule_cpu(n, V, "interleaved")
    vm, maps, batch, e = _engine_run(sc, wl, n, V)
    econt = {k: v[0] for k, v in maps["flows"].Contents().items()}
    vm.close()
    ovm, mids, pids = build_oracle(sc)
    o = ovm.run_xdp_batch(pids[0], wl.buf, wl.off, wl.lens, cpu, write_back=False)
    vals = ovm.map_values(mids["flows"], 0)
    ocont = {k: vals[s * 8:(s + 1) * 8] for k, s in ovm.map_entries(mids["flows"])}
    ovm.close()
    _same(o, e, ("r0", "status", "err_pc"))
    assert len(ocont) == len(econt) and len(ocont) > 100000
    assert ocont == econt, "key -> value contents differ"
    assert int((e["status"] != 0).sum()) == 0
    # steps: which of a key's packets miss the lookup depends on the order concurrent vCPUs reach
    # the map (two lanes may both miss and both update, as two workers of the reference's pool
    # could), so a packet's step count must be one the oracle shows for its key (its miss path or
    # its hit path); packets that never reach the map call agree one by one
    k, idx = W.flow_keys_np(wl.buf, wl.off, wl.lens, with_index=True)
    kid = np.full(n, -1, np.int64)
    kid[idx] = np.unique(np.ascontiguousarray(k).view(np.dtype((np.void, 16))).ravel(), return_inverse=True)[1]
    ost, est = np.asarray(o["steps"], np.int64), np.asarray(e["steps"], np.int64)
    far = kid < 0
    assert (ost[far] == est[far]).all()
    at = ~far
    assert (ost[at] < 1 << 20).all() and (est[at] < 1 << 20).all()
    assert np.isin((kid[at] << 20) | est[at], (kid[at] << 20) | ost[at]).all(), "a step count no oracle packet of the key shows"


def test_cfg5_skb_chain_bench_size_exact(gpu):
    from harness import run_oracle_skb

    wl, n, V = _workload("skb")
    assert n == 1 << 20 and V == 1 << 17
    sc = _scenario(wl, V)
    from mimic_amd import workloads as W

    cpu = W.schedule_cpu(n, V, "interleaved")
    vm, maps, batch, e = _engine_run(sc, wl, n, V, ctx=1)
    assert e["last_exec"] == "jit"
    e_pkt = batch.pkt_data.cpu().numpy()
    emaps = {m["name"]: maps[m["name"]].ValuesRange(0, V if m["type"] in (5, 6) else 1) for m in sc.maps}
    vm.close()
    o = run_oracle_skb(sc, wl.buf, wl.off, wl.lens, cpu, ifindex=1)
    _same(o, e)
    assert np.array_equal(o["pkt"][:len(e_pkt)], e_pkt[:len(o["pkt"])]), "packet memory differs"
    for m in sc.maps:
        rows = emaps[m["name"]]
        for c in range(rows.shape[0]):
            assert bytes(rows[c]) == o["maps"][m["name"]][c], (m["name"], c)
    assert e["steps_total"] == int(o["steps"].astype(np.int64).sum())
    st = np.bincount(e["status"], minlength=64)
    assert st[0] > 0.95 * n
