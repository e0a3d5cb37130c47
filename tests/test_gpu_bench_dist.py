"""bench.py's whole N-rank engine path, run before the driver's 8-GPU node does: `--gpus 2
--dist-backend gloo --one-device` starts two ranks through torch.distributed.run (the launcher the
driver uses), both engines on GPU 0 with CPU (gloo) collectives.  Each rank goes through main() as
it is: vCPU shard, program broadcast, barrier + timed region, max-over-ranks time, per-CPU counter
all-reduce, hash replica merge, one JSON line from rank 0.  Its numbers must be those of ONE
oracle process over both ranks' packets (vm.go:521-539; one shared table for cfg 4,
emulator_linux_map_hash.go:174-181)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from harness import Scenario, kernel_of

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WARMUP, STEPS = 1, 2


def jit_kernels():
    from mimic_amd import workloads as W

    return [kernel_of(Scenario(vcpus=1, maps=p.maps, progs=[(p.name, p.raw, p.relocs)]), 0)
            for p in (W.prog_classifier(), W.prog_flowtrack())]


def _bench2(cfg):
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--one-device", "--config", cfg,
           "--steps", str(STEPS), "--warmup", str(WARMUP), "--batches", "1", "--no-host-resident", "--no-cpu-baseline",
           "--digest"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _sha(b: bytes) -> str:
    import hashlib

    return hashlib.sha256(b).hexdigest()


def test_two_rank_classifier_counters_equal_one_oracle(gpu):
    """cfg 2 at bench size per rank (1M packets, 262 144 vCPUs each): the all-reduced per-CPU
    verdict counters = the verdict counts of one oracle run over both ranks' packets, times the
    launches before the readout; every packet's R0 on each rank = the oracle's (digests gathered to
    rank 0)."""
    import bench
    import oracle
    from mimic_amd import workloads as W

    d = _bench2("classifier")
    assert d["n_gpus"] == 2 and d["collectives"] == "gloo, world size 2" and d["one_device"]
    assert d["status_ok_frac"] == 1.0
    p = W.prog_classifier()
    want = np.zeros(4, np.int64)
    for r in range(2):
        wl = bench.Workload("classifier", 1 << 20, W.SEED + r, r, 2)
        vm = oracle.OracleVM(64)
        mid = vm.map_create("verdicts", 6, 4, 8, 4)
        pid = vm.prog_load(p.name, p.raw, [(s, mid) for s, _ in p.relocs])
        o = vm.run_xdp_batch(pid, wl.buf, wl.off, wl.lens, W.schedule_cpu(len(wl.lens), 64, "interleaved"),
                             write_back=False)
        want += np.bincount(o["r0"].astype(np.int64), minlength=4)[:4]
        assert d["digests"]["r0"][r] == _sha(np.asarray(o["r0"]).astype(np.uint64).tobytes()), r
        vm.close()
    assert d["counters_sum"] == [int(x) * (WARMUP + STEPS) for x in want]
    assert d["mean_insns_per_packet"] > 20


def test_two_rank_flowtrack_replicas_merge_to_one_oracle_table(gpu):
    """cfg 4 at bench size per rank (2M packets of ONE 4M-packet batch, E = 131 072): the merged
    replicas hold exactly the keys and values one oracle table holds after both shards, and every
    packet's R0 on each rank (the last launch: all lookups) is the oracle's for that packet (no flow is
    refused: the union fits E)."""
    import bench
    import oracle
    from mimic_amd import workloads as W

    d = _bench2("flowtrack")
    assert d["n_gpus"] == 2 and d["collectives"] == "gloo, world size 2"
    p = W.prog_flowtrack()
    m = p.maps[0]
    vm = oracle.OracleVM(64)
    mid = vm.map_create(m["name"], m["type"], m["key_size"], m["value_size"], m["max_entries"])
    pid = vm.prog_load(p.name, p.raw, [(s, mid) for s, _ in p.relocs])
    for r in range(2):
        wl = bench.Workload("flowtrack", 1 << 21, W.SEED + r, r, 2)
        o = vm.run_xdp_batch(pid, wl.buf, wl.off, wl.lens, W.schedule_cpu(len(wl.lens), 64, "interleaved"),
                             write_back=False)
        assert d["digests"]["r0"][r] == _sha(np.asarray(o["r0"]).astype(np.uint64).tobytes()), r
    ents = vm.map_entries(mid)
    ov = vm.map_values(mid, 0)
    want = len(ents)
    table = sorted((k, ov[s * 8:(s + 1) * 8]) for k, s in ents)
    vm.close()
    assert 120000 < want <= m["max_entries"]
    assert d["hash_keys"] == want
    assert d["digests"]["hash"] == _sha(b"".join(k + v for k, v in table))
