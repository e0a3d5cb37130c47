"""The multi-GPU path with the engine on one GPU: bench.py --rccl runs the setup / readout
collectives over RCCL (nccl backend) at world size 1 -- program bytes broadcast, per-CPU counter
all-reduce, hash replica merge, max-over-ranks time -- and must report exactly what the run
without collectives reports.  Each run is its own process (an RCCL communicator per run)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(cfg, rccl):
    cmd = [sys.executable, "bench.py", "--config", cfg, "--packets", "65536", "--vcpus", "4096", "--steps", "2",
           "--warmup", "1", "--batches", "1", "--no-host-resident", "--no-cpu-baseline"] + (["--rccl"] if rccl else [])
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("cfg", ["classifier", "flowtrack"])
def test_rccl_path_equals_single_rank(gpu, cfg):
    a, b = _bench(cfg, False), _bench(cfg, True)
    assert b.get("collectives") == "rccl, world size 1" and "collectives" not in a
    assert b["n_gpus"] == 1 and b["status_ok_frac"] == a["status_ok_frac"]
    assert b["counters_sum"] == a["counters_sum"] and b["hash_keys"] == a["hash_keys"]
    assert b["mean_insns_per_packet"] == a["mean_insns_per_packet"]
    if cfg == "classifier":
        assert sum(b["counters_sum"]) > 0
    else:
        assert b["hash_keys"] > 1000
