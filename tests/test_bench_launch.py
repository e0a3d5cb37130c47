"""bench.py --gpus N: the launcher starts N ranks (one process per GPU) when WORLD_SIZE is unset,
refuses a WORLD_SIZE that disagrees with --gpus, and refuses more ranks than visible GPUs.  The
ranks' setup / readout collectives are rehearsed on gloo (--launch-selftest, no engine)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout,
                          cwd=ROOT)


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_flag_launches_that_many_ranks():
    for n in (2, 3):
        p = _run(["--gpus", str(n), "--launch-selftest"], _env())
        assert p.returncode == 0, p.stderr[-2000:]
        d = _json_line(p.stdout)
        assert d["n_gpus"] == n and d["gpus_flag"] == n
        assert d["ranks"] == list(range(n)) and d["local_ranks"] == list(range(n))
        assert d["program_ok"] and d["hash_keys"] == n
        assert d["elapsed_max"] == 0.001 * n
        assert d["counters"] == [n * (n + 1) // 2, n]


def test_flowtrack_selftest_merges_bench_size_replicas():
    """--gpus N --config flowtrack --launch-selftest: every gloo rank builds its bench-size cfg-4
    shard (2M IMIX packets of the one batch) and the (key, value) records its replica would
    hold; the merge with the MaxEntries check (E = 131 072) completes at N = 2 and N = 8."""
    for n, lo in ((2, 128000), (8, 131072)):
        p = _run(["--gpus", str(n), "--config", "flowtrack", "--launch-selftest"], _env(OMP_NUM_THREADS="2"), timeout=600)
        assert p.returncode == 0, p.stderr[-2000:]
        d = _json_line(p.stdout)
        assert d["n_gpus"] == n and lo <= d["hash_keys"] <= 131072, d


def test_world_size_must_match_gpus_flag():
    p = _run(["--gpus", "2"], _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2
    assert "WORLD_SIZE=1" in p.stderr
    p = _run(["--gpus", "1"], _env(WORLD_SIZE="4", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2


def test_more_ranks_than_gpus_is_refused():
    import torch

    have = torch.cuda.device_count()
    p = _run(["--gpus", str(have + 1)], _env())
    assert p.returncode == 2, (p.stdout[-500:], p.stderr[-500:])
    assert f"only {have} GPU(s) visible" in p.stderr
    assert "{" not in p.stdout   # no bench line with a wrong n_gpus
