"""The process-memory lifetime rules (mimic_amd/csrc/blkcache.h) on the CPU: tests/blkcache_test.cpp
built with g++ (ThreadSanitizer when the toolchain has it) and run.  The engine's NewProcess / Run /
Cleanup (engine.cpp proc_alloc, proc_fence, proc_release_blk) use exactly this code with HIP events
as fences; the test drives it with a fake in-order stream from 8 creating threads and a Handoff
thread (vm.go:548-573), and checks that a block is never handed out while an earlier owner's work
on it is pending or while another process holds it."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "blkcache_test.cpp")


def _build(tmp_path, sanitize):
    exe = str(tmp_path / ("blkcache_tsan" if sanitize else "blkcache"))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", SRC, "-o", exe]
    if sanitize:
        cmd[1:1] = ["-fsanitize=thread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return exe if r.returncode == 0 else None, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("sanitize", [False, True], ids=["plain", "tsan"])
def test_block_cache_lifetime_rules(tmp_path, sanitize):
    exe, err = _build(tmp_path, sanitize)
    if exe is None:
        if sanitize:
            pytest.skip(f"no ThreadSanitizer in this toolchain: {err[-200:]}")
        raise AssertionError(err)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
