"""GPU parity: the HIP engine vs the CPU oracle on the same inputs (bit-exact)."""
import numpy as np
import pytest

from harness import Scenario, assert_same, packets_to_buffer, run_engine, run_oracle, single
from mimic_amd import asm as A
from mimic_amd import workloads as W

pytestmark = pytest.mark.gpu


def _prog_scenario(p: W.Program, vcpus: int) -> Scenario:
    return Scenario(vcpus=vcpus, maps=p.maps, progs=[(p.name, p.raw, p.relocs)])


def test_pass8(gpu):
    p = W.prog_pass8()
    sc = _prog_scenario(p, 2)
    buf, off, lens, cpu = single(sc)
    e = run_engine(sc, buf, off, lens, cpu)
    assert int(e["r0"][0]) == 2 and int(e["status"][0]) == 0 and int(e["steps"][0]) == 8
    assert_same(run_oracle(sc, buf, off, lens, cpu), e)


@pytest.mark.parametrize("mode", ["chunked", "interleaved"])
def test_classifier_small(gpu, mode):
    p = W.prog_classifier()
    sc = _prog_scenario(p, 64)
    buf, off, lens = W.make_packets(4096)
    cpu = W.schedule_cpu(4096, 64, mode)
    o = run_oracle(sc, buf, off, lens, cpu)
    e = run_engine(sc, buf, off, lens, cpu)
    assert_same(o, e)
    assert set(np.unique(o["r0"])) <= {1, 2}


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_programs(gpu, seed):
    rng = np.random.default_rng(1000 + seed)
    raw, rel = __import__("fuzz").random_program(rng, n_body=int(rng.integers(10, 80)), map_name="m")
    sc = Scenario(vcpus=8, maps=[dict(name="m", type=6, key_size=4, value_size=8, max_entries=4)],
                  progs=[("fz", raw, rel)])
    pk = [bytes(rng.integers(0, 256, int(rng.choice([0, 14, 60, 64, 100])), dtype=np.uint8)) for _ in range(64)]
    buf, off, lens = packets_to_buffer(pk)
    cpu = rng.integers(0, 8, 64).astype(np.int32)
    o = run_oracle(sc, buf, off, lens, cpu, step_budget=5000)
    e = run_engine(sc, buf, off, lens, cpu, step_budget=5000)
    assert_same(o, e)
