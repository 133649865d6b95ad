"""Randomized parity: random structured processes (tasks, exclusive split/merge with FEEL
conditions on `amount`, parallel fork/join, nested; tests/random_bpmn.py) driven through the gfx950
executor and the CPU oracle with the same seeded inputs -- records and state compared bit-exact
after the CREATE window and after every JOB:COMPLETE window (jobs completed in random order)."""
import numpy as np
import pytest

from helpers import amount_docs
from random_bpmn import random_process
from test_gpu_parity import drive

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(24))
def test_random_process_parity(seed):
    rng = np.random.default_rng(1000 + seed)
    xml = random_process(rng)
    part, orc = drive(xml, 96, lambda n: amount_docs(rng.integers(0, 1000, n), 0), phases=60,
                      rng_seed=seed, max_records=256)
    assert part.state() == orc.state()
    # every instance ran to completion: only the key counter row is left
    assert [r for r in part.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("seed", range(12))
def test_random_process_with_pass_through_elements_parity(seed):
    # undefined / manual tasks and none throw events among the random blocks
    rng = np.random.default_rng(2000 + seed)
    xml = random_process(rng, pass_through=True)
    part, orc = drive(xml, 96, lambda n: amount_docs(rng.integers(0, 1000, n), 0), phases=60,
                      rng_seed=seed, max_records=256)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
