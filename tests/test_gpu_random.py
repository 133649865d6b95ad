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


def _seeds_with_conditions(k, base=3000):
    # processes with conditions, all of them ordering comparisons (`and` / `or` over a NULL operand and
    # equality with a string are outside the device's FEEL subset: fallbacks, which the oracle refuses)
    out, s = [], 0
    while len(out) < k:
        x = random_process(np.random.default_rng(base + s), sub_processes=s % 2 == 1)
        if "conditionExpression" in x and " and " not in x and " or " not in x:
            out.append(s)
        s += 1
    return out


@pytest.mark.parametrize("seed", _seeds_with_conditions(8))
def test_random_process_incident_parity(seed):
    # random processes whose `amount` is an int, a string, nil or missing: conditions that are not
    # booleans raise incidents (ExpressionProcessor.java:356-368), gateways without a true condition and
    # no default flow raise CONDITION_ERROR; the instances with incidents stay active on the device
    # while their other branches run on (records and state equal to the oracle after every window)
    from helpers import create_commands
    from oracle.oracle import Oracle
    from test_gpu_parity import open_job_completions, run_both
    from zeebe_amd import abi
    from zeebe_amd.engine import Partition
    rng = np.random.default_rng(3000 + seed)
    xml = random_process(rng, sub_processes=seed % 2 == 1)
    n = 96
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=256), Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    ids = [(part.intern(x), orc.intern(x)) for x in ("amount", "other")]
    assert all(a == b for a, b in ids)
    sid = part.intern_string("bar")
    assert sid == orc.intern_string("bar")
    cmds = create_commands(n, 0)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(n)
    docs = amount_docs(rng.integers(0, 1000, n), 0)
    kind = rng.integers(0, 5, n)
    docs["type"] = np.where(kind == 2, abi.DOC_STR, np.where(kind == 3, abi.DOC_NIL, abi.DOC_INT))
    docs["value"] = np.where(kind == 2, sid, np.where(kind == 3, 0, docs["value"]))
    docs["name_id"] = np.where(kind == 4, ids[1][0], 0)  # `other`: amount is missing
    recs = [run_both(part, orc, cmds, docs)]
    assert part.state() == orc.state()
    jrng = np.random.default_rng(seed)
    for _ in range(60):
        c = open_job_completions(part, jrng)
        if c is None:
            break
        recs.append(run_both(part, orc, c))
        assert part.state() == orc.state()
    assert part.stats()["fallback"] == 0
    assert (np.concatenate(recs)["value_type"] == abi.VT_INCIDENT).any()
