"""zb-db state back into HBM: a partition's state exported as zb-db entries
(zbhip_export_state_db) and imported into a fresh handle (zbhip_import_state_db) continues exactly
as the partition that never stopped -- the device form of the reference's replay-equivalence
property (engine/src/test/.../processing/randomized/ReplayStateRandomizedPropertyTest.java:74-140:
the state after processing equals the state after a restart), checked against the CPU oracle too.

Bar: after the import the canonical state and the zb-db bytes equal the exporter's; afterwards every
window's records (all parity fields but source_index and aux, whose bases are the handle's own
window counters) and the state equal both the uninterrupted partition's and the oracle's."""
import numpy as np
import pytest

from helpers import amount_docs, create_commands
from oracle.oracle import Oracle
from random_bpmn import random_process
from test_gpu_parity import open_job_completions
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

FIELDS = [f for f in abi.PARITY_FIELDS if f not in ("source_index", "aux")]


def _same(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in FIELDS:
        if not np.array_equal(a[f], b[f]):
            bad = np.nonzero(a[f] != b[f])[0][:5]
            raise AssertionError("field %s at %s: %s vs %s" % (f, bad, a[f][bad], b[f][bad]))
    assert np.array_equal(a["aux"] < 0, b["aux"] < 0)


def _restart(part, xml, n, names, max_records):
    """A fresh handle with the same deployment and dictionaries, loaded from part's zb-db bytes."""
    fresh = Partition(max_instances=n, max_commands=max(n, 8), max_records_per_batch=max_records)
    assert fresh.deploy(xml) == 0
    for name in names:
        fresh.intern(name)
    entries = part.state_db()
    loaded = fresh.import_state_db(entries)
    assert fresh.state() == part.state()
    assert fresh.state_db() == entries
    return fresh, loaded


def _completions(part, keys):
    """JOB:COMPLETE commands for the given job keys through the handle's own key table: key
    ordinals are per handle (an imported instance's keys are numbered anew), the keys are not."""
    c = abi.make_commands(len(keys))
    for i, k in enumerate(keys):
        c[i]["instance"], c[i]["ref"] = part.resolve_key(k)
    c["kind"] = abi.CMD_JOB_COMPLETE
    return c


def _continue(parts, orc, rng, phases):
    """Drives every handle and the oracle with the same job completions until nothing is open."""
    for _ in range(phases):
        c0 = open_job_completions(parts[0], rng)
        if c0 is None:
            return
        keys = []
        for r in parts[0].state():
            if r.startswith("JOBS|"):
                k = int(r.split("|")[1])
                inst, ordv = parts[0].resolve_key(k)
                if any(int(x["instance"]) == inst and int(x["ref"]) == ordv for x in c0):
                    keys.append((inst, k))
        keys = [k for _, k in sorted(keys)]
        outs = []
        for p in parts:
            p.submit(_completions(p, keys))
            p.run()
            outs.append(p.drain())
            assert p.fallback() == []
        orc.clear_records()
        orc.submit(c0)
        orc.run()
        want = orc.records()
        for got in outs:
            _same(got, want)
        for p in parts:
            assert p.state() == orc.state()


@pytest.mark.parametrize("case", ["linear", "fork_join_tasks", "xor_then_tasks", "sub_parallel", "sub_chain"])
def test_export_import_continue(case):
    n = 64
    rng = np.random.default_rng(7)
    names = []
    docs = None
    if case == "linear":
        xml = bpmn.linear_process(5)
    elif case == "fork_join_tasks":
        xml = bpmn.fork_join_process(4, tasks=True)
    elif case == "sub_parallel":  # a sub-process instance with its join counter rows in the state
        xml = bpmn.sub_process_process("parallel")
    elif case == "sub_chain":  # nested sub-process instances (flow scopes two levels down)
        from test_gpu_subprocess import _sub_then_task_then_sub
        xml = _sub_then_task_then_sub()
    else:  # variables in the state (amount), a gateway behind a task
        xml = (bpmn.createExecutableProcess("p").startEvent("s").serviceTask("t1", "a").exclusiveGateway("x")
               .sequenceFlowId("hi").conditionExpression("= amount > 500").serviceTask("t2", "b").endEvent("e1")
               .moveToNode("x").sequenceFlowId("lo").defaultFlow().serviceTask("t3", "c").endEvent("e2").done())
        names = ["amount"]
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=128)
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    for name in names:
        assert part.intern(name) == orc.intern(name)
    cmds = create_commands(n)
    if names:
        docs = amount_docs(rng.integers(0, 1000, n), 0)
        cmds["doc_count"] = 1
        cmds["doc_begin"] = np.arange(n)
    part.submit(cmds, docs)
    part.run()
    _same(part.drain(), (orc.submit(cmds, docs), orc.run(), orc.records())[2])
    # a few completions, one job per instance per window (joins left waiting, tasks open)
    for _ in range(1 if case in ("xor_then_tasks", "sub_parallel") else 2):
        c = open_job_completions(part, rng)
        if c is None:
            break
        part.submit(c)
        part.run()
        part.drain()
        orc.clear_records()
        orc.submit(c)
        orc.run()
    assert part.state() == orc.state()
    fresh, loaded = _restart(part, xml, n, names, 128)
    assert loaded == sum(1 for r in part.state() if r.startswith("ELEMENT_INSTANCE_KEY|") and "bpmnElementType=1," in r)
    assert loaded > 0
    # the imported job keys resolve to the same instance slots
    for r in part.state():
        if r.startswith("JOBS|"):
            k = int(r.split("|")[1])
            assert fresh.resolve_key(k)[0] == part.resolve_key(k)[0]
    _continue([part, fresh], orc, rng, 40)
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == []


@pytest.mark.parametrize("seed,subs", [(s, False) for s in range(8)] + [(s, True) for s in (1, 3, 4, 7, 19, 22)])
def test_random_processes_restart_equivalence(seed, subs):
    # ReplayStateRandomizedPropertyTest in the device's terms: random processes, a restart (export
    # -> import into a fresh handle) at a random phase, and the state after every later window
    # equal to the uninterrupted partition's and the oracle's (subs: with embedded sub-processes)
    rng = np.random.default_rng(3000 + seed)
    xml = random_process(rng, sub_processes=subs)
    n = 48
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=256)
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    assert part.intern("amount") == orc.intern("amount")
    cmds = create_commands(n)
    docs = amount_docs(rng.integers(0, 1000, n), 0)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(n)
    part.submit(cmds, docs)
    part.run()
    part.drain()
    orc.submit(cmds, docs)
    orc.run()
    orc.clear_records()
    walk = np.random.default_rng(seed)
    for _ in range(int(rng.integers(0, 4))):
        c = open_job_completions(part, walk)
        if c is None:
            break
        for e in (part, orc):
            e.submit(c)
            e.run()
        part.drain()
        orc.clear_records()
    assert part.state() == orc.state()
    fresh, _ = _restart(part, xml, n, ["amount"], 256)
    _continue([part, fresh], orc, walk, 60)
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == []
