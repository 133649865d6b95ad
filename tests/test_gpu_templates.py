"""CREATE batch templates on the gfx950 path (kernels.hip tpl_create / tpl_record): a CREATE batch
that never waits is copied from the rows the general path (BpmnStreamProcessor FIFO over
ProcessProcessor, StartEventProcessor, ExclusiveGatewayProcessor, ParallelGatewayProcessor,
EndEventProcessor) emitted for an earlier CREATE of the same process, variable name and gateway
outcome.  The first launch records; later launches replay.

Bar: every window's records, rejections and state equal to the oracle's, and the later windows
served from templates (zbhip_stats.template_batches)."""
import numpy as np
import pytest

from helpers import amount_docs, create_commands
from oracle.oracle import Oracle
from test_gpu_parity import assert_same_records
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu


def windows(part, orc, batches):
    """Runs each (commands, documents) window on both engines; returns template batches per window."""
    used = []
    for cmds, docs in batches:
        part.submit(cmds, docs)
        part.run()
        got = part.drain()
        orc.clear_records()
        orc.submit(cmds, docs)
        orc.run()
        assert_same_records(got, orc.records(), part, orc)
        assert part.fallback() == []
        assert part.state() == orc.state()
        used.append(part.stats()["template_batches"])
    return used


@pytest.mark.parametrize("branches", [2, 8, 12])
def test_fork_join_pass_through(branches):
    n = 256
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=128), Oracle()
    xml = bpmn.fork_join_process(branches)
    assert part.deploy(xml) == orc.deploy(xml) == 0
    # completed instances free their slots: every window reuses them
    used = windows(part, orc, [(create_commands(n), None) for _ in range(3)])
    assert used[0] < n and used[1] == n and used[2] == n


@pytest.mark.parametrize("decimal", [False, True])
def test_exclusive_gateway_both_outcomes(decimal):
    n = 512
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=128), Oracle()
    xml = bpmn.xor_process()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    name = part.intern("amount")
    assert orc.intern("amount") == name
    rng = np.random.default_rng(0x5EED03)
    batches = []
    for _ in range(4):
        c = create_commands(n)
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
        v = rng.integers(0, 200000, n) / 100.0 if decimal else rng.integers(0, 2000, n)
        batches.append((c, amount_docs(v, name, decimal=decimal)))
    used = windows(part, orc, batches)
    assert used[-1] == n  # both outcomes recorded by then


def test_variable_name_and_document_shape_select_the_template():
    # documents with either variable or none: `other = null` is true without `other` (a variable
    # named amount, or no document) and false with it -- three templates, never mixed up
    n = 96
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=128), Oracle()
    xml = bpmn.xor_process(condition="= other = null")
    assert part.deploy(xml) == orc.deploy(xml) == 0
    names = [part.intern(x) for x in ("amount", "other")]
    assert [orc.intern(x) for x in ("amount", "other")] == names
    rng = np.random.default_rng(5)
    batches = []
    for w in range(4):
        c = create_commands(n)
        docs = abi.make_docs(n)
        docs["name_id"] = [names[(i + w) % 2] for i in range(n)]
        docs["type"] = abi.DOC_INT
        docs["value"] = rng.integers(0, 2000, n)
        c["doc_count"] = [0 if i % 3 == 0 else 1 for i in range(n)]
        c["doc_begin"] = np.arange(n)
        batches.append((c, docs))
    used = windows(part, orc, batches)
    assert used[-1] > 0


def test_mixed_processes_and_tasks():
    # a template process next to one with a wait state (never templated) in the same windows
    n = 128
    part, orc = Partition(max_instances=2 * n, max_commands=2 * n, max_records_per_batch=128), Oracle()
    for e in (part, orc):
        e.deploy(bpmn.fork_join_process(4, process_id="pass"), process_definition_key=2251799813685249)
        e.deploy(bpmn.fork_join_process(3, process_id="tasks", tasks=True), process_definition_key=2251799813685250)
    batches = [(np.concatenate([create_commands(n, 0, 0), create_commands(n, 1, n)]), None)]
    batches += [(create_commands(n, 0, 0), None) for _ in range(2)]
    used = windows(part, orc, batches)
    assert used[1] == n and used[2] == n


def test_batch_limit_disables_the_template():
    # a fork wider than the batch limit writes follow-ups unprocessed: such a batch is never a template
    n = 64
    part = Partition(max_instances=n, max_commands=64 * n, max_records_per_batch=256, max_commands_in_batch=10)
    orc = Oracle(max_commands_in_batch=10)
    xml = bpmn.fork_join_process(12)
    assert part.deploy(xml) == orc.deploy(xml) == 0
    used = windows(part, orc, [(create_commands(n), None) for _ in range(3)])
    assert used == [0, 0, 0]


def test_interleaved_processes_in_every_wave():
    # two template processes (and both outcomes of the gateway) side by side in every wave: each
    # (process, outcome) gets recorded, so the second window is served from templates entirely
    n = 512
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=128), Oracle()
    for e in (part, orc):
        e.deploy(bpmn.fork_join_process(3), process_definition_key=2251799813685249)
        e.deploy(bpmn.xor_process(), process_definition_key=2251799813685250)
    name = part.intern("amount")
    assert orc.intern("amount") == name
    rng = np.random.default_rng(17)
    batches = []
    for _ in range(3):
        c = create_commands(n)
        c["ref"] = np.arange(n) % 2
        c["doc_count"] = np.arange(n) % 2
        c["doc_begin"] = np.arange(n)
        batches.append((c, amount_docs(rng.integers(0, 2000, n), name)))
    used = windows(part, orc, batches)
    assert used[1] == n and used[2] == n


@pytest.mark.parametrize("seed", range(10))
def test_random_straight_through_processes(seed):
    # random processes without wait states (gateways, pass-through elements, nested): three CREATE
    # windows with documents; records and state equal to the oracle's, and every window's device log
    # bytes equal to the host serialiser's
    from random_bpmn import random_process

    rng = np.random.default_rng(4000 + seed)
    xml = random_process(rng, tasks=False)
    n = 128
    # a straight-through batch of these processes can run to a few hundred records
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=1024), Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    name = part.intern("amount")
    assert orc.intern("amount") == name
    ser = part.log_serializer()
    base = 0
    for w in range(3):
        c = create_commands(n)
        c["doc_count"] = 1
        c["doc_begin"] = np.arange(n)
        d = amount_docs(rng.integers(0, 1000, n), name)
        part.submit(c, d)
        part.run()
        pos = 1 + 2 * np.arange(n, dtype=np.int64)
        dev = part.serialize_log_device(pos, 2 * n + 1, 1700000000123)
        got = part.drain()
        assert dev == ser.serialize(got, c, d, base, base, pos, 2 * n + 1, 1700000000123)
        base += n
        orc.clear_records()
        orc.submit(c, d)
        orc.run()
        assert_same_records(got, orc.records(), part, orc)
        assert part.fallback() == []
        assert part.state() == orc.state()
