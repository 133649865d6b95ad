"""The ProcessingStateMachine restatement (tests/psm.py) with the oracle as its one-command engine
equals the oracle's own batch driver (zb_oracle.cpp batch_processing, pinned on the reference's
batch-limit case by test_oracle_golden.py::test_batch_limit_overflow_goes_to_log): the same batches
in the same order, the same records (processed flags of follow-up commands included), the same
state -- for limits 3, 5 and 100, fan-outs past the limit, job completions with documents.  This pins
the harness the adapter test (tests/test_gpu_psm.py) runs the device behind.  Also: the oracle's
one-command entry point and its hand-off import (zb-db text rows)."""
import numpy as np
import pytest

from psm import Client, Log, OracleEngine, StreamProcessor, open_jobs
from test_gpu_batch_limit import fork_to_ends
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import RecordValues
from zeebe_amd.engine import ProcessDefinition  # noqa: F401  (psm builds them)

KEY = 2251799813685249


def _native_batches(o, recs, doc_values):
    from psm import oracle_tables
    vals = RecordValues(oracle_tables(o), o.name, lambda i: o.string_value(i).decode())
    batches = []
    last = None
    for k, r in enumerate(recs):
        s = int(r["source_index"])
        if s != last:
            batches.append([])
            last = s
        rt = int(r["record_type"])
        v = None if rt == abi.RT_REJECTION else vals.value(r, (), lambda aux: doc_values[aux])
        ev = v.get("elementId") if isinstance(v, dict) else None
        batches[-1].append((rt, int(r["value_type"]), int(r["intent"]), int(r["key"]),
                            o.reason(k) if rt == abi.RT_REJECTION else "", ev,
                            bool(rt == abi.RT_COMMAND and not r["unprocessed"])))
    return batches


def _psm_batches(log, start):
    batches = []
    last = None
    for r in log.entries[start:]:
        if r.source_position < 0:
            continue  # the client's commands
        if r.source_position != last:
            batches.append([])
            last = r.source_position
        ev = r.value.get("elementId") if isinstance(r.value, dict) and r.record_type != abi.RT_REJECTION else None
        batches[-1].append((r.record_type, r.value_type, r.intent, r.key, r.rejection_reason, ev,
                            bool(r.record_type == abi.RT_COMMAND and r.processed)))
    return batches


def drive(xml, limit, n=6, phases=12, with_docs=False, seed=1):
    native = OracleEngine(max_commands_in_batch=limit).o
    eng = OracleEngine(max_commands_in_batch=limit)
    native.deploy(xml, KEY, 1)
    eng.deploy(xml, KEY, 1)
    log = Log()
    sp = StreamProcessor(log, [eng], limit)
    client = Client(log)
    pid = eng.tables[0].bpmn_process_id
    rng = np.random.default_rng(seed)
    doc_values = []
    # phase 0: CREATEs
    client.write(*[client.create(pid) for _ in range(n)])
    start = len(log.entries)
    sp.run()
    native.submit(__import__("helpers").create_commands(n))
    native.run()
    assert _psm_batches(log, start) == _native_batches(native, native.records(), doc_values)
    assert eng.state() == native.state()
    slot_of = {}
    for r in native.records():
        if r["value_type"] == abi.VT_PROCESS_INSTANCE_CREATION:
            slot_of[int(r["scope_key"])] = len(slot_of)
    for _ in range(phases):
        jobs = sorted(open_jobs(log).values(), key=lambda r: r.key)
        if not jobs:
            break
        rng.shuffle(jobs)
        cmds = abi.make_commands(len(jobs))
        docs = []
        recs = []
        for i, j in enumerate(jobs):
            inst = slot_of[j.value["processInstanceKey"]]
            cmds[i]["instance"], cmds[i]["kind"] = inst, abi.CMD_JOB_COMPLETE
            cmds[i]["ref"] = native.ordinal_of(inst, j.key)
            variables = ()
            if with_docs and i % 2 == 0:
                variables = (("v%d" % (i % 3), int(rng.integers(0, 100))),)
                cmds[i]["doc_count"], cmds[i]["doc_begin"] = 1, len(docs)
                docs.append((native.intern(variables[0][0]), variables[0][1]))
            recs.append(client.complete_job(j.key, variables))
        client.write(*recs)
        start = len(log.entries)
        sp.run()
        d = abi.make_docs(len(docs))
        for k, (nid, val) in enumerate(docs):
            d[k]["name_id"], d[k]["type"], d[k]["value"] = nid, abi.DOC_INT, val
        doc_values.extend(val for _, val in docs)
        native.clear_records()
        native.submit(cmds, d)
        native.run()
        assert _psm_batches(log, start) == _native_batches(native, native.records(), doc_values)
        assert eng.state() == native.state()
    return log


@pytest.mark.parametrize("limit", [3, 5, 100])
def test_psm_linear(limit):
    drive(bpmn.linear_process(4), limit, with_docs=True)


@pytest.mark.parametrize("limit", [3, 10, 100])
def test_psm_fork_join_tasks(limit):
    drive(bpmn.fork_join_process(6, tasks=True), limit)


@pytest.mark.parametrize("limit", [3, 100])
def test_psm_fan_out(limit):
    log = drive(fork_to_ends(12), limit, phases=0)
    # the follow-ups past the limit were written unprocessed and read back as batches of their own
    unprocessed = [r for r in log.entries if r.record_type == abi.RT_COMMAND and r.source_position > 0
                   and not r.processed]
    assert bool(unprocessed) == (limit == 3)


def test_psm_unwritten_followups_see_the_builder():
    # the platform counts the builder's entries after every step (lastProcessingResultSize): a
    # processor answering a follow-up with the same builder adds nothing, with a fresh one the
    # batch's commands would be collected twice
    log = drive(bpmn.linear_process(1), 100, n=1, phases=1)
    cmds = [r for r in log.entries if r.record_type == abi.RT_COMMAND and r.source_position > 0]
    assert len(cmds) == len({(r.source_position, r.key, r.intent, r.value["elementId"]) for r in cmds})


def test_oracle_import_rows_round_trip():
    # a hand-off: the rows of a waiting instance (the dump format) into a fresh engine, then its job
    # completed there -- the same records and state as on the engine that ran it all along
    xml = bpmn.fork_join_process(3, tasks=True)
    a, b = OracleEngine(), OracleEngine()
    for e in (a, b):
        e.deploy(xml, KEY, 1)
    log = Log()
    client = Client(log)
    client.write(client.create("forkjoin", (("x", 5),)))
    StreamProcessor(log, [a]).run()
    b.upsert([r for r in a.state() if not r.startswith("KEY|")])
    b.set_key_if_higher(a.current_key())
    assert b.state() == a.state()
    job = sorted(open_jobs(log))[1]
    out_a, out_b = Log(), Log()
    for eng, out in ((a, out_a), (b, out_b)):
        Client(out).write(Client.complete_job(job))
        StreamProcessor(out, [eng]).run()
    assert out_a.canonical() == out_b.canonical()
    assert a.state() == b.state()


@pytest.mark.parametrize("seq", [False, True])
@pytest.mark.parametrize("limit", [3, 100])
def test_psm_multi_instance(seq, limit):
    # PROCESS_INSTANCE_BATCH:ACTIVATE and the inner activations through the PSM restatement, past the
    # limit too; loop-variable records carry their values inline
    drive(bpmn.multi_instance_process((10, "b", 30), sequential=seq, after="after"), limit, with_docs=True)
