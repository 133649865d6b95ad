"""Log bytes of the GPU path: records drained from libzbhip.so, serialised by the partition's own
serializer (zbhip_handle_serializer), equal byte for byte to the oracle's serialisation
(oracle/logserial.py) of the CPU engine's records for the same windows; and the zb-db bytes of the
GPU-held state (zbhip_export_state_db) equal to oracle/statedb.py's encoding of the CPU engine's."""
import numpy as np
import pytest

from helpers import amount_docs, complete_commands, create_commands, process_xml
from oracle import logserial as LS
from oracle import statedb as SD
from oracle.oracle import Oracle
from test_logserial import check_entries, with_reason_codes
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

TS = 1700000000123


class Pair:
    def __init__(self, xml, n, names=()):
        self.part = Partition(max_instances=n, max_commands=10 * n, max_records_per_batch=64)
        self.orc = Oracle()
        assert self.part.deploy(xml) == self.orc.deploy(xml) == 0
        for nm in names:
            assert self.part.intern(nm) == self.orc.intern(nm)
        self.ser = self.part.log_serializer()
        self.source_base = self.doc_base = 0
        self.position = 1

    def window(self, cmds, docs=None):
        docs = docs if docs is not None else abi.make_docs(0)
        self.part.submit(cmds, docs)
        self.part.run()
        got_recs = self.part.drain()
        self.orc.clear_records()
        self.orc.submit(cmds, docs)
        self.orc.run()
        want_recs = self.orc.records()
        pos = self.position + 3 * np.arange(len(cmds), dtype=np.int64)
        first = int(pos[-1]) + 1
        got = self.ser.serialize(got_recs, cmds, docs, self.source_base, self.doc_base, pos, first, TS)
        names = self.orc.names()
        tables = LS.Tables(self.orc.process_tables(), lambda i: names[i], self.orc.string_value)
        sb, db = self.source_base, self.doc_base

        def docs_of_source(si):
            c = cmds[si - sb]
            return docs[int(c["doc_begin"]):int(c["doc_begin"]) + int(c["doc_count"])]

        want = LS.serialize(want_recs, tables, docs_of_source, lambda a: docs[a - db], self.orc.reason, first,
                            lambda si: int(pos[si - sb]), TS)
        assert got == want
        check_entries(got, got_recs, first, pos, sb)
        # the drained reason codes are the ones the CPU engine's texts classify to
        codes = with_reason_codes(want_recs, self.orc)
        assert np.array_equal(codes["reason"], got_recs["reason"])
        assert np.array_equal(codes["reason_arg"], got_recs["reason_arg"])
        # zb-db bytes of the state the GPU holds == the oracle's encoding of the CPU engine's state
        strings = self.orc.strings()
        assert self.part.state_db() == SD.encode_rows(self.orc.state(), self.orc.process_tables(),
                                                      lambda i: strings[i])
        self.source_base += len(cmds)
        self.doc_base += len(docs)
        self.position = first + len(got_recs)
        return got_recs


def drive(pair, n, docs=None):
    cmds = create_commands(n, 0)
    if docs is not None:
        cmds["doc_count"] = 1
        cmds["doc_begin"] = np.arange(n)
    recs = pair.window(cmds, docs)
    for _ in range(15):
        jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
        if not jobs:
            break
        res = [pair.part.resolve_key(k) for k in jobs]
        recs = pair.window(complete_commands([r[0] for r in res], [r[1] for r in res]))


@pytest.mark.parametrize("workload", ["one_task", "linear10", "fork_join8", "fork_join8_tasks", "pass_through"])
def test_gpu_log_bytes_match_oracle(workload):
    from test_logserial import PASS_THROUGH_XML
    xml = {"one_task": process_xml({"fixture": "one_task.bpmn"}), "linear10": bpmn.linear_process(10),
           "fork_join8": bpmn.fork_join_process(8), "fork_join8_tasks": bpmn.fork_join_process(8, tasks=True),
           "pass_through": PASS_THROUGH_XML}[workload]
    drive(Pair(xml, 200), 200)


def test_gpu_log_bytes_xor_documents():
    rng = np.random.default_rng(0x5EED03)
    pair = Pair(bpmn.xor_process(), 300, names=["amount"])
    drive(pair, 150, amount_docs(rng.integers(0, 2001, 150), 0))
    cmds = create_commands(150, 0, 150)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(150)
    pair.window(cmds, amount_docs(rng.integers(0, 200001, 150) * 10000, 0, decimal=True))


def test_gpu_log_bytes_of_activated_jobs():
    # JOB:COMPLETED of an ACTIVATED job is the stored job (JobCompleteProcessor.acceptCommand:
    # jobState.getJob, DbJobState.activate stored the deadline and worker): the drained record carries
    # them (message_key / correlation_key), both serialisers write them, and the device writer leaves
    # such a window to the host serialiser (the worker is a value-dictionary string)
    from zeebe_amd.native import ZbhipError
    n = 40
    pair = Pair(bpmn.linear_process(2, job_type="t"), n)
    recs = pair.window(create_commands(n, 0))
    g = pair.part.activate_jobs("t", worker="worker-A", timeout=60000, max_jobs=15, timestamp=500)
    o = pair.orc.activate_jobs("t", worker="worker-A", timeout=60000, max_jobs=15, timestamp=500)
    assert [int(k) for k in g[1]["key"]] == [int(k) for k in o[1]["key"]]
    pair.part.activate_jobs("t", worker="", timeout=1000, max_jobs=5, timestamp=600)
    pair.orc.activate_jobs("t", worker="", timeout=1000, max_jobs=5, timestamp=600)
    jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    res = [pair.part.resolve_key(k) for k in jobs]
    got = pair.window(complete_commands([r[0] for r in res], [r[1] for r in res]))
    done = got[(got["value_type"] == abi.VT_JOB) & (got["intent"] == abi.JOB_COMPLETED)]
    act = done[done["message_key"] != -1]
    assert len(act) == 20 and set(act["message_key"].tolist()) == {60500, 1600}
