"""zb-db byte encoding of the state: the product encoder
(zbhip_serializer_encode_state_row, host code, runs here without a GPU) against the oracle
restatement (oracle/statedb.py) on the CPU engine's state after every window of configs 1-4,
plus checks of the layout with an independent msgpack decoder."""
import struct

import msgpack
import numpy as np

from helpers import amount_docs, process_xml
from oracle import statedb as SD
from test_logserial import Run, _drive_simple
from zeebe_amd import bpmn


def _check_state(run):
    rows = run.orc.state()
    got = run.ser.encode_state_rows(rows)
    strings = run.orc.strings()
    want = SD.encode_rows(rows, run.orc.process_tables(), lambda i: strings[i])
    assert got == want
    encoded = {cf for cf, _, _ in got}
    assert len(got) == sum(1 for r in rows if r.split("|")[0] in SD.CF)
    for cf, k, v in got:
        assert struct.unpack(">q", k[:8])[0] == cf
        if cf == SD.CF["ELEMENT_INSTANCE_KEY"]:
            ei = msgpack.unpackb(v, raw=False)
            rec = ei["elementRecord"]
            assert rec["key"] == struct.unpack(">q", k[8:16])[0]
            assert rec["state"].startswith("ELEMENT_")
            assert rec["processInstanceRecord"]["tenantId"] == "<default>"
        elif v != b"\xff" and cf not in (SD.CF["ELEMENT_INSTANCE_CHILD_PARENT"], SD.CF["NUMBER_OF_TAKEN_SEQUENCE_FLOWS"]):
            msgpack.unpackb(v, raw=False)
    return encoded


class StateRun(Run):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.cfs = set()

    def window(self, cmds, docs=None):
        recs = super().window(cmds, docs)
        self.cfs |= _check_state(self)
        return recs


def test_state_bytes_linear_and_one_task():
    run = StateRun([bpmn.linear_process(3), process_xml({"fixture": "one_task.bpmn"})])
    _drive_simple(run, 30)
    assert {SD.CF[c] for c in ("KEY", "ELEMENT_INSTANCE_KEY", "JOBS", "JOB_STATES", "JOB_ACTIVATABLE",
                                "EVENT_SCOPE", "ELEMENT_INSTANCE_PARENT_CHILD")} <= run.cfs


def test_state_bytes_variables():
    rng = np.random.default_rng(3)
    run = StateRun([bpmn.linear_process(2)], names=["amount"])
    _drive_simple(run, 20, amount_docs(rng.integers(-100000, 100000, 20), 0))
    assert SD.CF["VARIABLES"] in run.cfs


def test_state_bytes_fork_join_counters():
    run = StateRun([bpmn.fork_join_process(4, tasks=True)])

    def one_branch_per_window(c):  # leave the join waiting between windows
        _, first = np.unique(c["instance"], return_index=True)
        return c[np.sort(first)], None

    _drive_simple(run, 20, mutate=one_branch_per_window)
    assert SD.CF["NUMBER_OF_TAKEN_SEQUENCE_FLOWS"] in run.cfs


def test_key_encodings_golden():
    import json
    import os
    from helpers import GOLDEN
    d = json.load(open(os.path.join(GOLDEN, "zbdb_keys.json")))
    for name, op, arg, want in d["vectors"]:
        if op == "dbstr":
            got = SD.dbstr(arg)
        elif op == "dblong":
            got = SD.dblong(arg)
        elif op == "tenant_prefix":
            got = SD.dbstr(arg[0]) + SD.dbstr(arg[1])
        else:
            got = SD.dbstr(arg[1]) + SD.dbstr(arg[0])
        assert got.hex() == want, name


# ---- the importer's front end: zb-db bytes back to canonical rows (zbhip_import_state_db) -------
class DecodeRun(Run):
    """After every window: the oracle's state rows -> product encoder -> product decoder gives the
    rows back exactly (string variable values through the value dictionary)."""

    def window(self, cmds, docs=None):
        recs = super().window(cmds, docs)
        rows = [r for r in self.orc.state() if r.split("|")[0] in SD.CF]
        entries = self.ser.encode_state_rows(rows)
        strings = [s.encode() if isinstance(s, str) else s for s in self.orc.strings()]
        back = self.ser.decode_state_entries(entries, intern=lambda b: strings.index(b))
        assert back == sorted(rows)
        self.rows_seen = getattr(self, "rows_seen", 0) + len(rows)
        return recs


def test_decode_inverts_encode_linear_and_variables():
    rng = np.random.default_rng(5)
    run = DecodeRun([bpmn.linear_process(3), process_xml({"fixture": "one_task.bpmn"})], names=["amount"])
    _drive_simple(run, 20, amount_docs(rng.integers(-100000, 100000, 20), 0))
    assert run.rows_seen > 0


def test_decode_inverts_encode_fork_join():
    run = DecodeRun([bpmn.fork_join_process(4, tasks=True)])

    def one_branch_per_window(c):
        _, first = np.unique(c["instance"], return_index=True)
        return c[np.sort(first)], None

    _drive_simple(run, 12, mutate=one_branch_per_window)
    assert run.rows_seen > 0


def test_decode_refuses_malformed_entries():
    import pytest
    from zeebe_amd.logwriter import LogSerializer
    from zeebe_amd.native import ZbhipError
    ser = LogSerializer()
    with pytest.raises(ZbhipError):
        ser.decode_state_entries([(7, struct.pack(">q", 7) + b"\x00" * 3, b"\x80")])  # short DbLong key
    with pytest.raises(ZbhipError):
        ser.decode_state_entries([(7, struct.pack(">q", 9) + b"\x00" * 8, b"\x80")])  # prefix != column family
    assert ser.decode_state_entries([(99, struct.pack(">q", 99), b"")]) == []  # not a column family of the path
