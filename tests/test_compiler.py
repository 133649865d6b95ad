"""Host compiler (BPMN XML -> CSR) against the reference's transformation rules and the oracle."""
import ctypes as C

import numpy as np
import pytest

from helpers import process_xml
from oracle.oracle import Oracle
from zeebe_amd import bpmn
from zeebe_amd.engine import ELEMENT_DTYPE, _Csr
from zeebe_amd.native import ZbhipError, check, load


class Compiled:
    def __init__(self, xml):
        self.L = load()
        if isinstance(xml, str):
            xml = xml.encode()
        self.csr = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = self.L.zbhip_compile_bpmn(xml, len(xml), 1, 1, C.byref(self.csr), err, 512)
        check(rc, err.value.decode())
        c = C.cast(self.csr, C.POINTER(_Csr)).contents
        self.els = np.frombuffer(C.string_at(c.elements, c.n_elements * ELEMENT_DTYPE.itemsize), dtype=ELEMENT_DTYPE)
        self.out = np.frombuffer(C.string_at(c.out_flow, max(c.n_out, 1) * 2), dtype="<u2")[: c.n_out]
        self.strings = [c.strings[i].decode() for i in range(c.n_strings)]

    def id(self, e):
        return self.strings[self.els[e]["id"]]

    def outgoing(self, eid):
        e = [self.id(i) for i in range(len(self.els))].index(eid)
        b, n = self.els[e]["out_begin"], self.els[e]["out_count"]
        return [self.id(f) for f in self.out[b:b + n]]

    def __del__(self):
        self.L.zbhip_free_csr(self.csr)


def test_element_indexing_matches_oracle():
    for xml in [process_xml({"fixture": "one_task.bpmn"}), bpmn.linear_process(10), bpmn.xor_process(),
                bpmn.fork_join_process(8), bpmn.fork_join_process(8, tasks=True)]:
        c = Compiled(xml)
        o = Oracle()
        p = o.deploy(xml)
        assert [c.id(i) for i in range(len(c.els))] == [o.element_id(p, i) for i in range(len(c.els))]


def test_outgoing_order_is_reverse_document_order():
    # ModelWalker.java:75-79 -> getOutgoing() of the fork lists f8 .. f1
    c = Compiled(bpmn.fork_join_process(8))
    assert c.outgoing("fork") == ["f%d" % i for i in range(8, 0, -1)]
    assert c.els[[c.id(i) for i in range(len(c.els))].index("join")]["in_count"] == 8


def test_join_slots_are_contiguous_per_gateway():
    c = Compiled(bpmn.fork_join_process(8))
    ids = [c.id(i) for i in range(len(c.els))]
    base = c.els[ids.index("join")]["join_slot"]
    slots = sorted(int(c.els[ids.index("f%d" % i)]["join_slot"]) for i in range(1, 9))
    assert slots == list(range(base, base + 8))


def test_condition_and_default_flow():
    c = Compiled(bpmn.xor_process())
    ids = [c.id(i) for i in range(len(c.els))]
    xor = c.els[ids.index("xor")]
    assert ids[xor["default_flow"]] == "low"
    assert c.els[ids.index("high")]["condition"] != 0xFFFF
    assert c.els[ids.index("low")]["condition"] == 0xFFFF


@pytest.mark.parametrize("cond", ["= amount.x > 1", "= f(amount)", "= amount > 1.1234567", "= amount >",
                                  "= amount > \"x\""])
def test_unsupported_feel_is_rejected_at_deploy(cond):
    with pytest.raises(ZbhipError):
        Compiled(bpmn.xor_process(condition=cond))


def test_unsupported_element_is_rejected():
    xml = process_xml({"fixture": "one_task.bpmn"}).replace("bpmn:serviceTask", "bpmn:userTask")
    with pytest.raises(ZbhipError):
        Compiled(xml)


def test_static_condition_is_rejected():
    # a condition without the `=` prefix is a static string (FeelExpressionLanguage.parseExpression):
    # evaluating it as a boolean raises an incident in the reference -> outside the subset
    xml = bpmn.xor_process().replace("= amount &gt; 1000", "amount &gt; 1000")
    with pytest.raises(ZbhipError):
        Compiled(xml)


def test_random_processes_compile_like_the_oracle():
    # tests/random_bpmn.py processes: the host compiler and the oracle agree on element indexing
    from random_bpmn import random_process
    for seed in range(30):
        xml = random_process(np.random.default_rng(1000 + seed))
        c = Compiled(xml)
        o = Oracle()
        assert o.deploy(xml) == 0
        assert [c.id(i) for i in range(len(c.els))] == [o.element_id(0, i) for i in range(len(c.els))]


def test_pass_through_elements_compile_like_the_oracle():
    # undefined task, manual task, none intermediate throw event: element type and event type as
    # the oracle's transformation (UNSPECIFIED for tasks, NONE for the throw event)
    from random_bpmn import random_process
    for seed in range(20):
        xml = random_process(np.random.default_rng(2000 + seed), pass_through=True)
        c = Compiled(xml)
        o = Oracle()
        assert o.deploy(xml) == 0
        tables = o.process_tables()[0]["elements"]
        assert [(c.id(i), int(c.els[i]["element_type"]), int(c.els[i]["event_type"])) for i in range(len(c.els))] == \
            [(t[2], t[0], t[1]) for t in tables]


@pytest.mark.parametrize("definition", ["messageEventDefinition", "signalEventDefinition", "linkEventDefinition"])
def test_throw_event_with_definition_is_rejected(definition):
    xml = (bpmn.createExecutableProcess("p").startEvent("s").intermediateThrowEvent("t").endEvent("e").done()
           .replace('<intermediateThrowEvent id="t"/>',
                    '<intermediateThrowEvent id="t"><%s id="d"/></intermediateThrowEvent>' % definition))
    with pytest.raises(ZbhipError):
        Compiled(xml)
    with pytest.raises(Exception):
        Oracle().deploy(xml)


def test_random_processes_with_error_boundary_events_compile_like_the_oracle():
    # random_bpmn's error boundary events on tasks and sub-processes: both sides accept them, with the
    # same element indexing
    from random_bpmn import random_process
    n_errors = 0
    for seed in range(40):
        xml = random_process(np.random.default_rng(9000 + seed), sub_processes=True, task_kinds=True, errors=True)
        n_errors += xml.count("errorEventDefinition")
        c = Compiled(xml)
        o = Oracle()
        assert o.deploy(xml) == 0
        assert [c.id(i) for i in range(len(c.els))] == [o.element_id(0, i) for i in range(len(c.els))]
    assert n_errors >= 20


def test_event_sub_processes_compile_like_the_oracle():
    # error-start event sub-processes in the process and in an embedded sub-process: the same element
    # indexing on both sides, the start event's error code in message_name, interrupting in job_retries
    from test_oracle_event_subprocess import esp_process
    b = bpmn.createExecutableProcess("wf").startEvent().subProcess("sub")
    b.eventSubProcess("inner-esp").startEvent("inner-start").error("E").serviceTask("fix", "fix").endEvent("ie")
    b.eventSubProcessDone().startEvent("s2").serviceTask("task", "test").endEvent("e2").subProcessDone()
    nested = b.endEvent("end").done()
    for xml in (esp_process(("esp", "esp-start", "E1"), ("esp2", "esp2-start", None)), nested):
        c = Compiled(xml)
        o = Oracle()
        assert o.deploy(xml) == 0
        assert [c.id(i) for i in range(len(c.els))] == [o.element_id(0, i) for i in range(len(c.els))]
        # (ZBHIP_EL_START_EVENT = 4, ZBHIP_EV_ERROR = 2 -- zbhip.h)
        starts = [i for i in range(len(c.els)) if int(c.els[i]["element_type"]) == 4
                  and int(c.els[i]["event_type"]) == 2]
        assert starts and all(int(c.els[i]["job_retries"]) & 1 for i in starts)
