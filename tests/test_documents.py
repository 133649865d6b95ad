"""Multi-entry variable documents: the order the reference merges them in.

IndexedDocument (engine/.../state/variable/IndexedDocument.java:20-63) indexes a document's msgpack map
into an agrona Int2IntHashMap (org.agrona 1.19.2, parent/pom.xml:38 -- a third-party dependency absent
from the reference tree) keyed by each key's byte offset, and VariableBehavior.mergeLocalDocument /
mergeDocument (VariableBehavior.java:60-150) iterate that map.  No test of the reference pins the order
of a multi-entry document's VARIABLE records (they compare variables as sets), so this order is parity
UNPINNED: the oracle restates agrona's published algorithm (oracle/zb_oracle.cpp AgronaIntMap, with
Iterator.remove's compactChain), the product computes the same order from the key offsets
(zbhip_doc_merge_order), and these tests hold the two to each other and to hand-derived cases."""
import numpy as np
import pytest

from psm import Client
from test_gpu_scheduled import KEY_A
from test_oracle_message_ttl import cluster, of, write
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import doc_entries, msgpack_key_offsets


def _order(variables):
    names = {}
    d = doc_entries(variables, lambda n: names.setdefault(n, len(names)), lambda s: 0, lambda items: 0)
    return [variables[int(p)][0] for p in d["pad"][:, 0]], bool(d["pad"][0, 1] & 1)


def test_key_offsets_follow_the_msgpack_encoding():
    # fixmap header, fixstr names, fixint / uint8 / int16 / float64 / str8 values
    v = [("a", 1), ("bb", 200), ("c", -300), ("d", 1.5), ("e", "x" * 40), ("f", None)]
    assert msgpack_key_offsets(v) == [1, 1 + 2 + 1, 4 + 3 + 2, 9 + 2 + 3, 14 + 2 + 9, 25 + 2 + 42]


@pytest.mark.parametrize("variables, order, displaced", [
    # offsets 1, 4: slots 1 and 4, iterated downwards
    ([("a", 1), ("b", 2)], ["b", "a"], False),
    # offsets 1, 9: both hash to slot 1, the second probes to slot 2
    ([("abc", "xyz"), ("q", 1)], ["q", "abc"], True),
    # offsets 1, 4, 7: the top slot (7) is taken, so the iteration starts below the first free slot, 0 --
    # wrapping to 7: the same order as from the top
    ([("a", 1), ("b", 2), ("c", 3)], ["c", "b", "a"], False),
    # offsets 1, 7, 15: 15 hashes to the taken top slot and wraps to slot 0; the first free slot is 2, so
    # the iteration visits 1, 0, 7 (from the top it would be 7, 1, 0)
    ([("a", "abc"), ("b", "abcde"), ("c", 1)], ["a", "c", "b"], True),
    # seven entries: past (int)(8 * 0.65f) = 5 the table doubles to 16 slots (offsets 1, 5, .., 25)
    ([("x%d" % i, i) for i in range(7)], ["x3", "x6", "x2", "x5", "x1", "x4", "x0"], True),
])
def test_hand_derived_merge_orders(variables, order, displaced):
    assert _order(variables) == (order, displaced)


def _created_names(cl, e):
    return [r.value["name"] for r in of(e, abi.VT_VARIABLE, abi.VAR_CREATED)]


def _random_doc(rng, n):
    names = ["v%d_%s" % (i, "x" * int(rng.integers(0, 40))) for i in range(n)]
    out = []
    for nm in names:
        k = int(rng.integers(0, 6))
        val = (int(rng.integers(-70000, 70000)) if k == 0 else int(rng.integers(0, 128)) if k == 1 else
               "s" * int(rng.integers(0, 300)) if k == 2 else bool(k == 3) if k == 3 else
               float(rng.integers(0, 1000)) / 4 if k == 4 else None)
        out.append((nm, val))
    return out


def test_product_order_equals_the_oracle_merge_order():
    # PROCESS_INSTANCE_CREATION's document through the engine-only loop (mergeLocalDocument): the oracle's
    # VARIABLE:CREATED order is the order zbhip_doc_merge_order hands the device, for documents of 2 to 14
    # entries (resizes at 6 and 11 entries, wrapping probe chains, str8 / str16 values)
    xml = bpmn.createExecutableProcess("p").startEvent().serviceTask("t", "t").endEvent().done()
    rng = np.random.default_rng(5)
    cl = cluster((xml, KEY_A, 1))
    seen_displaced = seen_wrap = 0
    for _ in range(120):
        doc = _random_doc(rng, int(rng.integers(2, 15)))
        order, displaced = _order(doc)
        e = write(cl, Client.create("p", variables=doc))
        assert _created_names(cl, e) == order
        seen_displaced += displaced
        offs = msgpack_key_offsets(doc)
        seen_wrap += any(o % 8 == 7 for o in offs)
    assert seen_displaced > 10 and seen_wrap > 10


def test_merge_document_removes_updated_entries_per_scope():
    # mergeDocument from a task inside a sub-process whose scope holds `y`: the sub-process's scope takes the
    # differing `y` (VARIABLE:UPDATED there, removed from the document), the process instance's the rest in
    # the order left; an equal value is not removed (it goes on to the process instance's scope)
    b = bpmn.createExecutableProcess("p").startEvent().subProcess("sub").startEvent().serviceTask("t", "t")
    xml = b.endEvent().subProcessDone().zeebeInputExpression("x", "y").endEvent().done()
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.create("p", variables=[("x", 3)]))
    job = of(e, abi.VT_JOB, abi.JOB_CREATED)[0]
    sub = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATED
           and r.value["elementId"] == "sub"][0]
    doc = [("a", 1), ("y", 9), ("b", 2), ("x", 3)]
    e = write(cl, Client.complete_job(job.key, variables=doc))
    var = [(r.value["name"], r.intent, r.value["scopeKey"]) for r in e if r.value_type == abi.VT_VARIABLE]
    pik = job.value["processInstanceKey"]
    rest = [n for n in _order(doc)[0] if n != "y"]
    assert var[0] == ("y", abi.VAR_UPDATED, sub.key)
    assert [(n, s) for n, _, s in var[1:]] == [(n, pik) for n in rest if n != "x"]
