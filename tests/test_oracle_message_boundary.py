"""Interrupting message boundary events on the oracle cluster (CPU, test infrastructure): the
subscription opened with the task, then either the message first (the task terminated, the boundary
event taken) or the job first (the subscription closed: PROCESS_MESSAGE_SUBSCRIPTION:DELETING,
MESSAGE_SUBSCRIPTION:DELETE / DELETED, PROCESS_MESSAGE_SUBSCRIPTION:DELETE / DELETED).

Pins (engine/src/test/.../message/MessageCatchElementTest.java, parameter "int boundary event",
BOUNDARY_EVENT_PROCESS :71-80): shouldOpenMessageSubscription / shouldOpenProcessMessageSubscription
(:172-212), shouldCorrelateMessageAndContinue (:340-365: the task ELEMENT_TERMINATED, the boundary's
flow taken), testMessageSubscriptionLifecycle / testProcessMessageSubscriptionLifecycle (:367-416),
shouldHaveSame(Process)MessageSubscriptionKey (:418-467), shouldCloseMessageSubscription /
shouldCloseProcessMessageSubscription (:282-338: DELETED with the created key and value; DELETING
then DELETED -- the same unsubscribeFromEvents path the completed job takes); BoundaryEventTest
.shouldActivateBoundaryEventWhenEventTriggered (:100-139) and shouldUseScopeToExtractCorrelationKeys
(:315-350: the correlation key comes from the flow scope)."""
import numpy as np
import pytest

from helpers import MessageCluster, OracleAdapter, complete_commands
from oracle.oracle import Oracle, subscription_partition
from zeebe_amd import abi, bpmn

XML = bpmn.message_boundary_process()
N = 6


def cluster(P, xml=XML):
    return MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, xml)


def keys(P, n=N):
    return ["order-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]


def start(cl, P, n=N):
    ks = keys(P, n)
    ids = cl.intern_keys(ks)
    cl.create(n, [ids[(p - 1) * n:p * n] for p in range(1, P + 1)])
    return ks, ids


def job_completions(cl, n=N, which=None):
    """JOB:COMPLETE per partition for the instances in `which` (slot indices), job key ordinals from
    each oracle partition's create window."""
    out = []
    for p, part in enumerate(cl.parts, start=1):
        recs = next(r for ph, q, r, _ in cl.log if ph == "create" and q == p)
        base = int(recs["source_index"].min())
        jobs = {}
        for r in recs:
            if int(r["value_type"]) == abi.VT_JOB and int(r["intent"]) == abi.JOB_CREATED:
                jobs[int(r["source_index"]) - base] = int(r["key"])
        sel = sorted(jobs) if which is None else [i for i in which if i in jobs]
        out.append(complete_commands(sel, [part.ordinal_of(i, jobs[i]) for i in sel]) if sel else None)
    return out


def all_records(cl):
    out = []
    for ph, p, recs, _ in cl.log:
        part = cl.parts[p - 1]
        for r in recs:
            out.append((ph, p, int(r["record_type"]), int(r["value_type"]), int(r["intent"]), int(r["key"]),
                        int(r["scope_key"]), int(r["process_instance_key"]),
                        part.element_id(int(r["process_idx"]), int(r["element_idx"])) if r["element_idx"] >= 0 and
                        int(r["value_type"]) != abi.VT_VARIABLE else None, r))
    return out


def of_instance(recs, pik):
    return [t for t in recs if t[7] == pik]


@pytest.mark.parametrize("P", [1, 3])
def test_message_first_terminates_the_task(P):
    cl = cluster(P)
    ks, ids = start(cl, P)
    cl.publish(ids, [subscription_partition(k, P) for k in ks])
    recs = all_records(cl)
    piks = sorted({t[7] for t in recs if t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 5 and t[8] == "boundaryEventProcess"})
    assert len(piks) == N * P  # every instance completed through the boundary event's end event
    for pik in piks:
        mine = of_instance(recs, pik)
        # (at P > 1 the commands a partition receives are its batches' sources, not records of them)
        ms = [(t[2], t[4], t[5]) for t in mine if t[3] == abi.VT_MESSAGE_SUBSCRIPTION]
        pms = [(t[2], t[4], t[5]) for t in mine if t[3] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION]
        if P == 1:
            assert [(rt, it) for rt, it, _ in ms] == [(abi.RT_COMMAND, abi.MS_CREATE), (abi.RT_EVENT, abi.MS_CREATED),
                                                     (abi.RT_EVENT, abi.MS_CORRELATING), (abi.RT_COMMAND, abi.MS_CORRELATE),
                                                     (abi.RT_EVENT, abi.MS_CORRELATED)]
            assert ms[0][2] == -1 and ms[3][2] == -1  # shouldHaveSameMessageSubscriptionKey
            assert [(rt, it) for rt, it, _ in pms] == [(abi.RT_EVENT, abi.PMS_CREATING), (abi.RT_COMMAND, abi.PMS_CREATE),
                                                      (abi.RT_EVENT, abi.PMS_CREATED), (abi.RT_COMMAND, abi.PMS_CORRELATE),
                                                      (abi.RT_EVENT, abi.PMS_CORRELATED)]
        ev = [(it, k) for rt, it, k in ms if rt == abi.RT_EVENT]
        assert [it for it, _ in ev] == [abi.MS_CREATED, abi.MS_CORRELATING, abi.MS_CORRELATED]
        assert len({k for _, k in ev}) == 1
        pev = [(it, k) for rt, it, k in pms if rt == abi.RT_EVENT]
        assert [it for it, _ in pev] == [abi.PMS_CREATING, abi.PMS_CREATED, abi.PMS_CORRELATED]
        assert len({k for _, k in pev}) == 1  # shouldHaveSameProcessMessageSubscriptionKey
        task_eik = next(t[5] for t in mine if t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 3 and t[8] == "task")
        assert all(t[6] == task_eik for t in mine if t[3] in (abi.VT_MESSAGE_SUBSCRIPTION, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION))
        # BoundaryEventTest.shouldActivateBoundaryEventWhenEventTriggered's subsequence (message trigger)
        seq = [(t[3], t[4], t[8]) for t in mine if t[3] in (abi.VT_PROCESS_INSTANCE, abi.VT_JOB)]
        want = [(abi.VT_PROCESS_INSTANCE, 6, "task"), (abi.VT_JOB, abi.JOB_CANCELED, "task"),
                (abi.VT_PROCESS_INSTANCE, 7, "task"), (abi.VT_PROCESS_INSTANCE, 2, "boundary")]
        it = iter(seq)
        assert all(w in it for w in want)
        assert any(t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 1 and t[8] == "to-end2" for t in mine)
        assert not any(t[8] == "end" for t in mine)
        assert not any(t[3] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and t[4] == abi.PMS_DELETING for t in mine)
    for part in cl.parts:
        st = part.state()
        assert not any(r.startswith(("PROCESS_SUBSCRIPTION_BY_KEY", "MESSAGE_SUBSCRIPTION_BY_KEY", "EVENT_SCOPE")) for r in st)


@pytest.mark.parametrize("P", [1, 3])
def test_job_first_closes_the_subscription(P):
    cl = cluster(P)
    ks, ids = start(cl, P)
    created = {}
    for t in all_records(cl):
        if t[3] == abi.VT_MESSAGE_SUBSCRIPTION and t[4] == abi.MS_CREATED:
            created[t[6]] = t
    cl.commands("complete", job_completions(cl))
    recs = all_records(cl)
    piks = sorted({t[7] for t in recs if t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 5 and t[8] == "boundaryEventProcess"})
    assert len(piks) == N * P
    for pik in piks:
        mine = of_instance(recs, pik)
        assert any(t[8] == "end" for t in mine) and not any(t[8] == "end2" for t in mine)
        pms = [(t[2], t[4], t[5]) for t in mine if t[3] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and t[2] == abi.RT_EVENT]
        # shouldCloseProcessMessageSubscription: DELETING then DELETED, the key of CREATING / CREATED
        assert [it for _, it, _ in pms] == [abi.PMS_CREATING, abi.PMS_CREATED, abi.PMS_DELETING, abi.PMS_DELETED]
        assert len({k for _, _, k in pms}) == 1
        ms = [t for t in mine if t[3] == abi.VT_MESSAGE_SUBSCRIPTION]
        want = [(abi.RT_COMMAND, abi.MS_CREATE), (abi.RT_EVENT, abi.MS_CREATED), (abi.RT_COMMAND, abi.MS_DELETE),
                (abi.RT_EVENT, abi.MS_DELETED)]
        got = [(t[2], t[4]) for t in ms]
        assert got == want if P == 1 else [g for g in got if g[0] == abi.RT_EVENT] == want[1::2]
        # shouldCloseMessageSubscription: DELETED with the created key, element instance key,
        # message name and correlation key
        d, c = ms[-1][9], created[ms[-1][6]][9]
        assert int(d["key"]) == int(c["key"]) and int(d["scope_key"]) == int(c["scope_key"])
        assert int(d["message_name"]) == int(c["message_name"]) and int(d["correlation_key"]) == int(c["correlation_key"])
        if len(ms) == 4:  # a local subscription: the DELETE command's value: closeMessageSubscription sets no bpmnProcessId / correlation key
            assert int(ms[2][9]["correlation_key"]) == abi.NO_STRING and int(ms[2][9]["bpmn_process_id"]) == 0xFFFF
        # unsubscribeFromEvents runs between the job's COMPLETED and the task's ELEMENT_COMPLETED
        order = [(t[3], t[4], t[8]) for t in mine]
        i_del = order.index((abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_DELETING, "boundary"))
        assert order.index((abi.VT_PROCESS_INSTANCE, 4, "task")) < i_del < order.index((abi.VT_PROCESS_INSTANCE, 5, "task"))
    for part in cl.parts:
        st = part.state()
        assert not any(r.startswith(("PROCESS_SUBSCRIPTION_BY_KEY", "MESSAGE_SUBSCRIPTION")) for r in st), st[:4]


def test_closing_subscription_is_state_until_deleted():
    # P = 3: the job completes on the PI partition; until the acknowledgement arrives the subscription
    # is CLOSING there (ProcessMessageSubscriptionDeletingApplier) -- also after the instance ended
    P = 3
    cl = cluster(P)
    ks, ids = start(cl, P, 2)
    remote = [i for i, k in enumerate(ks[:2]) if subscription_partition(k, P) != 1]
    assert remote
    cmds = job_completions(cl, 2, which=remote)
    cl._run("complete", 1, cmds[0])
    st = cl.parts[0].state()
    closing = [r for r in st if r.startswith("PROCESS_SUBSCRIPTION_BY_KEY") and "state=CLOSING" in r]
    assert len(closing) == len(remote)
    # the instances ended with the job (start -> task -> end): only the subscription rows remain
    assert not any(r.startswith("ELEMENT_INSTANCE_KEY") and "elementId=task" in r for r in st)


def test_correlation_key_from_the_flow_scope():
    # BoundaryEventTest.shouldUseScopeToExtractCorrelationKeys: the subscription's correlation key is
    # the process scope's variable (the task's own scope is not consulted)
    cl = cluster(1)
    ks, ids = start(cl, 1, 1)
    rec = next(t[9] for t in all_records(cl) if t[3] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and t[4] == abi.PMS_CREATING)
    assert int(rec["correlation_key"]) == ids[0]
    assert cl.parts[0].element_id(int(rec["process_idx"]), int(rec["element_idx"])) == "boundary"


NON_INT = bpmn.message_boundary_process("nonIntBoundaryEventProcess", interrupting=False)


@pytest.mark.parametrize("P", [1, 3])
def test_non_interrupting_boundary_correlates_every_message(P):
    # MessageCatchElementTest "non int boundary event" (NON_INT_BOUNDARY_EVENT_PROCESS :81-91): the
    # message activates the boundary event ("event" ELEMENT_COMPLETED, its flow taken) and the task stays
    # ACTIVATED; ProcessMessageSubscriptionCorrelatedApplier / MessageSubscriptionCorrelatedApplier keep
    # both subscriptions (OPENED with the CORRELATED record; not correlating, the message key kept), so a
    # second message correlates again (BoundaryEventTest.shouldTriggerMultipleNonInterruptingBoundaryEvents
    # :394-470); the job's completion then closes them (DELETING .. DELETED, the last message key in the
    # values) and the instance completes through the task's own end event
    cl = cluster(P, NON_INT)
    ks, ids = start(cl, P)
    parts = [subscription_partition(k, P) for k in ks]
    cl.publish(ids, parts)
    cl.publish(ids, parts)
    for part in cl.parts:
        rows = [r for r in part.state() if r.startswith(("PROCESS_SUBSCRIPTION_BY_KEY", "MESSAGE_SUBSCRIPTION_BY_KEY"))]
        for r in rows:
            assert "messageKey=-1" not in r
            assert "state=OPENED" in r or "correlating=0" in r, r
    assert sum(len([r for r in part.state() if r.startswith("PROCESS_SUBSCRIPTION_BY_KEY")]) for part in cl.parts) == N * P
    cl.commands("complete", job_completions(cl))
    recs = all_records(cl)
    piks = sorted({t[7] for t in recs if t[3] == abi.VT_PROCESS_INSTANCE and t[4] == 5 and t[8] == "nonIntBoundaryEventProcess"})
    assert len(piks) == N * P
    for pik in piks:
        mine = of_instance(recs, pik)
        pi = [(t[4], t[8]) for t in mine if t[3] == abi.VT_PROCESS_INSTANCE and t[2] == abi.RT_EVENT]
        assert pi.count((5, "boundary")) == 2 and pi.count((5, "end2")) == 2 and pi.count((5, "end")) == 1
        assert (7, "task") not in pi and pi.count((5, "task")) == 1
        pev = [(t[4], t[5], t[9]) for t in mine if t[3] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and t[2] == abi.RT_EVENT]
        assert [it for it, _, _ in pev] == [abi.PMS_CREATING, abi.PMS_CREATED, abi.PMS_CORRELATED, abi.PMS_CORRELATED,
                                            abi.PMS_DELETING, abi.PMS_DELETED]
        assert len({k for _, k, _ in pev}) == 1 and not int(pev[2][2]["interrupting"])
        # the stored record after the second correlation: its message key
        assert int(pev[4][2]["message_key"]) == int(pev[3][2]["message_key"]) != int(pev[2][2]["message_key"])
        ms = [t[4] for t in mine if t[3] == abi.VT_MESSAGE_SUBSCRIPTION and t[2] == abi.RT_EVENT]
        assert ms == [abi.MS_CREATED, abi.MS_CORRELATING, abi.MS_CORRELATED, abi.MS_CORRELATING, abi.MS_CORRELATED,
                      abi.MS_DELETED]
    for part in cl.parts:
        assert [r for r in part.state() if not r.startswith(("KEY|", "MESSAGE_STATS"))] == []


def test_correlation_key_incident_on_the_task():
    # BoundaryEventTest.shouldHaveScopeKeyIfBoundaryEvent (:352-391): a correlation key that is not a
    # string or a number -> EXTRACT_VALUE_ERROR on the task (elementId task, elementInstanceKey = the
    # task's ACTIVATING key, variableScopeKey = the process instance), no subscription, no job, the task
    # left ACTIVATING.  (The gfx950 path falls back on such keys: no device counterpart.)
    o = Oracle()
    o.deploy(bpmn.message_boundary_process(correlation_key="orderId"))
    name = o.intern("orderId")
    from helpers import create_commands
    c = create_commands(1)
    c["doc_count"] = 1
    d = abi.make_docs(1)
    d["name_id"], d["type"], d["value"] = name, abi.DOC_BOOL, 1
    o.submit(c, d)
    o.run()
    recs = o.records()
    el = lambda r: o.element_id(int(r["process_idx"]), int(r["element_idx"]))  # noqa: E731
    task = [r for r in recs if int(r["value_type"]) == abi.VT_PROCESS_INSTANCE and el(r) == "task"]
    assert [int(r["intent"]) for r in task if int(r["record_type"]) == abi.RT_EVENT] == [2]  # ACTIVATING only
    inc = [r for r in recs if int(r["value_type"]) == abi.VT_INCIDENT]
    assert len(inc) == 1
    r = inc[0]
    assert int(r["partition"]) == 4  # ErrorType.EXTRACT_VALUE_ERROR
    assert el(r) == "task" and int(r["scope_key"]) == int(task[-1]["key"])
    pik = int(r["process_instance_key"])
    assert int(r["message_key"]) == pik  # variableScopeKey: the task's flow scope
    assert not any(int(x["value_type"]) in (abi.VT_JOB, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION) for x in recs)
