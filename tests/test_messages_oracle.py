"""Config 5 on the CPU oracle: SubscriptionUtil known answers, the App. A.5 sequences (remote and
local message partition), state after each protocol phase, and the multi-partition example of
MessageCorrelationMultiplePartitionsTest.  CPU only."""
import numpy as np
import pytest

from oracle.oracle import Oracle, java_hash, subscription_partition
from zeebe_amd import abi, bpmn

from helpers import MessageCluster, OracleAdapter, load_appendix_a5, symbolic

XML = bpmn.message_catch_process()


def test_subscription_hash_known_answers():
    # SubscriptionUtilTest.java:23-38
    assert java_hash("a") == 97 and java_hash("b") == 98 and java_hash("c") == 99
    assert java_hash("foobar") == -1268878963
    assert java_hash("") == 0
    assert subscription_partition("a", 10) == 7 + 1
    assert subscription_partition("b", 3) == 2 + 1
    assert subscription_partition("c", 11) == 0 + 1
    assert subscription_partition("foobar", 100) == 63 + 1


def test_signed_byte_hash():
    # bytes >= 0x80 are added as negative Java bytes (SubscriptionUtil.java:27-29)
    s = "été"  # UTF-8 c3 a9 74 c3 a9
    h = 0
    for b in s.encode():
        h = (31 * h + (b - 256 if b >= 128 else b)) & 0xFFFFFFFF
    h = h - (1 << 32) if h >= 1 << 31 else h
    assert java_hash(s) == h


def test_multiple_partitions_correlation_keys():
    # MessageCorrelationMultiplePartitionsTest.java:36-40: item-2 -> 1, item-1 -> 2, item-0 -> 3
    assert [subscription_partition("item-%d" % i, 3) for i in (2, 1, 0)] == [1, 2, 3]


def _cluster(P):
    return MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, XML)


def _sym(cl, recs, p):
    o = cl.parts[p - 1]
    return [t for t in symbolic(recs, o.element_id, o.name, partition=p)]


@pytest.mark.parametrize("case", ["remote", "local"])
def test_appendix_a5(case):
    spec = load_appendix_a5()[case]
    P = spec["partitions"]
    cl = _cluster(P)
    key = spec["correlation_key"]
    kid = cl.intern_keys([key])[0]
    owner = 1  # the instance lives on partition 1
    keys = [[kid] if p == owner else [] for p in range(1, P + 1)]
    # create one instance on partition 1 only
    cmds_out = []
    for p in range(1, P + 1):
        if p != owner:
            cmds_out.append(abi.make_xparts(0))
            continue
        from helpers import create_commands, string_docs
        c = create_commands(1)
        c["doc_count"] = 1
        cmds_out.append(cl._run("create", p, c, string_docs(cl.var_id, [kid])))
    cl.exchange("subscribe", cmds_out)
    cl.publish([kid], [subscription_partition(key, P)])
    kinds = {abi.CMD_MSG_SUB_CREATE: "MSG_SUB_CREATE", abi.CMD_PMS_CREATE: "PMS_CREATE",
             abi.CMD_PMS_CORRELATE: "PMS_CORRELATE", abi.CMD_MSG_SUB_CORRELATE: "MSG_SUB_CORRELATE"}
    assert len(cl.log) == len(spec["steps"])
    for (phase, p, recs, ob), step in zip(cl.log, spec["steps"]):
        assert p == step["partition"], (phase, p)
        got = [t[:6] for t in _sym(cl, recs, p)]
        want = [list(t) for t in step["batch"]]
        assert got == want, (phase, p)
        assert [[kinds[int(x["kind"])], int(x["target_partition"])] for x in ob] == step["outbox"], phase
    # the protocol leaves nothing behind but the message statistics row and the key counters
    for p, o in enumerate(cl.parts, 1):
        st = [r for r in o.state() if not r.startswith("KEY|")]
        msg_partition = subscription_partition(key, P)
        assert st == (["MESSAGE_STATS|messagesDeadlineCount|0"] if p == msg_partition else []), (p, st)


def test_record_values_of_the_remote_protocol():
    cl = _cluster(2)
    kid = cl.intern_keys(["a"])[0]
    from helpers import create_commands, string_docs
    c = create_commands(1)
    c["doc_count"] = 1
    ob = cl._run("create", 1, c, string_docs(cl.var_id, [kid]))
    x = ob[0]
    pik = (1 << 51) + 1
    eik = (1 << 51) + 6
    assert int(x["element_instance_key"]) == eik and int(x["process_instance_key"]) == pik
    assert int(x["instance"]) == 0 and int(x["element_ord"]) == 5  # k6 is the instance's 6th key
    assert int(x["correlation_key"]) == kid and int(x["message_name"]) == cl.name_id
    assert int(x["interrupting"]) == 1 and int(x["message_key"]) == -1
    creating = [r for r in cl.log[0][2] if r["value_type"] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION][0]
    assert int(creating["partition"]) == 2 and int(creating["correlation_key"]) == kid
    assert int(creating["bpmn_process_id"]) == cl.parts[0].intern("process")
    # state between the phases: OPENING, then OPENED once the message partition acknowledged
    st = cl.parts[0].state()
    assert any(r.startswith("PROCESS_SUBSCRIPTION_BY_KEY|%d|msg|" % eik) and "state=OPENING" in r for r in st)
    assert any(r.startswith("EVENT_SCOPE|%d|" % eik) for r in st)
    cl.exchange("subscribe", [ob, abi.make_xparts(0)])
    assert any("state=OPENED" in r for r in cl.parts[0].state())
    st2 = cl.parts[1].state()
    assert "MESSAGE_SUBSCRIPTION_BY_NAME_AND_CORRELATION_KEY|<default>|msg|a|%d" % eik in st2
    assert any(r.startswith("MESSAGE_SUBSCRIPTION_BY_KEY|%d|msg|" % eik) and "correlating=0" in r for r in st2)
    # the PMS:CORRELATE command carries the message key of the publish
    cl.publish([kid], [2])
    pub = [r for r in cl.log if r[0] == "publish" and r[1] == 2][0]
    corr = [r for r in cl.log if r[0] == "correlate" and r[1] == 1][0]
    msg_key = int(pub[2][0]["key"])
    correlated = [r for r in corr[2] if r["value_type"] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION][0]
    assert int(correlated["message_key"]) == msg_key and int(correlated["partition"]) == 2


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_cluster_completes_every_instance(P):
    n = 40
    cl = _cluster(P)
    all_keys = ["k-%d-%d" % (p, i) for p in range(1, P + 1) for i in range(n)]
    ids = cl.intern_keys(all_keys)
    keys = [ids[(p - 1) * n:p * n] for p in range(1, P + 1)]
    cl.create(n, keys)
    cl.publish(ids, [subscription_partition(k, P) for k in all_keys])
    completed = sum(o.counters()["completed_instances"] for o in cl.parts)
    assert completed == n * P
    for p, o in enumerate(cl.parts, 1):
        st = [r for r in o.state() if not r.startswith("KEY|")]
        assert all(r.startswith("MESSAGE_STATS") for r in st), st[:3]


def test_one_message_correlates_once_per_process():
    # MessagePublishProcessor.correlateToSubscriptions: two instances of one process waiting on
    # the same key -> only the subscription with the lower element instance key correlates
    cl = _cluster(1)
    kid = cl.intern_keys(["shared"])[0]
    cl.create(2, [[kid, kid]])
    cl.publish([kid], [1])
    o = cl.parts[0]
    assert o.counters()["completed_instances"] == 1
    pub = cl.log[-1][2]
    assert sum(1 for r in pub if r["value_type"] == abi.VT_MESSAGE_SUBSCRIPTION and r["intent"] == abi.MS_CORRELATING) == 1
    st = o.state()
    assert sum(1 for r in st if r.startswith("PROCESS_SUBSCRIPTION_BY_KEY")) == 1


def test_duplicate_subscription_open_is_rejected():
    # MessageSubscriptionCreateProcessor: a second CREATE for the same element and name -> ack + rejection
    cl = _cluster(2)
    kid = cl.intern_keys(["a"])[0]
    from helpers import create_commands, string_docs
    c = create_commands(1)
    c["doc_count"] = 1
    ob = cl._run("create", 1, c, string_docs(cl.var_id, [kid]))
    from zeebe_amd.exchange import window_from_xparts
    twice = np.concatenate([ob, ob])
    cmds, xp = window_from_xparts(twice)
    recs, ob2 = OracleAdapter.window(cl.parts[1], cmds, None, xp)
    assert [int(r["record_type"]) for r in recs] == [abi.RT_EVENT, abi.RT_REJECTION]
    assert cl.parts[1].reason(1).startswith("Expected to open a new message subscription for element with key")
    assert len(ob2) == 2 and all(int(x["kind"]) == abi.CMD_PMS_CREATE for x in ob2)
