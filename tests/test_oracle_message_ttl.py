"""The oracle's buffered messages (zb_oracle.cpp publish_message / message_subscription_create /
expire_message; MessagePublishProcessor.java:83-185, MessageCorrelator.java:41-96, DbMessageState.java:
225-349, MessageTimeToLiveChecker.java:35-124, MessageBatchExpireProcessor.java:33-52) pinned on the
reference's own tests -- PublishMessageTest, ExpireMessageTest and MessageCorrelationTest (engine/src/test/
.../processing/message/) -- run through the restated processing loop with its scheduled tasks (tests/psm.py,
one partition over the oracle engine, a controlled clock).  Message variables are outside the oracle's
subset: the tests that check them through variables are pinned here on the message keys instead."""
from psm import Client, Clock
from test_gpu_scheduled import KEY_A, KEY_B, Cluster, PartitionLoop
from test_oracle_timers import NOW
from zeebe_amd import abi, bpmn

HOUR = 3600000


def cluster(*deployments):
    clock = Clock(NOW)
    cl = Cluster([PartitionLoop(clock, list(deployments))], clock)
    cl.settle()
    return cl


def write(cl, *recs):
    start = len(cl.parts[0].log.entries)
    Client(cl.parts[0].log).write(*recs)
    cl.settle()
    return cl.parts[0].log.entries[start:]


def of(entries, vt, intent, rt=abi.RT_EVENT):
    return [r for r in entries if r.value_type == vt and r.intent == intent and r.record_type == rt]


def test_publish_buffers_and_the_ttl_checker_expires():
    # PublishMessageTest.shouldPublishMessage (:50-70); ExpireMessageTest.shouldExpireMessageAfterTTL (:52-84)
    # and shouldHaveNoSourceRecordPositionOnExpire (:108-125)
    cl = cluster()
    t = cl.clock.now
    e = write(cl, Client.publish_message("order canceled", "order-123", timestamp=t, time_to_live=100),
              Client.publish_message("order shipped", "order-123", timestamp=t, time_to_live=100))
    pub = of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)
    assert [r.value["timeToLive"] for r in pub] == [100, 100] and not of(e, abi.VT_MESSAGE, abi.MSG_EXPIRED)
    v = pub[0].value
    assert (v["name"], v["correlationKey"], v["messageId"], v["deadline"]) == ("order canceled", "order-123", "", t + 100)
    keys = [r.key for r in pub]
    state = cl.parts[0].state()
    assert "MESSAGE_STATS|messagesDeadlineCount|2" in state and "MESSAGE_DEADLINES|%d|%d" % (t + 100, keys[0]) in state
    cl.increase_time(60000)  # EngineConfiguration.DEFAULT_MESSAGES_TTL_CHECKER_INTERVAL
    log = cl.parts[0].log.entries
    batch = [r for r in log if r.value_type == abi.VT_MESSAGE_BATCH]
    assert len(batch) == 1 and batch[0].value["messageKeys"] == tuple(keys) and batch[0].source_position < 0
    expired = of(log, abi.VT_MESSAGE, abi.MSG_EXPIRED)
    assert [r.key for r in expired] == keys
    assert expired[0].value == {"name": "", "correlationKey": "", "timeToLive": -1, "variables": (), "messageId": "",
                                "deadline": -1, "tenantId": "<default>"}
    state = cl.parts[0].state()
    assert "MESSAGE_STATS|messagesDeadlineCount|0" in state and not [r for r in state if r.startswith("MESSAGE_KEY|")]


def test_zero_and_negative_ttl_expire_immediately():
    # ExpireMessageTest.shouldExpireMessageImmediatelyWithZeroTTL (:86-106); PublishMessageTest
    # shouldPublishMessageWithZeroTTL / WithNegativeTTL (:93-109)
    cl = cluster()
    e = write(cl, Client.publish_message("order canceled", "order-123", time_to_live=0),
              Client.publish_message("order canceled", "order-123", time_to_live=-1))
    exp = of(e, abi.VT_MESSAGE, abi.MSG_EXPIRED)
    assert [r.key for r in exp] == [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    assert [(r.value["name"], r.value["correlationKey"], r.value["timeToLive"], r.value["messageId"]) for r in exp] == \
        [("order canceled", "order-123", 0, ""), ("order canceled", "order-123", -1, "")]


def test_message_ids():
    # PublishMessageTest.shouldRejectToPublishSameMessageWithId (:176-188), shouldPublishSecondMessageWith
    # DifferentId (:124-135), shouldPublishSameMessageWithEmptyId (:163-174); the id is free again once the
    # message expired (DbMessageState.remove :328-333)
    cl = cluster()
    e = write(cl, Client.publish_message("order canceled", "order-123", timestamp=cl.clock.now, time_to_live=1000, message_id="id-1"),
              Client.publish_message("order canceled", "order-123", timestamp=cl.clock.now, time_to_live=1000, message_id="id-1"),
              Client.publish_message("order canceled", "order-123", timestamp=cl.clock.now, time_to_live=1000, message_id="id-2"),
              Client.publish_message("order canceled", "order-123", timestamp=cl.clock.now, time_to_live=1000, message_id=""),
              Client.publish_message("order canceled", "order-123", timestamp=cl.clock.now, time_to_live=1000, message_id=""))
    rej = [r for r in e if r.record_type == abi.RT_REJECTION]
    assert len(rej) == 1 and rej[0].rejection_type == abi.REJ_ALREADY_EXISTS
    assert rej[0].rejection_reason == ("Expected to publish a new message with id 'id-1', but a message with that id "
                                       "was already published")
    assert rej[0].value["messageId"] == "id-1"
    assert len(of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)) == 4
    assert "MESSAGE_IDS|<default>|order canceled|order-123|id-2" in cl.parts[0].state()
    cl.increase_time(60000)
    e = write(cl, Client.publish_message("order canceled", "order-123", time_to_live=0, message_id="id-1"))
    assert of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)


def test_correlate_message_published_before():
    # MessageCorrelationTest.shouldCorrelateMessageIfPublishedBefore (:133-162) and shouldCorrelateFirst
    # PublishedMessage (:225-253): MESSAGE_SUBSCRIPTION:CREATE correlates the first buffered message
    # (CORRELATING with its key, PROCESS_MESSAGE_SUBSCRIPTION:CORRELATE instead of the CREATE
    # acknowledgement); the message stays buffered, correlated to the process (MESSAGE_CORRELATED)
    xml = bpmn.message_catch_process("process", "message", "key", "receive-message")
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.publish_message("message", "order-123", timestamp=cl.clock.now, time_to_live=HOUR),
              Client.publish_message("message", "order-123", timestamp=cl.clock.now, time_to_live=HOUR))
    m1, m2 = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    e = write(cl, Client.create("process", (("key", "order-123"),)))
    corr = of(e, abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CORRELATING)
    assert len(corr) == 1 and corr[0].value["messageKey"] == m1
    assert not of(e, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CREATE, abi.RT_COMMAND)
    assert [r.value["messageKey"] for r in of(e, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATED)] == [m1]
    assert [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
            and r.value["bpmnElementType"] == "PROCESS"]
    state = cl.parts[0].state()
    assert "MESSAGE_CORRELATED|%d|process" % m1 in state and "MESSAGE_KEY|%d" % m2 in "".join(state)
    assert not [r for r in state if r.startswith(("MESSAGE_SUBSCRIPTION_BY_KEY|", "PROCESS_SUBSCRIPTION_BY_KEY|"))]


def test_correlate_only_once_per_process():
    # MessageCorrelationTest.shouldCorrelateMessageOnlyOnceIfPublishedBefore (:482-510): two catch events of
    # one name; the first message correlates to the first, then (MESSAGE_CORRELATED) the second message to
    # the second; shouldCorrelateMessageOnlyOncePerProcess (:394-429): two instances subscribed before
    xml = (bpmn.createExecutableProcess("process").startEvent().intermediateCatchEvent("message1")
           .message("ping", "key").intermediateCatchEvent("message2").message("ping", "key").done())
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.publish_message("ping", "123", timestamp=cl.clock.now, time_to_live=HOUR),
              Client.publish_message("ping", "123", timestamp=cl.clock.now, time_to_live=HOUR))
    m1, m2 = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    e = write(cl, Client.create("process", (("key", "123"),)))
    got = [(r.value["elementId"], r.value["messageKey"]) for r in of(e, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION,
                                                                         abi.PMS_CORRELATED)]
    assert got == [("message1", m1), ("message2", m2)]
    single = bpmn.message_catch_process("single", "message", "key", "receive-message")
    cl = cluster((single, KEY_B, 1))
    e = write(cl, Client.create("single", (("key", "order-123"),)), Client.create("single", (("key", "order-123"),)))
    piks = [r.key for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATED
            and r.value["bpmnElementType"] == "PROCESS"]
    e = write(cl, Client.publish_message("message", "order-123", timestamp=cl.clock.now, time_to_live=HOUR),
              Client.publish_message("message", "order-123", timestamp=cl.clock.now, time_to_live=HOUR))
    keys = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    got = [(r.value["messageKey"], r.value["processInstanceKey"])
           for r in of(e, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATED)]
    assert got == list(zip(keys, piks))


def test_no_correlation_after_the_ttl():
    # MessageCorrelationTest.shouldNotCorrelateMessageAfterTTL (:942-992): TTL 0, 10 s and 20 s messages; 10 s
    # later the subscription opens: only the third one correlates (deadline > now)
    xml = (bpmn.createExecutableProcess("wf").startEvent().serviceTask("task", "test").intermediateCatchEvent("catch")
           .message("a", "key").endEvent().done())
    cl = cluster((xml, KEY_A, 1))
    e = write(cl, Client.create("wf", (("key", "key-1"),)))
    job = [r.key for r in e if r.value_type == abi.VT_JOB and r.intent == abi.JOB_CREATED][0]
    t = cl.clock.now
    e = write(cl, *[Client.publish_message("a", "key-1", timestamp=t, time_to_live=ttl) for ttl in (0, 10000, 20000)])
    keys = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    cl.clock.now += 10000
    e = write(cl, Client.complete_job(job))
    assert [r.value["messageKey"] for r in of(e, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATED)] == [keys[2]]
