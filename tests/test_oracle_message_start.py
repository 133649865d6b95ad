"""The oracle's message start events (zb_oracle.cpp publish_message -> trigger_message_start_event,
on_activate of the process, correlate_buffered_start_message; MessagePublishProcessor.java:157-180,
EventHandle.java:176-235, ProcessProcessor.java:98-114,186-206, BpmnBufferedMessageStartEventBehavior.java:
56-120, MessageStartEventSubscriptionCorrelatedApplier.java:27-39, BufferedStartMessageEventStateApplier.java:
36-66) pinned on the reference's MessageStartEventTest (engine/src/test/.../processing/message/), run through
the restated processing loop (tests/psm.py, one partition over the oracle engine, a controlled clock).  The
test client publishes with a time-to-live of one hour (PublishMessageClient.java:27).  Message variables are
outside the oracle's subset: the tests that tell the messages apart by a variable `x` are pinned here on the
message keys of MESSAGE_START_EVENT_SUBSCRIPTION:CORRELATED instead (its messageKey names the message that
started the instance)."""
from psm import Client
from test_gpu_scheduled import KEY_A, KEY_B
from test_oracle_message_ttl import HOUR, cluster, of, write
from zeebe_amd import abi, bpmn

SINGLE = bpmn.createExecutableProcess("wf").startEvent("start").message("a").serviceTask("task", "test").done()


def single(start_id):
    return bpmn.createExecutableProcess("wf").startEvent(start_id).message("a").serviceTask("task", "test").done()


def multiple():
    # MessageStartEventTest.multipleStartEvents (:71-77)
    b = bpmn.createExecutableProcess("wf")
    b.startEvent("start-a").message("a").serviceTask("task", "test")
    b.moveToNode("task")
    b.current = None
    b.startEvent("start-b").message("b").connectTo("task")
    return b.done()


def publish(cl, name, key, ttl=HOUR):
    return Client.publish_message(name, key, timestamp=cl.clock.now, time_to_live=ttl)


def started(entries):
    """(messageKey, processInstanceKey) of every MESSAGE_START_EVENT_SUBSCRIPTION:CORRELATED."""
    return [(r.value["messageKey"], r.value["processInstanceKey"])
            for r in of(entries, abi.VT_MESSAGE_START_EVENT_SUBSCRIPTION, abi.MSES_CORRELATED)]


def jobs(entries):
    return [r for r in of(entries, abi.VT_JOB, abi.JOB_CREATED)]


def test_message_starts_an_instance():
    # shouldCorrelateMessageToStartEvent (:79-104), shouldCorrelateMessageSubscription (:106-134),
    # shouldCreateNewInstanceWithNameLiteral (:136-158)
    cl = cluster((SINGLE, KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"))
    msg = of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)[0]
    corr = of(e, abi.VT_MESSAGE_START_EVENT_SUBSCRIPTION, abi.MSES_CORRELATED)
    assert len(corr) == 1
    pi = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATING
          and r.value["bpmnElementType"] == "PROCESS"][0]
    start = [r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATING
             and r.value["bpmnElementType"] == "START_EVENT"][0]
    v = start.value
    assert (v["processDefinitionKey"], v["bpmnProcessId"], v["version"], v["processInstanceKey"], v["flowScopeKey"]) == \
        (pi.value["processDefinitionKey"], "wf", 1, pi.key, pi.key)
    assert v["bpmnEventType"] == "MESSAGE" and v["elementId"] == "start"
    c = corr[0].value
    assert (c["processDefinitionKey"], c["bpmnProcessId"], c["processInstanceKey"], c["startEventId"], c["messageKey"],
            c["messageName"], c["correlationKey"]) == (KEY_A, "wf", pi.key, "start", msg.key, "a", "key-1")
    # the batch of the publish: PUBLISHED, CORRELATED, PROCESS_EVENT:TRIGGERING (the process definition's event
    # scope), ACTIVATE_ELEMENT of the process; then (follow-ups) the process and the triggered start event
    seq = [(r.value_type, r.intent, r.record_type) for r in e]
    assert seq[:5] == [(abi.VT_MESSAGE, abi.MSG_PUBLISH, abi.RT_COMMAND), (abi.VT_MESSAGE, abi.MSG_PUBLISHED, abi.RT_EVENT),
                       (abi.VT_MESSAGE_START_EVENT_SUBSCRIPTION, abi.MSES_CORRELATED, abi.RT_EVENT),
                       (abi.VT_PROCESS_EVENT, abi.PE_TRIGGERING, abi.RT_EVENT),
                       (abi.VT_PROCESS_INSTANCE, abi.PI_INTENT_IDS["ACTIVATE_ELEMENT"], abi.RT_COMMAND)]
    trig = of(e, abi.VT_PROCESS_EVENT, abi.PE_TRIGGERING)[0]
    assert trig.value["scopeKey"] == KEY_A and trig.value["targetElementId"] == "start"
    assert of(e, abi.VT_PROCESS_EVENT, abi.PE_TRIGGERED)[0].key == trig.key
    job = jobs(e)[0]
    e = write(cl, Client.complete_job(job.key))
    log = cl.parts[0].log.entries
    got = [(r.value["bpmnElementType"], abi.PI_INTENTS[r.intent]) for r in log if r.value_type == abi.VT_PROCESS_INSTANCE
           and r.value["processInstanceKey"] == pi.key]
    want = [("PROCESS", "ELEMENT_ACTIVATING"), ("PROCESS", "ELEMENT_ACTIVATED"),
            ("START_EVENT", "ELEMENT_ACTIVATING"), ("START_EVENT", "ELEMENT_ACTIVATED"),
            ("START_EVENT", "COMPLETE_ELEMENT"), ("START_EVENT", "ELEMENT_COMPLETING"),
            ("START_EVENT", "ELEMENT_COMPLETED")]
    assert any(got[i:i + len(want)] == want for i in range(len(got)))  # containsSequence
    assert got[-1] == ("PROCESS", "ELEMENT_COMPLETED")
    state = cl.parts[0].state()
    assert "MESSAGE_START_EVENT_SUBSCRIPTION_BY_NAME_AND_KEY|<default>|a|%d|key=%d,bpmnProcessId=wf,startEventId=start" \
        % (KEY_A, KEY_A) in state
    assert not [r for r in state if r.startswith(("MESSAGE_PROCESSES_ACTIVE", "MESSAGE_PROCESS_INSTANCE_CORRELATION"))]


def test_one_instance_per_correlation_key_then_the_buffered_messages():
    # shouldCreateOnlyOneInstancePerCorrelationKey (:388-423): messages [1, 3] start instances, 2 waits for the
    # key's instance; shouldCreateNewInstanceForBufferedMessageAfterCompletion (:538-578): completing the
    # instance starts the next buffered message's, in publish order; shouldCreateNewInstanceAfterCompletion
    # (:470-504)
    cl = cluster((SINGLE, KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"))
    (m1, p1), = started(e)
    assert "MESSAGE_PROCESSES_ACTIVE_BY_CORRELATION_KEY|wf|key-1" in cl.parts[0].state()
    assert "MESSAGE_PROCESS_INSTANCE_CORRELATION_KEYS|%d|key-1" % p1 in cl.parts[0].state()
    e = write(cl, publish(cl, "a", "key-1"), publish(cl, "a", "key-2"), publish(cl, "a", "key-1"))
    m2, m3, m4 = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    assert [m for m, _ in started(e)] == [m3]
    job1 = [j for j in jobs(cl.parts[0].log.entries) if j.value["processInstanceKey"] == p1][0]
    e = write(cl, Client.complete_job(job1.key))
    (m, p2), = started(e)
    assert m == m2
    # the new instance's lock replaces the old one in the completing batch
    state = cl.parts[0].state()
    assert "MESSAGE_PROCESS_INSTANCE_CORRELATION_KEYS|%d|key-1" % p2 in state
    assert "MESSAGE_PROCESS_INSTANCE_CORRELATION_KEYS|%d|key-1" % p1 not in state
    job2 = [j for j in jobs(e) if j.value["processInstanceKey"] == p2][0]
    e = write(cl, Client.complete_job(job2.key))
    assert [m for m, _ in started(e)] == [m4]
    assert "MESSAGE_CORRELATED|%d|wf" % m2 in cl.parts[0].state()


def test_empty_correlation_key_starts_every_time():
    # shouldCreateMultipleInstancesIfCorrelationKeyIsEmpty (:358-386): no lock without a correlation key
    cl = cluster((SINGLE, KEY_A, 1))
    e = write(cl, publish(cl, "a", ""), publish(cl, "a", ""))
    assert [m for m, _ in started(e)] == [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    assert not [r for r in cl.parts[0].state() if r.startswith("MESSAGE_PROCESSES_ACTIVE")]


def test_buffered_message_after_its_ttl_is_not_correlated():
    # shouldNotCreateNewInstanceForBufferedMessageAfterTTL (:722-765): TTL 10 s and 20 s; 10 s later the
    # instance completes: the second message (deadline == now) is not taken, the third is
    cl = cluster((SINGLE, KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"), publish(cl, "a", "key-1", ttl=10000), publish(cl, "a", "key-1", ttl=20000))
    keys = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    assert [m for m, _ in started(e)] == keys[:1]
    cl.clock.now += 10000
    e = write(cl, Client.complete_job(jobs(e)[0].key))
    assert [m for m, _ in started(e)] == [keys[2]]


def test_multiple_start_events():
    # shouldCreateNewInstanceWithMultipleStartEvents (:258-284), shouldCreateOnlyOneInstancePerCorrelationKey
    # WithMultipleStartEvents (:767-802): the lock is per process, over both start events;
    # shouldCreateNewInstanceForBufferedMessageWithMultipleStartEvents (:804-851): the buffered messages of both
    # names start the next instances in publish order
    cl = cluster((multiple(), KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"), publish(cl, "b", "key-2"))
    assert [m for m, _ in started(e)] == [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    assert [r.value["elementId"] for r in e if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_ACTIVATED and r.value["bpmnElementType"] == "START_EVENT"] == ["start-a", "start-b"]
    cl = cluster((multiple(), KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"), publish(cl, "b", "key-1"), publish(cl, "a", "key-1"),
              publish(cl, "b", "key-1"))
    keys = [r.key for r in of(e, abi.VT_MESSAGE, abi.MSG_PUBLISHED)]
    got = [m for m, _ in started(e)]
    for _ in range(3):
        open_jobs = [j for j in jobs(cl.parts[0].log.entries)
                     if not [c for c in of(cl.parts[0].log.entries, abi.VT_JOB, abi.JOB_COMPLETED) if c.key == j.key]]
        e = write(cl, Client.complete_job(open_jobs[0].key))
        got += [m for m, _ in started(e)]
    assert got == keys


def test_latest_version_only():
    # shouldCreateInstanceOfLatestVersion (:233-256): a second version replaces the first's subscription;
    # shouldCreateNewInstanceOfLatestProcessVersionForBufferedMessage (:681-720): a message buffered while the
    # v1 instance runs starts a v2 instance once it completes
    cl = cluster((single("v1"), KEY_A, 1))
    e = write(cl, publish(cl, "a", "key-1"))
    job = jobs(e)[0]
    cl.parts[0].engine.deploy(single("v2"), KEY_B, 2)
    e = write(cl, publish(cl, "a", "key-1"))
    assert not started(e)
    e = write(cl, Client.complete_job(job.key))
    assert [r.value["elementId"] for r in e if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_ACTIVATED and r.value["bpmnElementType"] == "START_EVENT"] == ["v2"]
    state = cl.parts[0].state()
    assert [r for r in state if r.startswith("MESSAGE_START_EVENT_SUBSCRIPTION_BY_NAME_AND_KEY|")] == \
        ["MESSAGE_START_EVENT_SUBSCRIPTION_BY_NAME_AND_KEY|<default>|a|%d|key=%d,bpmnProcessId=wf,startEventId=v2"
         % (KEY_B, KEY_B)]


def test_start_event_and_catch_event_of_one_publish():
    # MessagePublishProcessor.handleNewMessage (:106-125): one publish correlates to the open subscriptions
    # (CORRELATING) and to the start events of processes it did not correlate to; shouldTriggerOnlyMessage
    # StartEvent (:286-306): a process with a none start event too is started at its message start event
    catch = bpmn.message_catch_process("process", "a", "key", "receive-message")
    both = bpmn.createExecutableProcess("both")
    both.startEvent("none-start").endEvent("end-1")
    both.current = None
    both.startEvent("message-start").message("a").endEvent("end-2")
    cl = cluster((catch, KEY_A, 1), (both.done(), KEY_B, 1))
    write(cl, Client.create("process", (("key", "key-1"),)))
    e = write(cl, publish(cl, "a", "key-1"))
    assert len(of(e, abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CORRELATING)) == 1
    assert len(started(e)) == 1
    assert [r.value["elementId"] for r in e if r.value_type == abi.VT_PROCESS_INSTANCE
            and r.intent == abi.PI_ELEMENT_ACTIVATED and r.value["bpmnElementType"] == "START_EVENT"] == ["message-start"]
    assert len([r for r in e if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
                and r.value["bpmnElementType"] == "PROCESS"]) == 2
