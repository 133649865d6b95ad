"""The oracle's JOB:FAIL (zb_oracle.cpp fail_job) pinned on the reference's own tests: FailJobTest.java
(engine/src/test/.../processing/job/FailJobTest.java:60-265) and JobFailIncidentTest.java
(engine/src/test/.../processing/incident/JobFailIncidentTest.java:112-145), run through the restated
processing loop over the oracle engine (tests/psm.py)."""
from psm import Client, Log, OracleEngine, StreamProcessor, open_jobs
from zeebe_amd import abi, bpmn

KEY = 2251799813685249


def loop(xml=None):
    log = Log()
    eng = OracleEngine()
    eng.deploy(xml or bpmn.linear_process(1, process_id="process", job_type="test"), KEY, 1)
    sp = StreamProcessor(log, [eng])
    return log, eng, sp


def run(log, sp, *recs):
    start = len(log.entries)
    Client(log).write(*recs)
    sp.run()
    return log.entries[start:]


def job_events(entries, intent):
    return [r for r in entries if r.value_type == abi.VT_JOB and r.intent == intent and r.record_type == abi.RT_EVENT]


def test_should_fail():
    # FailJobTest.shouldFail (:60-85): FAILED carries the worker, type, the new retries and the deadline
    log, eng, sp = loop()
    run(log, sp, Client.create("process"))
    batch = run(log, sp, Client.activate_jobs("test", worker="w", timeout=1000, timestamp=5))[-1]
    job_key = batch.value["jobKeys"][0]
    failed = job_events(run(log, sp, Client.fail_job(job_key, 23)), abi.JOB_FAILED)
    assert len(failed) == 1
    v = failed[0].value
    assert (failed[0].key, v["worker"], v["type"], v["retries"], v["deadline"]) == (job_key, "w", "test", 23, 1005)
    assert "JOB_STATES|%d|ACTIVATABLE" % job_key in eng.state()


def test_should_fail_with_message_and_retry():
    # FailJobTest.shouldFailWithMessage (:87-115), shouldFailJobAndRetry (:117-170): the job is activatable
    # again and the next batch activates it, with the retries the failure left
    log, eng, sp = loop()
    run(log, sp, Client.create("process"))
    job_key = run(log, sp, Client.activate_jobs("test"))[-1].value["jobKeys"][0]
    failed = job_events(run(log, sp, Client.fail_job(job_key, 3, "failed job")), abi.JOB_FAILED)[0]
    assert failed.value["errorMessage"] == "failed job" and failed.value["retries"] == 3
    again = run(log, sp, Client.activate_jobs("test"))[-1]
    assert again.intent == 1 and again.value["jobKeys"] == (job_key,) and again.value["jobs"][0]["retries"] == 3
    kinds = [(r.record_type, r.intent) for r in log.entries if r.value_type == abi.VT_JOB]
    assert kinds[:3] == [(abi.RT_EVENT, abi.JOB_CREATED), (abi.RT_COMMAND, abi.JOB_FAIL), (abi.RT_EVENT, abi.JOB_FAILED)]


def test_should_fail_if_job_created_and_reject_the_others():
    # shouldFailIfJobCreated (:208-218), shouldRejectFailIfJobNotFound (:220-231),
    # shouldRejectFailIfJobAlreadyFailed (:233-248), shouldRejectFailIfJobCompleted (:250-265)
    log, eng, sp = loop()
    run(log, sp, Client.create("process"), Client.create("process"))
    a, b = sorted(open_jobs(log))
    assert job_events(run(log, sp, Client.fail_job(a, 0)), abi.JOB_FAILED)
    rej = [r for r in run(log, sp, Client.fail_job(123, 3)) if r.record_type == abi.RT_REJECTION]
    assert rej[0].rejection_type == abi.REJ_NOT_FOUND
    assert rej[0].rejection_reason == "Expected to fail job with key '123', but no such job was found"
    rej = [r for r in run(log, sp, Client.fail_job(a, 3)) if r.record_type == abi.RT_REJECTION]
    assert rej[0].rejection_type == abi.REJ_INVALID_STATE and "it is in state 'FAILED'" in rej[0].rejection_reason
    run(log, sp, Client.complete_job(b))
    rej = [r for r in run(log, sp, Client.fail_job(b, 3)) if r.record_type == abi.RT_REJECTION]
    assert rej[0].rejection_type == abi.REJ_NOT_FOUND
    # a FAILED job cannot be completed or timed out (JobCommandPreconditionChecker / JobTimeOutProcessor)
    rej = [r for r in run(log, sp, Client.complete_job(a)) if r.record_type == abi.RT_REJECTION]
    assert rej[0].rejection_type == abi.REJ_INVALID_STATE and "it is in state 'FAILED'" in rej[0].rejection_reason


def test_incident_if_no_retries_left():
    # JobFailIncidentTest.shouldCreateIncidentIfJobHasNoRetriesLeft (:112-145)
    xml = (bpmn.createExecutableProcess("process").startEvent().serviceTask("failingTask", "test").endEvent().done())
    log, eng, sp = loop(xml)
    run(log, sp, Client.create("process"))
    job_key = sorted(open_jobs(log))[0]
    entries = run(log, sp, Client.fail_job(job_key, 0))
    failed = job_events(entries, abi.JOB_FAILED)[0]
    incident = [r for r in entries if r.value_type == abi.VT_INCIDENT][0]
    task = [r for r in log.entries if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_ACTIVATED
            and r.value["elementId"] == "failingTask"][0]
    assert incident.key > 0 and incident.source_position == failed.source_position
    v = incident.value
    assert (v["errorType"], v["errorMessage"], v["bpmnProcessId"], v["processDefinitionKey"], v["elementId"],
            v["elementInstanceKey"], v["variableScopeKey"], v["jobKey"]) == \
        ("JOB_NO_RETRIES", "No more retries left.", "process", KEY, "failingTask", task.key, task.key, job_key)
    state = eng.state()
    assert "JOB_STATES|%d|FAILED" % job_key in state
    assert "INCIDENT_JOBS|%d|%d" % (job_key, incident.key) in state
    # the job's own message, when it has one
    run(log, sp, Client.create("process"))
    other = max(open_jobs(log))
    inc = [r for r in run(log, sp, Client.fail_job(other, 0, "custom")) if r.value_type == abi.VT_INCIDENT][0]
    assert inc.value["errorMessage"] == "custom"


def test_state_rows_survive_the_zb_db_encoding():
    # the failed job's stored fields and the incident rows as RocksDB bytes (oracle/statedb.py)
    from oracle import statedb as SD
    log, eng, sp = loop()
    run(log, sp, Client.create("process"), Client.create("process"))
    a, b = sorted(open_jobs(log))
    run(log, sp, Client.fail_job(a, 2, "a, b|c"), Client.fail_job(b, 0, "d"))
    rows = eng.state()
    tables, strings = eng.o.process_tables(), eng.o.strings()
    enc = SD.encode_rows(rows, tables, lambda i: strings[i])
    assert {cf for cf, _, _ in enc} >= {16, 17, 34, 36}
    # the state rows come back through the oracle's import (the hand-off's RawDbWriter)
    fresh = OracleEngine()
    fresh.deploy(bpmn.linear_process(1, process_id="process", job_type="test"), KEY, 1)
    fresh.upsert([r for r in rows if not r.startswith("KEY|")])
    assert [r for r in fresh.state() if not r.startswith("KEY|")] == [r for r in rows if not r.startswith("KEY|")]


def test_error_message_limited_in_utf16_code_units():
    # JobFailProcessor.java:42 / failJob: StringUtil.limitString(errorMessage, 10000) (util/.../StringUtil
    # .java:50-56) counts Java chars -- UTF-16 code units, not UTF-8 bytes: a two-byte character is one
    # unit, a character beyond the BMP two; a cut between a surrogate pair leaves a lone high surrogate,
    # which the UTF-8 encoding of the record writes as '?'
    cases = [("é" * 10001, "é" * 10000 + "..."), ("é" * 10000, "é" * 10000),
             ("\U0001D11E" * 5001, "\U0001D11E" * 5000 + "..."), ("a" + "\U0001D11E" * 5000, "a" + "\U0001D11E" * 4999 + "?...")]
    log, eng, sp = loop()
    run(log, sp, *[Client.create("process") for _ in cases])
    jobs = sorted(open_jobs(log))
    for job_key, (msg, want) in zip(jobs, cases):
        failed = job_events(run(log, sp, Client.fail_job(job_key, 1, msg)), abi.JOB_FAILED)[0]
        assert failed.value["errorMessage"] == want
