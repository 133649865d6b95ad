"""Config 5 through the drop-in boundary inside the reference's processing loop, on three partitions.

Every partition runs ProcessingStateMachine (tests/psm.py) over its own log; the reference cluster runs
[engine] on each, the device cluster [GpuBatchProcessor (zeebe_amd/adapter.py), engine].  Commands a
batch sends to another partition (SubscriptionCommandSender.handleFollowUpCommandBasedOnPartition,
:320-338) are written to the receiver's log after the batch is committed, by the test form of
InterPartitionCommandSender (TestInterPartitionCommandSender.java:23-59).  The bar: every partition's
log -- every record, position, source position and processed flag -- and every partition's state equal
the reference cluster's.

Workload: MessageCorrelationMultiplePartitionsTest.java:36-40,57-175 -- correlation keys "item-2",
"item-1", "item-0" whose subscription partitions are 1, 2, 3 (SubscriptionUtil), instances created on
every partition with every key (remote and local subscriptions), then messages published on each
key's partition until every instance is correlated (time-to-live 0: one subscription per publish)."""
import pytest

from psm import Client, InterPartitionCommandSender, Log, OracleEngine, StreamProcessor, run_cluster
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import GpuBatchProcessor

pytestmark = pytest.mark.gpu

P = 3
KEY = 2251799813685249
CORRELATION_KEYS = {1: "item-2", 2: "item-1", 3: "item-0"}  # MessageCorrelationMultiplePartitionsTest.java:36-40
XML = bpmn.message_catch_process(message_name="message", correlation_key="key", catch_id="receive-message")


class Cluster:
    def __init__(self, device, limit=100, window=48, xml=XML):
        self.logs = {p: Log() for p in range(1, P + 1)}
        sender = InterPartitionCommandSender(self.logs)
        self.engines, self.adapters, self.sps = {}, {}, []
        for p in range(1, P + 1):
            eng = OracleEngine(partition_id=p, partition_count=P, max_commands_in_batch=limit, command_sender=sender)
            eng.deploy(xml, KEY, 1)
            procs = [eng]
            if device:
                ad = GpuBatchProcessor(eng, self.logs[p].reader(), [(xml, KEY, 1)], zeebe_db=eng, key_generator=eng,
                                       partition_id=p, partition_count=P, instances=256, window=window,
                                       max_commands_in_batch=limit, correlation_keys=64, command_sender=sender)
                ad.init()
                self.adapters[p] = ad
                procs = [ad, eng]
            self.engines[p] = eng
            self.sps.append(StreamProcessor(self.logs[p], procs, limit))

    def state(self, p):
        eng = self.engines[p]
        if p not in self.adapters:
            return eng.state()
        part = self.adapters[p].part
        dev = [r for r in part.state() if not r.startswith("KEY|")]
        assert part.current_key() <= eng.current_key()  # one key generator per partition
        return sorted(dev + eng.state())


def phase(ref, gpu, writes):
    for p, recs in writes:
        Client(ref.logs[p], gpu.logs[p]).write(*recs)
    run_cluster(ref.sps)
    try:
        run_cluster(gpu.sps)
    except Exception as e:
        raise AssertionError("device fallbacks %s" % {p: a.fallback_reasons for p, a in gpu.adapters.items()}) from e
    for p in range(1, P + 1):
        want, got = ref.logs[p].canonical(), gpu.logs[p].canonical()
        if got != want:
            n = min(len(got), len(want))
            bad = next((i for i in range(n) if got[i] != want[i]), n)
            raise AssertionError("partition %d log entry %d of %d/%d:\n got  %s\n want %s" % (
                p, bad, len(got), len(want), got[bad] if bad < len(got) else None, want[bad] if bad < len(want) else None))
        assert gpu.state(p) == sorted(ref.state(p)), p


# three subscribers per key (the device keeps 4 MESSAGE_SUBSCRIPTION rows per correlation key,
# zb_internal.h kSubs): the test's keys plus seven more spread over the partitions
KEYS = [CORRELATION_KEYS[1], CORRELATION_KEYS[2], CORRELATION_KEYS[3]] + ["order-%d" % j for j in range(7)]


def create_phase(process_id="process"):
    """30 instances, 3 per correlation key, every partition creating instances of keys of every
    partition (local and remote subscriptions): instance i on partition 1 + (i + i // 10) % 3 with key
    KEYS[i % 10]."""
    creates = {p: [] for p in range(1, P + 1)}
    for i in range(30):
        creates[1 + (i + i // 10) % 3].append(Client.create(process_id, (("key", KEYS[i % 10]),)))
    return sorted(creates.items())


def test_message_correlation_on_three_partitions_in_the_processing_loop():
    ref, gpu = Cluster(device=False), Cluster(device=True)
    phase(ref, gpu, create_phase())
    # shouldOpenMessageSubscriptionsOnDifferentPartitions: MESSAGE_SUBSCRIPTION:CREATED of key k only on
    # its subscription partition
    for cl in (ref, gpu):
        created = [(p, r.value["correlationKey"]) for p in range(1, P + 1) for r in cl.logs[p].entries
                   if r.value_type == abi.VT_MESSAGE_SUBSCRIPTION and r.record_type == abi.RT_EVENT
                   and r.intent == abi.MS_CREATED]
        assert len(created) == 30
        assert {(p, k) for p, k in created if k.startswith("item")} == set(CORRELATION_KEYS.items())
    # a message nobody waits for (published and expired), then one message per subscription, each on
    # its key's subscription partition (SubscriptionUtil.getSubscriptionPartitionId)
    from oracle.oracle import subscription_partition
    # (the commands carry a broker timestamp: MESSAGE records' deadline = timestamp + timeToLive,
    # MessagePublishProcessor.java:110)
    pubs = {p: [Client.publish_message("message", "nobody", timestamp=1700000000000 + p)] for p in range(1, P + 1)}
    for j, k in enumerate(KEYS):
        pubs[subscription_partition(k, P)] += [Client.publish_message("message", k, timestamp=1700000000100 + 7 * j + n)
                                               for n in range(3)]
    phase(ref, gpu, sorted(pubs.items()))
    published = [r for p in range(1, P + 1) for r in gpu.logs[p].entries
                 if r.value_type == abi.VT_MESSAGE and r.intent == abi.MSG_PUBLISHED]
    assert len(published) == 33 and all(r.value["deadline"] >= 1700000000000 for r in published)
    done = sum(1 for p in range(1, P + 1) for r in gpu.logs[p].entries
               if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == 5
               and r.value["bpmnElementType"] == "PROCESS")
    assert done == 30
    c = [gpu.adapters[p].counts for p in range(1, P + 1)]
    assert all(x["fallbacks"] == 0 for x in c), [gpu.adapters[p].fallback_reasons for p in range(1, P + 1)]
    assert sum(x["device_commands"] for x in c) >= 30 + 3 * 11 + 2 * 30  # creates, publishes, received commands


BOUNDARY_XML = bpmn.message_boundary_process(message_name="message", correlation_key="key")


def test_message_boundary_events_on_three_partitions_in_the_processing_loop():
    """Interrupting message boundary events (MessageCatchElementTest's BOUNDARY_EVENT_PROCESS) in the
    loop: the jobs of half the correlation keys' instances complete first -- their subscriptions close
    through PROCESS_MESSAGE_SUBSCRIPTION:DELETING, MESSAGE_SUBSCRIPTION:DELETE / DELETED and
    PROCESS_MESSAGE_SUBSCRIPTION:DELETE / DELETED across the partitions, some after the instance ended --
    then messages for the other half's keys terminate their tasks (JOB:CANCELED) through the boundary
    event."""
    from psm import open_jobs
    from oracle.oracle import subscription_partition
    ref, gpu = Cluster(device=False, xml=BOUNDARY_XML), Cluster(device=True, xml=BOUNDARY_XML)
    phase(ref, gpu, create_phase("boundaryEventProcess"))
    job_first = set(KEYS[0::2])
    jobs = {}
    for p in range(1, P + 1):
        keys_of = {r.value["processInstanceKey"]: str(r.value["value"]).strip('"') for r in ref.logs[p].entries
                   if r.value_type == abi.VT_VARIABLE and r.record_type == abi.RT_EVENT and r.value["name"] == "key"}
        jobs[p] = [Client.complete_job(k) for k, r in sorted(open_jobs(ref.logs[p]).items())
                   if keys_of.get(r.value["processInstanceKey"]) in job_first]
    phase(ref, gpu, sorted(jobs.items()))
    for cl in (ref, gpu):
        deleted = sum(1 for p in range(1, P + 1) for r in cl.logs[p].entries
                      if r.value_type == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION and r.intent == abi.PMS_DELETED)
        assert deleted == 15
    pubs = {p: [] for p in range(1, P + 1)}
    for k in KEYS[1::2]:
        pubs[subscription_partition(k, P)] += [Client.publish_message("message", k) for _ in range(3)]
    phase(ref, gpu, sorted(pubs.items()))
    canceled = sum(1 for p in range(1, P + 1) for r in gpu.logs[p].entries
                   if r.value_type == abi.VT_JOB and r.intent == abi.JOB_CANCELED)
    assert canceled == 15
    c = [gpu.adapters[p].counts for p in range(1, P + 1)]
    assert all(x["fallbacks"] == 0 for x in c), [gpu.adapters[p].fallback_reasons for p in range(1, P + 1)]


NON_INT_XML = bpmn.message_boundary_process("nonIntBoundaryEventProcess", message_name="message", correlation_key="key",
                                            interrupting=False)


def test_non_interrupting_message_boundary_events_in_the_processing_loop():
    """Non-interrupting message boundary events (NON_INT_BOUNDARY_EVENT_PROCESS) on three partitions:
    each key gets three messages -- every one activates the boundary event again while the task stays
    (both subscriptions open, their records holding the last message key) -- then every job completes
    and closes its subscription; logs and state equal the engine-only cluster's at every phase."""
    from psm import open_jobs
    from oracle.oracle import subscription_partition
    ref, gpu = Cluster(device=False, xml=NON_INT_XML), Cluster(device=True, xml=NON_INT_XML)
    phase(ref, gpu, create_phase("nonIntBoundaryEventProcess"))
    pubs = {p: [] for p in range(1, P + 1)}
    for k in KEYS:
        pubs[subscription_partition(k, P)] += [Client.publish_message("message", k) for _ in range(3)]
    phase(ref, gpu, sorted(pubs.items()))
    jobs = {p: [Client.complete_job(k) for k in sorted(open_jobs(ref.logs[p]))] for p in range(1, P + 1)}
    phase(ref, gpu, sorted(jobs.items()))
    boundary = [sum(1 for p in range(1, P + 1) for r in cl.logs[p].entries
                    if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
                    and r.value["elementId"] == "boundary") for cl in (ref, gpu)]
    assert boundary[0] == boundary[1] > len(KEYS)  # (a message meeting a CORRELATING subscription skips it)
    c = [gpu.adapters[p].counts for p in range(1, P + 1)]
    assert all(x["fallbacks"] == 0 for x in c), [gpu.adapters[p].fallback_reasons for p in range(1, P + 1)]
