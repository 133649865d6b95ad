"""The reference cluster of tests/test_gpu_psm_messages.py on the CPU: three partitions, each
ProcessingStateMachine (tests/psm.py) over the oracle engine, commands between partitions through
InterPartitionCommandSender -- pinned on MessageCorrelationMultiplePartitionsTest.java:74-118
(shouldOpenMessageSubscriptionsOnDifferentPartitions: MESSAGE_SUBSCRIPTION:CREATED of a key only on its
subscription partition) and on App. A.5's protocol (every subscription opened on both sides, every
instance correlated and completed, the acknowledgements closing both sides)."""
from test_gpu_psm_messages import CORRELATION_KEYS, KEYS, P, Cluster, create_phase
from oracle.oracle import subscription_partition
from psm import Client, run_cluster
from zeebe_amd import abi


def count(cl, vt, intent, rt=abi.RT_EVENT):
    return {p: sum(1 for r in cl.logs[p].entries if r.value_type == vt and r.intent == intent and r.record_type == rt)
            for p in range(1, P + 1)}


def test_reference_cluster_pins():
    ref = Cluster(device=False)
    for p, recs in create_phase():
        Client(ref.logs[p]).write(*recs)
    run_cluster(ref.sps)
    created = [(p, r.value["correlationKey"]) for p in range(1, P + 1) for r in ref.logs[p].entries
               if r.value_type == abi.VT_MESSAGE_SUBSCRIPTION and r.record_type == abi.RT_EVENT and r.intent == abi.MS_CREATED]
    assert len(created) == 30 and {(p, k) for p, k in created if k.startswith("item")} == set(CORRELATION_KEYS.items())
    assert all(p == subscription_partition(k, P) for p, k in created)
    assert count(ref, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CREATED) == {1: 10, 2: 10, 3: 10}
    # the open commands crossed partitions as commands with key -1 (TestInterPartitionCommandSender)
    received = [r for p in range(1, P + 1) for r in ref.logs[p].entries
                if r.record_type == abi.RT_COMMAND and r.value_type == abi.VT_MESSAGE_SUBSCRIPTION
                and r.intent == abi.MS_CREATE and r.source_position < 0]
    local = sum(1 for p, recs in create_phase() for r in recs
                if subscription_partition(r.value["variables"][0][1], P) == p)
    assert 0 < local < 30 and len(received) == 30 - local and all(r.key == -1 for r in received)
    for k in KEYS:
        Client(ref.logs[subscription_partition(k, P)]).write(*[Client.publish_message("message", k) for _ in range(3)])
    run_cluster(ref.sps)
    by_part = {p: 3 * sum(1 for k in KEYS if subscription_partition(k, P) == p) for p in range(1, P + 1)}
    assert count(ref, abi.VT_MESSAGE_SUBSCRIPTION, abi.MS_CORRELATED) == by_part
    assert count(ref, abi.VT_PROCESS_MESSAGE_SUBSCRIPTION, abi.PMS_CORRELATED) == {1: 10, 2: 10, 3: 10}
    done = sum(1 for p in range(1, P + 1) for r in ref.logs[p].entries
               if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == 5 and r.value["bpmnElementType"] == "PROCESS")
    assert done == 30
    # no subscription is left on either side
    for p in range(1, P + 1):
        assert not [r for r in ref.engines[p].state() if "SUBSCRIPTION" in r.split("|")[0]]
