"""Message boundary events on the gfx950 executor (KMsg) against the oracle cluster -- interrupting:
the subscription opened with the job worker task, then the message first (PROCESS_MESSAGE_SUBSCRIPTION
:CORRELATE terminates the task -- JOB:CANCELED -- and activates the boundary event) or the job first
(the task's unsubscribeFromEvents: PROCESS_MESSAGE_SUBSCRIPTION:DELETING, MESSAGE_SUBSCRIPTION:DELETE /
DELETED on the message partition, PROCESS_MESSAGE_SUBSCRIPTION:DELETE / DELETED back on the PI
partition, also after the instance ended).  Bar as for config 5: every window's records (all parity
fields), outbox entries and exported state bit-exact, at P = 1 and P = 3.  The oracle's lifecycles
are pinned on MessageCatchElementTest / BoundaryEventTest (tests/test_oracle_message_boundary.py).
Non-interrupting ones (NON_INT_BOUNDARY_EVENT_PROCESS): every message activates the boundary event while
the task stays, both subscriptions stay open with the last message key in their records, and the
job's completion closes them."""
import numpy as np
import pytest

from helpers import MessageCluster, OracleAdapter
from oracle.oracle import Oracle, subscription_partition
from test_gpu_messages import GpuAdapter, assert_same_logs, assert_same_state
from test_oracle_message_boundary import job_completions, keys
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

XML = bpmn.message_boundary_process()


NON_INT = bpmn.message_boundary_process("nonIntBoundaryEventProcess", interrupting=False)


def clusters(P, n_inst, xml=XML):
    gpu = MessageCluster([Partition(partition_id=p, partition_count=P, max_instances=n_inst, max_commands=4 * n_inst,
                                    max_correlation_keys=4 * n_inst * P, max_records_per_batch=256)
                          for p in range(1, P + 1)], GpuAdapter, xml)
    orc = MessageCluster([Oracle(partition_id=p, partition_count=P) for p in range(1, P + 1)], OracleAdapter, xml)
    return gpu, orc


def start(gpu, orc, P, n):
    ks = keys(P, n)
    for cl in (gpu, orc):
        ids = cl.intern_keys(ks)
        cl.create(n, [ids[(p - 1) * n:p * n] for p in range(1, P + 1)])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)  # PROCESS_SUBSCRIPTION_BY_KEY OPENED, MESSAGE_SUBSCRIPTION rows, EVENT_SCOPE
    return ks, ids


@pytest.mark.parametrize("P", [1, 3])
def test_gpu_message_first(P):
    n = 24
    gpu, orc = clusters(P, n)
    ks, ids = start(gpu, orc, P, n)
    for cl in (gpu, orc):
        cl.publish(ids, [subscription_partition(k, P) for k in ks])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    canceled = sum(int(np.sum((r["value_type"] == abi.VT_JOB) & (r["intent"] == abi.JOB_CANCELED))) for _, _, r, _ in gpu.log)
    assert canceled == n * P


@pytest.mark.parametrize("P", [1, 3])
def test_gpu_job_first(P):
    n = 24
    gpu, orc = clusters(P, n)
    start(gpu, orc, P, n)
    cmds = job_completions(orc, n)
    for cl in (gpu, orc):
        cl.commands("complete", cmds)
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)  # every subscription deleted on both sides
    deleted = sum(int(np.sum((r["value_type"] == abi.VT_PROCESS_MESSAGE_SUBSCRIPTION) & (r["intent"] == abi.PMS_DELETED)))
                  for _, _, r, _ in gpu.log)
    assert deleted == n * P


def test_gpu_closing_subscription_state():
    # P = 3, the PI partition's window alone: the subscriptions of the ended instances are CLOSING
    # (exported from the device slot rows of instances that are gone), then the exchange deletes them
    P, n = 3, 16
    gpu, orc = clusters(P, n)
    start(gpu, orc, P, n)
    cmds = job_completions(orc, n)
    outs = []
    for cl in (gpu, orc):
        outs.append(cl._run("complete", 1, cmds[0]))
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    assert any("state=CLOSING" in r for r in gpu.parts[0].state())
    for cl, ob in zip((gpu, orc), outs):
        cl.exchange("close", [ob] + [abi.make_xparts(0) for _ in range(P - 1)])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    assert not any("state=CLOSING" in r for r in gpu.parts[0].state())


@pytest.mark.parametrize("P", [1, 3])
def test_gpu_mixed_outcomes(P):
    # half the instances get their message, the other half complete their job, in the same windows
    n = 32
    gpu, orc = clusters(P, n)
    ks, ids = start(gpu, orc, P, n)
    half = list(range(0, n, 2))
    cmds = job_completions(orc, n, which=half)
    for cl in (gpu, orc):
        cl.commands("complete", cmds)
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    rest = [(k, i) for k, i, j in zip(ks, ids, range(len(ks))) if (j % n) % 2 == 1]
    for cl in (gpu, orc):
        cl.publish([i for _, i in rest], [subscription_partition(k, P) for k, _ in rest])
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)


@pytest.mark.parametrize("P", [1, 3])
def test_gpu_non_interrupting_boundary(P):
    # two messages per instance (the boundary event activated twice, the task kept), then the jobs;
    # the state between the steps carries the open subscriptions with their last message key
    n = 24
    gpu, orc = clusters(P, n, NON_INT)
    ks, ids = start(gpu, orc, P, n)
    for _ in range(2):
        for cl in (gpu, orc):
            cl.publish(ids, [subscription_partition(k, P) for k in ks])
        assert_same_logs(gpu, orc)
        assert_same_state(gpu, orc)
    assert any("messageKey=-1" not in r for r in gpu.parts[0].state() if r.startswith("PROCESS_SUBSCRIPTION_BY_KEY"))
    cmds = job_completions(orc, n)
    for cl in (gpu, orc):
        cl.commands("complete", cmds)
    assert_same_logs(gpu, orc)
    assert_same_state(gpu, orc)
    done = sum(int(np.sum((r["value_type"] == abi.VT_PROCESS_INSTANCE) & (r["intent"] == abi.PI_ELEMENT_COMPLETED)
                          & (r["element_idx"] == 0))) for _, _, r, _ in gpu.log)
    assert done == n * P
    assert not [r for p in gpu.parts for r in p.state() if not r.startswith(("KEY|", "MESSAGE_STATS"))]
