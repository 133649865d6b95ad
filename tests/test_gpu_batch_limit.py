"""Batch limit on the gfx950 path: ProcessingStateMachine.batchProcessing /
collectBatchProcessingStepResult (stream-platform/.../ProcessingStateMachine.java:328-417).  A
follow-up command is processed in its batch only while pending + processed + new <
maxCommandsInBatch; beyond that it is written to the log unprocessed and read back later as a batch
of its own, after the window's commands, in the order written.  The device flags such records
(zbhip_record.unprocessed) and runs them as continuation batches (kernels.hip overflow,
CMD_FOLLOWUP).  Large fan-outs that exceed the LDS FIFO ring spill to the lane's global FIFO.

Bar: records (unprocessed flag and source indices included), rejections and state equal to the
oracle with the same limit (its restatement is pinned on the CPU by
test_oracle_golden.py::test_batch_limit_overflow_goes_to_log)."""
import numpy as np
import pytest

from helpers import complete_commands, create_commands, process_xml
from oracle.oracle import Oracle
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

FIELDS = abi.PARITY_FIELDS


def fork_to_ends(branches, process_id="fanout"):
    """start -> fork(parallel, N out) -> N none end events (no join: N tokens pending at once)."""
    b = bpmn.createExecutableProcess(process_id).startEvent("start").parallelGateway("fork")
    for i in range(1, branches + 1):
        b.moveToNode("fork").sequenceFlowId("f%d" % i).endEvent("end%d" % i)
    return b.done()


def _same(got, want, part, orc):
    assert len(got) == len(want), (len(got), len(want))
    for f in FIELDS:
        if not np.array_equal(got[f], want[f]):
            bad = np.nonzero(got[f] != want[f])[0][:5]
            raise AssertionError("field %s at %s: got %s want %s" % (f, bad, got[f][bad], want[f][bad]))
    for i in np.nonzero(got["record_type"] == abi.RT_REJECTION)[0]:
        assert part.reason(got[i]) == orc.reason(int(i))


def drive(xml, limit, n=24, max_records=512, phases=12):
    part = Partition(max_instances=n, max_commands=64 * n, max_records_per_batch=max_records,
                     max_commands_in_batch=limit)
    orc = Oracle(max_commands_in_batch=limit)
    assert part.deploy(xml) == orc.deploy(xml) == 0
    cmds = create_commands(n)
    unprocessed = 0
    for _ in range(phases):
        part.submit(cmds)
        part.run()
        got = part.drain()
        assert part.fallback() == [], [part.command_status(i) for i in range(len(cmds))][:3]
        orc.clear_records()
        orc.submit(cmds)
        orc.run()
        want = orc.records()
        _same(got, want, part, orc)
        assert part.state() == orc.state()
        unprocessed += int(got["unprocessed"].sum())
        jobs = got[(got["value_type"] == abi.VT_JOB) & (got["intent"] == abi.JOB_CREATED)]
        if len(jobs) == 0:
            break
        pairs = sorted(part.resolve_key(int(k)) for k in jobs["key"])
        cmds = complete_commands([p[0] for p in pairs], [p[1] for p in pairs])
    return unprocessed


@pytest.mark.parametrize("limit", [3, 100])
def test_one_task_batch_limit(limit):
    # the twin of test_oracle_golden.py::test_batch_limit_overflow_goes_to_log (one_task.bpmn)
    got = drive(process_xml({"fixture": "one_task.bpmn"}), limit)
    assert (got > 0) == (limit == 3)


@pytest.mark.parametrize("limit", [3, 5, 100])
def test_linear_batch_limit(limit):
    got = drive(bpmn.linear_process(4), limit)
    assert (got > 0) == (limit == 3)


@pytest.mark.parametrize("limit", [3, 10, 20, 100])
def test_fork_join_12_batch_limit(limit):
    got = drive(bpmn.fork_join_process(12), limit)  # 13 taken-flow counters (<= 16, kJoinWords)
    assert (got > 0) == (limit <= 10)


@pytest.mark.parametrize("limit", [3, 10, 100])
def test_fan_out_beyond_the_lds_ring(limit):
    # 40 tokens pending at once: more than the LDS ring of KGeneric (16), the rest in the global FIFO
    got = drive(fork_to_ends(40), limit)
    assert (got > 0) == (limit < 100)  # the oracle's count: the parity check compares every record


@pytest.mark.parametrize("limit", [4, 100])
def test_fork_join_with_tasks_batch_limit(limit):
    drive(bpmn.fork_join_process(6, tasks=True), limit)


@pytest.mark.parametrize("limit", [16, 17, 100])
def test_fork_join_8_tasks_straight_line_batches(limit):
    # the bench's variant 4b: KGeneric's straight-line CREATE into the fork (limit > 16) and the branch
    # completions into the join, against the general path's records (limit 16: CREATE on the FIFO)
    drive(bpmn.fork_join_process(8, tasks=True), limit)


def boundary_chain(n_tasks):
    b = bpmn.createExecutableProcess("boundaryChain").startEvent("start")
    for i in range(n_tasks):
        b.serviceTask("task%d" % i, "t").boundaryEvent("late%d" % i).timerWithDuration("PT1H")
        b.endEvent("lateEnd%d" % i).moveToActivity("task%d" % i)
    return b.endEvent("end").done()


@pytest.mark.parametrize("limit", [4, 5, 100])
def test_timer_boundary_chain_straight_line_batches(limit):
    # boundary10's shape: KScope's straight-line CREATE and completions (each cancels a timer and
    # creates the next), and the general path at the tight limit
    drive(boundary_chain(4), limit)
