"""Multi-instance activities on the gfx950 path (KScope) against the CPU oracle
(pinned on MultiInstanceActivityTest by tests/test_oracle_multi_instance.py): parallel and sequential
bodies over static collections of integers and strings, with and without an inputElement, job worker
and undefined-task inner activities, inside a sub-process, batch limits 3 and 100, job activation
(the loop variables in the activated job's document), export -> import -> continue, and the fallback
of a job document that names an inner instance's own loop variable.

Bar: records (every parity field: the loop variables' inline values, the batch command's index,
unprocessed flags) and exported state (the body's childCount / childActivatedCount /
childCompletedCount / multiInstanceLoopCounter, the inner instances' loop counters and loop
variables) equal to the oracle after every window."""
import numpy as np
import pytest

from helpers import create_commands
from oracle.oracle import Oracle
from test_gpu_batch_limit import drive as drive_limit
from test_gpu_import import _continue, _restart, _same
from test_gpu_parity import drive, open_job_completions, run_both
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu


def _in_sub(seq):
    b = bpmn.createExecutableProcess("process").startEvent("s").subProcess("sub").startEvent("ss")
    b.serviceTask("task", "task").multiInstance("= [1, 2, 3]", "item", seq)
    return b.endEvent("se").subProcessDone().serviceTask("after", "after").endEvent("e").done()


SHAPES = {
    "parallel": lambda: bpmn.multi_instance_process((10, 20, 30)),
    "sequential": lambda: bpmn.multi_instance_process((10, 20, 30), sequential=True),
    "parallel_no_input": lambda: bpmn.multi_instance_process((1, 2), input_element=None),
    "sequential_strings": lambda: bpmn.multi_instance_process(("a", "bb", "ccc", "d"), sequential=True),
    "parallel_mixed_after": lambda: bpmn.multi_instance_process((7, "x", True, None), after="after"),
    "parallel_empty": lambda: bpmn.multi_instance_process(()),
    "sequential_one": lambda: bpmn.multi_instance_process((5,), sequential=True, after="after"),
    "parallel_undefined": lambda: bpmn.multi_instance_process((1, 2, 3), inner="task", after="after"),
    "sequential_undefined": lambda: bpmn.multi_instance_process((1, 2, 3), sequential=True, inner="manualTask"),
    "parallel_in_sub": lambda: _in_sub(False),
    "sequential_in_sub": lambda: _in_sub(True),
    "parallel_six": lambda: bpmn.multi_instance_process(tuple(range(6))),
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_gpu_multi_instance_parity(shape):
    part, orc = drive(SHAPES[shape](), 200, phases=30, rng_seed=11, max_records=128)
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
    assert part.stats()["fallback"] == 0


@pytest.mark.parametrize("seq", [False, True])
@pytest.mark.parametrize("limit", [3, 100])
def test_gpu_multi_instance_batch_limit(seq, limit):
    # every open job of every instance completed in each window; with a limit of 3 the inner
    # activations / the batch command go past it and run as continuation batches
    unprocessed = drive_limit(bpmn.multi_instance_process((10, 20, 30, 40), sequential=seq, after="after"), limit,
                              n=24, phases=20)
    assert (unprocessed > 0) == (limit == 3)


def test_gpu_multi_instance_mid_window_state():
    # the state between windows: bodies with children active and completed, inner instances with
    # their loop variables, jobs ACTIVATABLE
    part, orc = drive(bpmn.multi_instance_process((3, 1, 4, 1, 5)), 50, phases=2, rng_seed=3)
    st = part.state()
    body = [r for r in st if "bpmnElementType=19," in r]
    assert body and all("childActivatedCount=5" in r and "multiInstanceLoopCounter=5" in r for r in body)
    assert any(r.startswith("VARIABLES|") and "|loopCounter|" in r for r in st)


@pytest.mark.parametrize("seq", [False, True])
def test_gpu_multi_instance_job_activation(seq):
    # shouldSetInputElementVariable (:491-523): the activated jobs carry item and loopCounter (the
    # inner scope first, then the process instance's variables, DbString order)
    xml = bpmn.multi_instance_process((10, 20, 30), sequential=seq, job_type="mi")
    part = Partition(max_instances=8, max_commands=8, max_records_per_batch=128)
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    amount = part.intern("amount")
    assert orc.intern("amount") == amount
    d = abi.make_docs(4)
    d["name_id"], d["type"], d["value"] = amount, abi.DOC_INT, [5, 6, 7, 8]
    c = create_commands(4)
    c["doc_count"], c["doc_begin"] = 1, np.arange(4)
    run_both(part, orc, c, d)
    for step in range(4):
        got = part.activate_jobs("mi", max_jobs=3, timestamp=1000 + step)
        want = orc.activate_jobs("mi", max_jobs=3, timestamp=1000 + step)
        assert got[0] == want[0] and got[2] == want[2]
        assert len(got[1]) == len(want[1]) > 0
        for g, w in zip(got[1], want[1]):
            for f in ("key", "element_instance_key", "process_instance_key", "deadline", "n_variables"):
                assert g[f] == w[f], f
            n = int(g["n_variables"])
            assert [tuple(v) for v in g["variables"][:n][["name_id", "type", "value"]]] == \
                   [tuple(v) for v in w["variables"][:n][["name_id", "type", "value"]]]
        assert part.state() == orc.state()
        # complete what was activated (the sequential body then creates its next job)
        cmds = abi.make_commands(len(got[1]))
        for i, j in enumerate(got[1]):
            cmds[i]["instance"], cmds[i]["ref"] = part.resolve_key(int(j["key"]))
        cmds["kind"] = abi.CMD_JOB_COMPLETE
        run_both(part, orc, cmds)
        assert part.state() == orc.state()


@pytest.mark.parametrize("seq", [False, True])
def test_gpu_multi_instance_export_import_continue(seq):
    n = 48
    xml = bpmn.multi_instance_process((10, "twenty", 30), sequential=seq, after="after")
    rng = np.random.default_rng(5)
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=128)
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    run_both(part, orc, create_commands(n))
    c = open_job_completions(part, rng)
    run_both(part, orc, c)
    assert part.state() == orc.state()
    fresh, loaded = _restart(part, xml, n, [], 128)
    assert loaded == n
    _continue([part, fresh], orc, rng, 40)


def test_gpu_multi_instance_loop_variable_document_falls_back():
    # a job completed with a variable named like the inner instance's inputElement updates that local
    # variable (mergeDocument finds it in the inner scope): outside the device's derived loop variables,
    # the command falls back (FB_DOC) and the CPU engine runs it
    xml = bpmn.multi_instance_process((10, 20), sequential=True)
    part = Partition(max_instances=2, max_commands=4, max_records_per_batch=128)
    part.deploy(xml)
    item = part.intern("item")
    part.submit(create_commands(1))
    part.run()
    recs = part.drain()
    job = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB][0]
    c = abi.make_commands(1)
    c[0]["instance"], c[0]["ref"] = part.resolve_key(job)
    c["kind"], c["doc_count"] = abi.CMD_JOB_COMPLETE, 1
    d = abi.make_docs(1)
    d["name_id"], d["type"], d["value"] = item, abi.DOC_INT, 99
    part.submit(c, d)
    part.run()
    assert part.fallback() == [0] and part.command_status(0)[1] == "doc"


@pytest.mark.parametrize("shape", ["parallel", "sequential_strings", "parallel_mixed_after", "sequential_undefined"])
def test_gpu_multi_instance_log_and_db_bytes(shape):
    # host serialiser over the drained records (PROCESS_INSTANCE_BATCH values, inline loop-variable
    # values) == oracle/logserial.py; zb-db bytes of the state (body counters) == oracle/statedb.py
    from test_gpu_logserial import Pair
    from test_gpu_logserial import drive as drive_log
    drive_log(Pair(SHAPES[shape](), 60), 60)
