"""Multi-instance activities as the reference writes them, on the device, in the reference's processing
loop: the inputCollection a list variable (`= items`, ZBHIP_DOC_LIST values from the list dictionary),
an outputCollection collecting an outputElement (the device writes the item and its index, the host
completes the array in log order: runtime.cpp track_mi), and a completionCondition (the FEEL bytecode
with the inner instance's own variables and the body's numberOf* as its primary context).

The workloads of tests/test_oracle_mi_collections.py (pinned there on MultiInstanceActivityTest.java)
run through the loop over the engine alone and over [adapter, engine] at batch limits 3 and 100: every
log (record, key, value -- lists as tuples --, position) and every state row equal.  A satisfied
condition with other inner instances active terminates them on the device (PROCESS_INSTANCE_BATCH
:TERMINATE); a batch past the limit goes to the engine with the instance, through the hand-off's
state rows."""
import numpy as np
import pytest

from psm import Client, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, check, single, write
from test_oracle_mi_collections import ITEMS, RESULTS, process
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu
MODES = [("parallel", False), ("sequential", True)]


def complete_jobs(ref, gpu, count, results=RESULTS, job_type="task"):
    """completeJobs (MultiInstanceActivityTest.java:1579-1613): one job activated at a time (the results
    taken in turn), until `count` or no job is left (the logs compared at each step)."""
    for i in range(count):
        write(ref, gpu, Client.activate_jobs(job_type, max_jobs=1, timestamp=ref.clock.now))
        batch = [r for r in gpu.parts[0].log.entries if r.value_type == abi.VT_JOB_BATCH][-1]
        if not batch.value["jobKeys"]:
            return i
        assert len(batch.value["jobKeys"]) == 1, "job %d" % i
        write(ref, gpu, Client.complete_job(batch.value["jobKeys"][0], (("result", results[i % len(results)]),)))
    return count


def variables(gpu, name):
    return [r.value["value"] for r in gpu.parts[0].log.entries if r.value_type == abi.VT_VARIABLE
            and r.value["name"] == name]


@pytest.mark.parametrize("limit", [100, 3])
@pytest.mark.parametrize("mode,seq", MODES)
def test_collections_in_the_processing_loop(mode, seq, limit):
    xml = process(seq)
    ref, gpu = single([(xml, KEY_A, 1)], [(xml, KEY_A, 1)], limit=limit)
    write(ref, gpu, Client.create("process", (("items", ITEMS),)), Client.create("process", (("items", (5,)),)),
          Client.create("process", (("items", ()),)))
    complete_jobs(ref, gpu, 4)
    assert [v for v in variables(gpu, "results") if len(v) == 3 and None not in v]
    ad = gpu.parts[0].adapter
    assert ad.counts["device_commands"] > 0
    check(ref, gpu)


@pytest.mark.parametrize("mode,seq", MODES)
@pytest.mark.parametrize("elem", ["= item", "= loopCounter"])
def test_output_element_forms(mode, seq, elem):
    xml = process(seq, outputElement=elem)
    ref, gpu = single([(xml, KEY_A, 1)], [(xml, KEY_A, 1)])
    write(ref, gpu, *[Client.create("process", (("items", ITEMS),)) for _ in range(3)])
    complete_jobs(ref, gpu, 9)
    check(ref, gpu)


@pytest.mark.parametrize("mode,seq", MODES)
@pytest.mark.parametrize("cond,jobs", [("= item = 20", 2), ("= numberOfCompletedInstances >= 2", 2),
                                       ("= result > 20", 2), ("= false", 3)])
def test_completion_conditions(mode, seq, cond, jobs):
    xml = process(seq, completionCondition=cond)
    ref, gpu = single([(xml, KEY_A, 1)], [(xml, KEY_A, 1)])
    write(ref, gpu, *[Client.create("process", (("items", ITEMS),)) for _ in range(2)])
    complete_jobs(ref, gpu, 2 * jobs)
    live = sorted(open_jobs(ref.parts[0].log))
    write(ref, gpu, *[Client.complete_job(k, (("result", 1),)) for k in live])
    check(ref, gpu)
    ad = gpu.parts[0].adapter
    # the parallel form of a satisfied condition terminates the other inner instances on the device
    # (PROCESS_INSTANCE_BATCH:TERMINATE)
    assert ad.counts["fallbacks"] == 0, ad.fallback_reasons


def test_restart_keeps_the_collections():
    """The state rows of list variables, inner instances' own variables and a body's outputCollection
    come back through the import (zbhip_import_state_db) and the run goes on."""
    xml = process(False)
    ref, gpu = single([(xml, KEY_A, 1)], [(xml, KEY_A, 1)])
    write(ref, gpu, *[Client.create("process", (("items", ITEMS),)) for _ in range(3)])
    complete_jobs(ref, gpu, 4)
    from zeebe_amd.engine import Partition
    part = gpu.parts[0].adapter.part
    fresh = Partition(max_instances=256, max_commands=48)
    fresh.deploy(xml, process_definition_key=KEY_A)
    fresh.import_state_db(part.state_db())
    assert fresh.state() == part.state()
    assert any("type=6" in r for r in part.state())


def test_random_collections():
    """Several processes of list collections side by side (static lists, list variables, outputs and
    conditions), jobs completed in a seeded random order."""
    procs = [(process(False), KEY_A, 1),
             (bpmn.createExecutableProcess("p2").startEvent().serviceTask("t", "t2")
              .multiInstance("= [1, 2, 3, 4]", "x", True, outputCollection="out", outputElement="= x",
                             completionCondition="= x >= 3").endEvent().done(), KEY_B, 1)]
    ref, gpu = single(procs, procs)
    rng = np.random.default_rng(11)
    creates = [Client.create("process", (("items", tuple(int(v) for v in rng.integers(0, 100, rng.integers(0, 5)))),))
               for _ in range(6)] + [Client.create("p2") for _ in range(4)]
    write(ref, gpu, *creates)
    for _ in range(12):
        live = sorted(open_jobs(ref.parts[0].log))
        if not live:
            break
        rng.shuffle(live)
        write(ref, gpu, *[Client.complete_job(k, (("result", int(rng.integers(0, 50))),)) for k in live[:3]])
    check(ref, gpu)


def test_output_collections_of_one_name_in_sequence():
    """Two multi-instance activities one after the other collecting into the same outputCollection:
    the second body's propagateVariable finds the first's array in the process instance's scope and
    updates it (VARIABLE:UPDATED -- mergeDocument, VariableBehavior.java:105-150) when the arrays differ
    (lengths 3 and 2 here); direct parity with the oracle, no fallback."""
    from test_gpu_parity import run_both
    from helpers import complete_commands, create_commands
    from oracle.oracle import Oracle
    from zeebe_amd.engine import Partition
    b = bpmn.createExecutableProcess("process").startEvent("s")
    b.serviceTask("a", "a").multiInstance("= [1, 2, 3]", "x", True, outputCollection="out", outputElement="= x")
    b.serviceTask("b", "b").multiInstance("= [7, 8]", "x", False, outputCollection="out", outputElement="= loopCounter")
    xml = b.endEvent("e").done()
    n = 8
    part, orc = Partition(max_instances=n, max_commands=n, max_records_per_batch=128), Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    run_both(part, orc, create_commands(n, 0))
    for _ in range(6):
        keys = sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))
        if not keys:
            break
        by = {}
        for k in keys:
            inst, ordv = part.resolve_key(k)
            by.setdefault(inst, ordv)
        insts = sorted(by)
        run_both(part, orc, complete_commands(insts, [by[i] for i in insts]))
        assert part.state() == orc.state()
    assert part.stats()["fallback"] == 0
    assert [r for r in part.state() if not r.startswith("KEY|")] == []
