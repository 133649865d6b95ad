"""Static zeebe:taskHeaders on the device path (ABI 10: zbhip_process_csr.header_begin / header_bytes):
the jobs of a job worker with task headers carry them as customHeaders (BpmnJobBehavior.java:194-248,
365-399) -- in the drained records' values (RecordValues), the host serialiser's log bytes (equal to the
oracle's oracle/logserial.py bytes), the device log writer's bytes (equal to the host's), the zb-db JOBS
values (equal to oracle/statedb.py's encoding) and the restart round trip; the entry order is the Java
HashMap order the compiler and the oracle each restate (tests/test_task_headers.py)."""
import pytest

from helpers import complete_commands, create_commands
from test_gpu_logdev import Log
from test_gpu_logserial import Pair
from zeebe_amd import abi, bpmn
from zeebe_amd.adapter import RecordValues

pytestmark = pytest.mark.gpu

HEADERS = [("z-last", "1"), ("a-first", "2"), ("Aa", "x"), ("BB", "y"), ("workerVersion", "42"),
           ("küche", "ü"), ("long", "v" * 40)]


def process(mi=False):
    b = bpmn.createExecutableProcess("headers").startEvent("s").serviceTask("t1", "job-a")
    for k, v in HEADERS:
        b.zeebeTaskHeader(k, v)
    b.serviceTask("t2", "job-b").zeebeTaskHeader("only", "one")
    if mi:
        b.multiInstance("[1,2,3]")
    return b.serviceTask("t3", "job-c").endEvent("e").done()


@pytest.mark.parametrize("mi", [False, True])
def test_task_headers_in_records_log_bytes_and_state(mi):
    n = 64
    pair = Pair(process(mi), n)
    p = pair.part.processes[0]
    assert dict(p.custom_headers[p.element_ids.index("t1")]) == dict(HEADERS)
    recs = pair.window(create_commands(n, 0))
    values = RecordValues(pair.part.processes, pair.part.name, pair.part.string_value)
    created = [r for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
    assert len(created) == n
    v = values.value(created[0])
    assert dict(v["customHeaders"]) == dict(HEADERS)
    for _ in range(6):  # complete every job, window by window (log bytes and zb-db state checked each time)
        jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
        if not jobs:
            break
        res = [pair.part.resolve_key(k) for k in jobs]
        recs = pair.window(complete_commands([r[0] for r in res], [r[1] for r in res]))
    done = sum(1 for r in recs if r["value_type"] == abi.VT_PROCESS_INSTANCE and r["intent"] == abi.PI_ELEMENT_COMPLETED
               and pair.part.processes[0].element_types[int(r["element_idx"])] == "PROCESS")
    assert done == n


def test_task_headers_in_device_log_bytes():
    n = 200
    log = Log(process(), n)
    recs = log.window(create_commands(n))
    for _ in range(4):
        jobs = [int(r["key"]) for r in recs if r["value_type"] == abi.VT_JOB and r["intent"] == abi.JOB_CREATED]
        if not jobs:
            break
        c = abi.make_commands(len(jobs))
        for i, k in enumerate(jobs):
            c[i]["instance"], c[i]["ref"] = log.part.resolve_key(k)
        c["kind"] = abi.CMD_JOB_COMPLETE
        recs = log.window(c)
    assert log.windows >= 4


def test_task_headers_survive_a_restart():
    # zb-db export of the open jobs (customHeaders from the element) and import into a fresh partition
    from zeebe_amd.engine import Partition
    n = 32
    pair = Pair(process(), n)
    pair.window(create_commands(n, 0))
    rows = pair.part.state_db()
    fresh = Partition(max_instances=n, max_commands=10 * n, max_records_per_batch=64)
    fresh.deploy(process())
    fresh.import_state_db(rows)
    assert fresh.state() == pair.part.state()
    assert fresh.state_db() == rows
    jobs = [(c, k, v) for c, k, v in rows if c == 16]
    assert jobs and all(b"customHeaders\x87" in v or b"customHeaders\x81" in v or b"customHeaders\x80" in v
                        for _, _, v in jobs)
    assert sum(b"workerVersion" in v for _, _, v in jobs) == n
