"""Multi-entry variable documents on the device (merge order: tests/test_documents.py, parity unpinned
against the reference itself -- agrona's Int2IntHashMap iteration, restated by the oracle).  Creations
and job completions carrying documents of two to four entries -- new variables, updates, equal values,
strings, decimals, lists, entries off their home slot -- through the processing loop over the engine
alone and through [adapter, engine], every log and state equal at batch limits 3 and 100; the device
takes them (no declines), except the shapes outside its subset, which hand their instance to the engine:
a removal from a document with an entry off its home slot, a repeated name, more variables than an
instance holds on the device."""
import pytest

from psm import Client, open_jobs
from test_gpu_scheduled import KEY_A, KEY_B, check, single, write
from zeebe_amd import abi, bpmn

pytestmark = pytest.mark.gpu


def processes():
    a = bpmn.createExecutableProcess("docs").startEvent().serviceTask("a", "a").serviceTask("b", "b").endEvent().done()
    b = bpmn.createExecutableProcess("subDocs").startEvent().subProcess("sub").startEvent().serviceTask("t", "t")
    b = b.endEvent().subProcessDone().zeebeInputExpression("x", "y").endEvent().done()
    return a, b


def _jobs(ref, typ):
    return sorted(k for k, r in open_jobs(ref.parts[0].log).items() if r.value["type"] == typ)


@pytest.mark.parametrize("limit", [3, 100])
def test_multi_entry_documents_in_the_processing_loop(limit):
    a, b = processes()
    deps = [(a, KEY_A, 1), (b, KEY_B, 1)]
    ref, gpu = single(deps, deps, limit=limit)
    creates = [
        [("amount", 5), ("name", "x"), ("flag", True)],
        [("abc", "xyz"), ("q", 1)],                       # an entry off its home slot (no removal: fine)
        [("price", 1.5), ("items", [1, 2, 3]), ("n", None)],
        [("a", "abc"), ("b", "abcde"), ("c", 1)],         # a probe chain wrapping the table
        [("d", 1), ("d", 2)],                             # a repeated name: the engine's
        [("v%d" % i, i) for i in range(5)],               # five variables: past the device's four
    ]
    write(ref, gpu, *[Client.create("docs", variables=v) for v in creates])
    write(ref, gpu, *[Client.create("subDocs", variables=v) for v in ([("x", 3)], [("x", 4), ("w", "s")],
                                                                       [("x", 5)], [("x", 6)])])
    ja = _jobs(ref, "a")
    write(ref, gpu, *[Client.complete_job(k, variables=v) for k, v in zip(ja, (
        [("amount", 7), ("note", "n")],                   # an update and a new variable
        [("q", 1), ("abc", "other")],                     # equal, then updated
        [("items", [4]), ("price", 2.25)],
        [("c", 2), ("e", "e")],
    ))])
    jb = _jobs(ref, "b")
    write(ref, gpu, *[Client.complete_job(k, variables=[("name", "x"), ("flag", False)]) for k in jb])
    jt = _jobs(ref, "t")
    write(ref, gpu, *[Client.complete_job(k, variables=v) for k, v in zip(jt, (
        [("y", 9), ("z", 1)],                             # y updated in the sub-process's scope (removed)
        [("z", 1), ("y", 4)],                             # y equal: not removed, created in the process's scope
        [("abc", "xyz"), ("y", 9)],                       # a removal with an entry off its home slot: the engine's
        [("u", 1), ("t", 2)],
    ))])
    for _ in range(3):
        live = sorted(open_jobs(ref.parts[0].log))
        if not live:
            break
        write(ref, gpu, *[Client.complete_job(k) for k in live])
    check(ref, gpu)
    log = gpu.parts[0].log.entries
    done = sum(1 for r in log if r.value_type == abi.VT_PROCESS_INSTANCE and r.intent == abi.PI_ELEMENT_COMPLETED
               and r.value["bpmnElementType"] == "PROCESS")
    assert done == len(creates) + 4
    ad = gpu.parts[0].adapter
    assert ad.counts["device_commands"] >= 14
    # the declines: the repeated name and the displaced removal (FB_DOC); the five variables at creation and
    # the instances whose scopes reach more than kVars variables (FB_VARS)
    assert sorted(set(ad.fallback_reasons)) == ["doc", "vars"] and ad.fallback_reasons.count("doc") == 2


def random_document_campaign(seed, ref, emit, n=24, rounds=30):
    """Each round completes every open job with a random document of zero to three entries over the names
    amount / p / q / r (ints, strings, booleans, decimals; amount stays an integer for the conditions)."""
    import numpy as np
    rng = np.random.default_rng(seed)

    def value(name):
        k = int(rng.integers(0, 4))
        if name == "amount" or k == 0:
            return int(rng.integers(0, 1000))
        return ("s%d" % int(rng.integers(0, 5)), bool(int(rng.integers(0, 2))), int(rng.integers(0, 8)) / 4)[k - 1]

    emit(*[Client.create("random", variables=[("amount", int(a)), ("p", value("p"))]) for a in rng.integers(0, 1000, n)])
    for _ in range(rounds):
        jobs = sorted(open_jobs(ref.parts[0].log))
        if not jobs:
            break
        cmds = []
        for k in jobs:
            names = [x for x in ("amount", "p", "q", "r") if int(rng.integers(0, 3)) == 0]
            rng.shuffle(names)
            cmds.append(Client.complete_job(k, variables=[(x, value(x)) for x in names]))
        emit(*cmds)


# (seeds whose processes wait in job worker tasks: 1, 3, 4, 9, 15, 18 update the most variables)
@pytest.mark.parametrize("seed", [1, 3, 4, 9, 15, 18])
def test_random_processes_with_multi_entry_documents(seed):
    import numpy as np
    from random_bpmn import random_process
    xml = random_process(np.random.default_rng(9500 + seed), sub_processes=True, task_kinds=True)
    deps = [(xml, KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=100)
    random_document_campaign(seed, ref, lambda *r: write(ref, gpu, *r))
    check(ref, gpu)
    ad = gpu.parts[0].adapter
    assert ad.counts["device_commands"] >= 24
    print("handed off", len(ad.handed_off), "fallbacks", ad.fallback_reasons)


def _doc_window(rng, names, n, width):
    """n documents of `width` scalar entries (ints, booleans, decimals, nil) over `names`, their merge order
    set: the docs array and each command's (doc_begin, doc_count)."""
    import numpy as np
    from zeebe_amd.adapter import set_merge_order
    rows, spans = [], []
    for _ in range(n):
        pick = list(rng.choice(len(names), size=width, replace=False))
        variables = []
        for j in pick:
            k = int(rng.integers(0, 4))
            variables.append((names[j][0], (int(rng.integers(-100000, 100000)), bool(k & 1), int(rng.integers(0, 99)) / 4,
                                             None)[k]))
        d = abi.make_docs(width)
        for e, (nm, v) in enumerate(variables):
            d[e]["name_id"] = dict(names)[nm]
            if v is None:
                d[e]["type"] = abi.DOC_NIL
            elif isinstance(v, bool):
                d[e]["type"], d[e]["value"] = abi.DOC_BOOL, int(v)
            elif isinstance(v, float):
                d[e]["type"], d[e]["value"] = abi.DOC_DEC, round(v * 10 ** abi.DEC_SCALE)
            else:
                d[e]["type"], d[e]["value"] = abi.DOC_INT, v
        spans.append((sum(len(r) for r in rows), width))
        rows.append(set_merge_order(d, variables))
    return np.concatenate(rows), spans


@pytest.mark.parametrize("width", [2, 3, 4])
def test_multi_entry_documents_log_bytes(width):
    # creations and two rounds of job completions with multi-entry documents: the device's records and state
    # equal the oracle's, its log bytes equal the host serialiser's, which equal the Python restatement's
    # (tests/test_gpu_logserial.Pair), and the device log writer takes the windows (no host fallback)
    import numpy as np
    from helpers import create_commands
    from test_gpu_logdev import Log, job_completions
    from test_gpu_logserial import Pair
    xml = bpmn.createExecutableProcess("docs").startEvent().serviceTask("a", "a").serviceTask("b", "b").endEvent().done()
    words = ("amount", "p", "q", "r_long_variable_name")
    n = 64
    pair, log = Pair(xml, n, names=words), Log(xml, n, names=words)
    names = [(w, pair.part.intern(w)) for w in words]
    assert names == [(w, log.part.intern(w)) for w in words]
    rng = np.random.default_rng(width)
    cmds = create_commands(n)
    docs, spans = _doc_window(rng, names, n, width)
    cmds["doc_begin"], cmds["doc_count"] = [s[0] for s in spans], [s[1] for s in spans]
    pair.window(cmds, docs)
    recs = log.window(cmds, docs)
    assert log.part.state() == pair.orc.state()
    for _ in range(2):
        c = job_completions(recs, log.part)
        docs, spans = _doc_window(rng, names, len(c), width)
        c["doc_begin"], c["doc_count"] = [s[0] for s in spans], [s[1] for s in spans]
        pair.window(c, docs)
        recs = log.window(c, docs)
        assert log.part.state() == pair.orc.state()
    assert log.declined == 0 and log.part.stats()["fallback"] == 0
    assert [r for r in log.part.state() if not r.startswith("KEY|")] == []
