"""Debug helper: the random boundary-event (mode "boundary") or multi-instance (mode "mi") GPU test
for one seed; on the first mismatching window -- or an oracle refusal -- the records around the first
difference (both sides, element ids) and the process XML.  Usage: debug_mi_random.py MODE SEED"""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
from helpers import amount_docs
from random_bpmn import random_process
from test_gpu_timers import _open_work
from test_oracle_timers import NOW
from helpers import create_commands
from oracle.oracle import Oracle
from zeebe_amd.engine import Partition
from zeebe_amd import abi

mode, seed = sys.argv[1], int(sys.argv[2])
rng = np.random.default_rng((7000 if mode == "mi" else 6000) + seed)
xml = random_process(rng, sub_processes=True, task_kinds=True, boundaries=True, multi_instance=mode == "mi")
n = 96
part = Partition(max_instances=n, max_commands=n, max_records_per_batch=256)
orc = Oracle()
part.deploy(xml); orc.deploy(xml)
clock = NOW
for e in (part, orc):
    e.set_clock(clock)
cmds = create_commands(n, 0)
part.intern("amount"); orc.intern("amount")
docs = amount_docs(rng.integers(0, 1000, n), 0)
cmds["doc_count"] = 1
cmds["doc_begin"] = np.arange(n)
wrng = np.random.default_rng(seed)
F = ("value_type", "intent", "record_type", "element_idx", "key", "scope_key", "source_index", "aux")


def show(a, i, who, e):
    r = a[i]
    el = e.element_id(int(r["process_idx"]), int(r["element_idx"])) if r["element_idx"] >= 0 and r["value_type"] != abi.VT_VARIABLE else ""
    return "%s %d %s %s" % (who, i, tuple(int(r[f]) for f in F), el)


for phase in range(81):
    c = cmds if phase == 0 else _open_work(part, wrng)
    if c is None:
        break
    if phase:
        clock += 1000
        for e in (part, orc):
            e.set_clock(clock)
    part.submit(c, docs if phase == 0 else None)
    part.run()
    got = part.drain()
    orc.clear_records()
    orc.submit(c, docs if phase == 0 else None)
    try:
        orc.run()
    except Exception as ex:  # noqa: BLE001
        want = orc.records()
        print("phase", phase, "oracle refused:", ex, "records so far", len(want), "device", len(got), "stats", part.stats())
        print("declined:", [(i, part.command_status(i)) for i in range(len(c)) if part.command_status(i)[0] != 0][:10])
        last = int(want["source_index"][-1]) if len(want) else 0
        for i in range(len(got)):
            if int(got["source_index"][i]) in (last, last + 1):
                print(show(got, i, "G", part))
        for i in range(max(0, len(want) - 12), len(want)):
            print(show(want, i, "W", orc))
        print("commands:", [(int(x["instance"]), int(x["kind"]), int(x["ref"])) for x in c][last:last + 3])
        print(xml)
        break
    want = orc.records()
    m = min(len(got), len(want))
    bad = next((i for i in range(m) if any(got[f][i] != want[f][i] for f in ("value_type", "intent", "record_type", "element_idx", "key", "aux"))), m)
    if len(got) != len(want) or bad < m:
        print("phase", phase, "got", len(got), "want", len(want), "stats", part.stats(), "fallback", part.fallback())
        print("declined:", [(i, part.command_status(i)) for i in range(len(c)) if part.command_status(i)[0] != 0][:10])
        for i in range(max(0, bad - 6), min(max(len(got), len(want)), bad + 8)):
            if i < len(got):
                print(show(got, i, "G", part))
            if i < len(want):
                print(show(want, i, "W", orc))
        src = int(want["source_index"][bad]) if bad < len(want) else -1
        print("commands:", [(int(x["instance"]), int(x["kind"]), int(x["ref"])) for x in c][:20])
        print(xml)
        break
else:
    print("no mismatch")
