"""Wider randomized parity campaign on the GPU (not part of the suite): random structured processes
(tests/random_bpmn.py) in five flavours -- plain, pass-through elements, job-worker kinds with
sub-processes, timer boundary events, multi-instance activities -- driven through the device and
the CPU oracle window by window (each round completes an open job or fires an open timer per
instance, at random).  Every window the device took in full must equal the oracle bit-exact
(records and state); a window in which the device declined commands (a fallback: the adapter hands
those instances to the engine) ends that run as "declined".  Usage:
python scripts/fuzz_random.py FIRST LAST [budget_s]; exit 1 on any parity failure.  FUZZ_MAX_RECORDS sets
the device's records per batch (default 256; smaller values exercise the continuation batches)."""
import collections
import os
import sys
import time
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))

from helpers import amount_docs, create_commands  # noqa: E402
from random_bpmn import random_process  # noqa: E402
from test_gpu_parity import assert_same_records  # noqa: E402
from test_gpu_timers import _open_work  # noqa: E402
from test_oracle_timers import NOW  # noqa: E402
from oracle.oracle import Oracle, OracleError  # noqa: E402
from zeebe_amd.engine import Partition  # noqa: E402

FLAVOURS = {"plain": (1000, {}), "pass_through": (2000, {"pass_through": True}),
            "kinds_subs": (4000, {"sub_processes": True, "task_kinds": True}),
            "boundary": (6000, {"sub_processes": True, "task_kinds": True, "boundaries": True}),
            "multi_instance": (7000, {"sub_processes": True, "task_kinds": True, "boundaries": True,
                                      "multi_instance": True})}


def run(flavour, seed, n=96, phases=80):
    base, kw = FLAVOURS[flavour]
    rng = np.random.default_rng(base + seed)
    xml = random_process(rng, **kw)
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=int(os.environ.get("FUZZ_MAX_RECORDS", 256)))
    orc = Oracle()
    assert part.deploy(xml) == orc.deploy(xml) == 0
    clock = NOW
    for e in (part, orc):
        e.set_clock(clock)
    assert part.intern("amount") == orc.intern("amount")
    cmds, docs = create_commands(n, 0), amount_docs(rng.integers(0, 1000, n), 0)
    cmds["doc_count"] = 1
    cmds["doc_begin"] = np.arange(n)
    wrng = np.random.default_rng(seed)
    for phase in range(phases + 1):
        c = cmds if phase == 0 else _open_work(part, wrng)
        if c is None:
            return "passed"
        if phase:
            clock += 1000
            for e in (part, orc):
                e.set_clock(clock)
        f0 = part.stats()["fallback"]
        part.submit(c, docs if phase == 0 else None)
        part.run()
        got = part.drain()
        declined = part.stats()["fallback"] > f0 or any(part.command_status(i)[0] for i in range(len(c)))
        if declined:
            return "declined:" + ",".join(sorted({str(part.command_status(i)[1]) for i in range(len(c))
                                                   if part.command_status(i)[0]}))
        orc.clear_records()
        orc.submit(c, docs if phase == 0 else None)
        try:
            orc.run()
        except OracleError as ex:
            raise AssertionError("the device took a window the oracle refuses: %s" % ex)
        assert_same_records(got, orc.records(), part, orc)
        assert part.state() == orc.state()
    return "passed"


def main(first, last, budget):
    t0 = time.time()
    outcome, fails = collections.Counter(), []
    for seed in range(first, last):
        for fl in FLAVOURS:
            if time.time() - t0 > budget:
                break
            try:
                outcome[run(fl, seed)] += 1
            except Exception as e:  # noqa: BLE001
                outcome["FAILED"] += 1
                fails.append((fl, seed))
                print("FAIL %s seed %d: %s" % (fl, seed, (str(e).splitlines() or [type(e).__name__])[0][:300]), flush=True)
                traceback.print_exc(limit=2)
        if seed % 10 == 0:
            print("seed %d, %.0f s: %s" % (seed, time.time() - t0, dict(outcome)), flush=True)
    print("summary: %s failures %s" % (dict(outcome), fails), flush=True)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]) if len(sys.argv) > 3 else 1e9))
