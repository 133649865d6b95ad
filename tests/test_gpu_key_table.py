"""Key relabelling across compactions of the host's resolve-key table (runtime.cpp KeyTable::compact,
run by the key bookkeeping once ended instances' entries are a third of a table of >= 2^20 entries).

Long-lived instances are created first; several rounds of 400 000 short instances then run to
completion in reused slots (1.2 x 10^6 table entries per round, all dead at the round's end), so
the table is compacted while the long-lived entries sit between dead ones.  When the long-lived
instances finally continue, every key their records carry must be the one created for them in the
first window (process instance, flow scope, the task's element instance) or a key of the final
window's own range.  Reference behaviour: keys are assigned once and never change
(DbKeyGenerator, BpmnStateTransitionBehavior) -- a compaction that dropped or shifted a live entry
would resolve a stale or foreign key here."""
import numpy as np
import pytest

from helpers import complete_commands, create_commands
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu


def test_long_lived_keys_survive_key_table_compaction():
    L, S, rounds = 1000, 400_000, 4
    part = Partition(max_instances=L + S, max_commands=S, max_records_per_batch=64)
    part.deploy(bpmn.linear_process(2))
    part.submit(create_commands(L, 0, 0))
    part.run()
    stats = [part.stats()]
    first = part.drain()
    assert len(first) and (first["source_index"] < L).all()
    old = [set() for _ in range(L)]
    pik = np.full(L, -1, dtype=np.int64)
    for r in first:
        i = int(r["source_index"])
        old[i].update(int(k) for k in (r["key"], r["scope_key"], r["process_instance_key"]) if k > 0)
        pik[i] = r["process_instance_key"]
    assert (pik > 0).all()
    base = int(first["key"][first["key"] > 0].min()) - 1  # key of counter value 0

    short = np.arange(L, L + S)
    for _ in range(rounds):
        # (full runs: RUN_NO_RESULTS skips the key bookkeeping, which is what is under test)
        part.submit(create_commands(S, 0, L))
        part.run()
        stats.append(part.stats())
        for job_ord in (5, 9):
            part.submit(complete_commands(short, np.full(S, job_ord)))
            part.run()
            stats.append(part.stats())
        assert stats[-1]["completed_instances"] == S
    assert all(s["fallback"] == 0 for s in stats)
    before = sum(int(s["keys"]) for s in stats)

    part.submit(complete_commands(np.arange(L), np.full(L, 5)))
    part.run()
    last = part.drain()
    new = int(part.stats()["keys"])
    assert part.stats()["fallback"] == 0 and len(last)
    lo, hi = base + before, base + before + new
    s0 = int(last["source_index"].min())  # (source indexes count the handle's commands; command i: instance i)
    for r in last:
        i = int(r["source_index"]) - s0
        assert r["process_instance_key"] == pik[i]
        for k in (int(r["key"]), int(r["scope_key"])):
            assert k <= 0 or k in old[i] or lo < k <= hi, (i, k, lo, hi, k - base, int(r["value_type"]),
                                                           int(r["intent"]), int(r["element_idx"]), int(r["ordinal"]))
    # the task's element instance key (from the first window) is completed in the last one
    done = last[(last["value_type"] == abi.VT_PROCESS_INSTANCE) & (last["intent"] == 5)]  # ELEMENT_COMPLETED
    assert len(done) >= L
    assert all(int(r["key"]) in old[int(r["source_index"]) - s0] for r in done[:L])
