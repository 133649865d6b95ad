"""Key bookkeeping journaled on the device (runtime.cpp fold_journal): windows written through
zbhip_serialize_log_device over a device-built command table leave their key bookkeeping in HBM, and
the host tables (key histories, resolve table, instance processes and generations) catch up only when
a host consumer reads them.  A partition that journals many windows and then drains, resolves and
exports must be indistinguishable from one that booked every window on the host (ZBHIP_NO_JOURNAL):
the same log bytes per window, records, state, zb-db bytes and key resolution -- also when the
journal overflows (ZBHIP_JOURNAL_WINDOWS=2: the oldest windows are folded as new ones arrive)."""
import os

import numpy as np
import pytest

from helpers import create_commands
from zeebe_amd import abi, bpmn
from zeebe_amd.engine import Partition

pytestmark = pytest.mark.gpu

TS = 1700000000123


class Side:
    def __init__(self, xml, n, journal_windows=None, journal=True):
        env = {"ZBHIP_JOURNAL": "1"}
        if journal_windows:
            env["ZBHIP_JOURNAL_WINDOWS"] = str(journal_windows)
        self.env = env if journal else {"ZBHIP_NO_JOURNAL": "1"}
        self.part = Partition(max_instances=n, max_commands=4 * n, max_records_per_batch=128)
        assert self.part.deploy(xml) == 0
        self.position = 100

    def window(self, cmds):
        self.part.submit(cmds, abi.make_docs(0))
        self.part.run(abi.RUN_DEVICE_RECORDS)
        pos = self.position + 2 * np.arange(len(cmds), dtype=np.int64)
        first = int(pos[-1]) + 1
        old = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)
        try:
            dev = self.part.serialize_log_device(pos, first, TS)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        self.position = first + int(self.part.L.zbhip_pending_records(self.part.h))
        return dev


def completions(keys, part):
    c = abi.make_commands(len(keys))
    for i, k in enumerate(keys):
        c[i]["instance"], c[i]["ref"] = part.resolve_key(k)
    c["kind"] = abi.CMD_JOB_COMPLETE
    return c


def job_keys(part):
    return sorted(int(r.split("|")[1]) for r in part.state() if r.startswith("JOBS|"))


@pytest.mark.parametrize("journal_windows", [None, 2])
def test_journaled_windows_equal_host_booked(journal_windows):
    n, tasks = 200, 6
    xml = bpmn.linear_process(tasks)
    A = Side(xml, n, journal_windows)        # journals every window
    B = Side(xml, n, journal=False)          # books every window on the host
    rng = np.random.default_rng(5)
    assert A.window(create_commands(n)) == B.window(create_commands(n))
    for w in range(tasks):
        # B resolves the open jobs (its host tables are current); A is handed the same commands
        # and never reads its host tables until the end.  Half the jobs per window, so instances
        # spread over windows and some end while others run.
        keys = job_keys(B.part)
        rng.shuffle(keys)
        keys = keys[: max(1, len(keys) // 2)] if w < tasks - 1 else keys
        c = completions(sorted(keys), B.part)
        assert A.window(c) == B.window(c), w
    # the consumers: the last window's records, state, zb-db bytes, key resolution
    ra, rb = A.part.drain(), B.part.drain()
    assert np.array_equal(ra, rb)
    assert A.part.state() == B.part.state()
    assert A.part.state_db() == B.part.state_db()
    for k in job_keys(B.part):
        assert A.part.resolve_key(k) == B.part.resolve_key(k)
    # and both continue alike
    while job_keys(B.part):
        c = completions(job_keys(B.part), B.part)
        assert A.window(c) == B.window(c)
    assert A.part.state() == B.part.state()
    assert not [r for r in A.part.state() if r.startswith("JOBS|")]
