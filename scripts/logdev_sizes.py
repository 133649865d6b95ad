"""Debug aid: the device log-byte path over growing linear-10 windows (ZBHIP_DEBUG timings)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from zeebe_amd import abi, bpmn  # noqa: E402
from zeebe_amd.engine import Partition  # noqa: E402

for n in [int(x) for x in sys.argv[1:]] or [10000, 100000, 1000000]:
    part = Partition(max_instances=n, max_commands=n, max_records_per_batch=64)
    part.deploy(bpmn.linear_process(10))
    c = abi.make_commands(n)
    c["instance"] = np.arange(n)
    c["kind"] = abi.CMD_CREATE
    part.submit(c)
    part.run(abi.RUN_DEVICE_RECORDS)
    t = time.perf_counter()
    ptr, used = part.serialize_log_device(np.arange(n, dtype=np.int64) * 2 + 1, 1, 1700000000123, copy=False)
    print("n=%d used=%d %.2f ms" % (n, used, (time.perf_counter() - t) * 1e3), flush=True)
