"""Names the commands a loop-level campaign seed hands to the engine: every GpuBatchProcessor fallback prints
its window command (kind, subject), the record's value type / intent / elementId and the instance's
live element instances from the engine-only loop's log.  Usage: debug_fallback.py SEED [--documents]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "scripts")]

from zeebe_amd import adapter  # noqa: E402

orig = adapter.GpuBatchProcessor._fall_back


def traced(self, i, record, out):
    c = self.window.cmds[i]
    v = getattr(record, "value", {}) or {}
    print("FALLBACK cmd kind=%d instance=%d reason=%s | record vt=%s intent=%s key=%s elementId=%s" %
          (int(c["kind"]), int(c["instance"]), self.fallback_reasons[-1], record.value_type, record.intent,
           record.key, v.get("elementId") if hasattr(v, "get") else None), flush=True)
    return orig(self, i, record, out)


adapter.GpuBatchProcessor._fall_back = traced

import fuzz_loop_errors as F  # noqa: E402

seed = int(sys.argv[1])
print(F.run_documents(seed) if "--documents" in sys.argv[2:] else (F.run(seed, False), F.run(seed, True)))
