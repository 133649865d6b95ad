"""Loop-level random campaign for error events (not part of the suite): tests/random_bpmn.py processes
with error boundary events and, in the second flavour, error-start event sub-processes, driven through
the platform's processing loop twice -- the engine alone and [adapter, engine] -- by
tests/test_gpu_error_events.py's campaign (complete, leave or throw E1 / E2 / E3 per open job each
round); with --documents, processes without error events whose jobs complete with documents of zero to
three entries (tests/test_gpu_documents.py's campaign: the multi-entry merge order).  A seed passes when every record and the state agree after every write.  Batch limits alternate
between 100 and 3 by seed.  Usage: python scripts/fuzz_loop_errors.py FIRST LAST [--documents]"""
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
from random_bpmn import random_process  # noqa: E402
from test_gpu_documents import random_document_campaign  # noqa: E402
from test_gpu_error_events import random_error_campaign  # noqa: E402
from test_gpu_scheduled import KEY_A, single, write  # noqa: E402


def run(seed, esp):
    xml = random_process(np.random.default_rng(9000 + seed), sub_processes=True, task_kinds=True, errors=True,
                         event_sub_processes=esp)
    deps = [(xml, KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=3 if seed % 2 else 100)
    thrown = random_error_campaign(seed, ref, lambda *r: write(ref, gpu, *r), xml)
    ad = gpu.parts[0].adapter
    return thrown, ad.counts["device_commands"], sorted(set(ad.fallback_reasons))


def run_documents(seed):
    xml = random_process(np.random.default_rng(9500 + seed), sub_processes=True, task_kinds=True)
    deps = [(xml, KEY_A, 1)]
    ref, gpu = single(deps, deps, limit=3 if seed % 2 else 100)
    random_document_campaign(seed, ref, lambda *r: write(ref, gpu, *r))
    ad = gpu.parts[0].adapter
    return 0, ad.counts["device_commands"], sorted(set(ad.fallback_reasons))


def main():
    first, last = int(sys.argv[1]), int(sys.argv[2])
    docs = "--documents" in sys.argv[3:]
    t0 = time.time()
    passed = failed = thrown = dev = 0
    declined = {}
    for seed in range(first, last):
        for esp in ((None,) if docs else (False, True)):
            tag = "%d/%s" % (seed, "documents" if docs else "esp" if esp else "boundary")
            try:
                t, d, reasons = run_documents(seed) if docs else run(seed, esp)
            except Exception:  # a parity difference (check's AssertionError) or a crash
                failed += 1
                print("FAIL", tag, traceback.format_exc().splitlines()[-1][:400], flush=True)
                continue
            passed += 1
            if reasons:
                print("FALLBACK", tag, reasons, flush=True)
            thrown += t
            dev += d
            for r in reasons:
                declined[r] = declined.get(r, 0) + 1
        if (seed - first) % 10 == 9:
            print("seed %d: %d passed, %d failed, %.0f s" % (seed, passed, failed, time.time() - t0), flush=True)
    print("SUMMARY seeds %d-%d: %d processes passed, %d failed; %d errors thrown, %d device commands; "
          "seeds with a fallback by reason %s; %.0f s" % (first, last - 1, passed, failed, thrown, dev, declined,
                                                         time.time() - t0), flush=True)
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
