"""Summarise rocprofv3 PMC passes (scripts/pmc.sh) into per-launch HBM traffic of one kernel.

FETCH_SIZE / WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts half of the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is doubled here;
WRITE_SIZE is taken as reported.  Usage: python scripts/pmc_traffic.py gpurun_out/pmc out.json [kernel]
[steps]: per launch of the kernels whose name contains `kernel` (default k_step); with `steps` (the
bench steps the profiled run executed, warmup and the timed pass included) also the traffic of all
those kernels per step (config 5: k_step + key scan + bucketing)."""
import collections
import csv
import glob
import json
import os
import sys


def main(pmc_dir, out, kernel="k_step", steps=None):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            per[f][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[f].add(r["Dispatch_Id"])
    counters = {}
    for f, cs in per.items():
        n = len(disp[f])
        for c, v in cs.items():
            counters[c] = v / n
    fetch = counters.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = counters.get("WRITE_SIZE", 0.0) * 1024
    res = {"kernel": kernel, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write, "fetch_correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950)",
           "counters_per_launch": counters}
    if steps:
        tot = {}
        for f, cs in per.items():
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in cs:
                    tot[c] = cs[c]
        res["steps"] = int(steps)
        res["traffic_bytes_per_step"] = (tot.get("FETCH_SIZE", 0.0) * 2 + tot.get("WRITE_SIZE", 0.0)) * 1024 / int(steps)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    main(*sys.argv[1:])
