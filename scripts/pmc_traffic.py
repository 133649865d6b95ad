"""Summarise rocprofv3 PMC passes (scripts/pmc.sh) into per-launch HBM traffic of one kernel.

FETCH_SIZE / WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts half of the bytes of
wide coalesced reads (MI355X_MICROARCH.md, HBM/rocprofv3 section), so it is doubled here;
WRITE_SIZE is taken as reported.  Usage: python scripts/pmc_traffic.py gpurun_out/pmc out.json"""
import collections
import csv
import glob
import json
import os
import sys


def main(pmc_dir, out, kernel="k_step"):
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
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    main(*sys.argv[1:])
