"""Per-dispatch HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) of zb:: kernels from
separate rocprofv3 --pmc passes, in dispatch order, joined by dispatch index within each pass.
Usage: python scripts/pmc_dispatch.py <pmc_dir> [last_n]"""
import collections
import csv
import glob
import os
import sys


def load(f):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "zb::" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        e = per.setdefault(d, {"name": r["Kernel_Name"], "v": 0.0})
        e["v"] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main(pmc_dir, last_n="60"):
    passes = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv"))):
        c = next(csv.DictReader(open(f)))["Counter_Name"]
        passes[c] = load(f)
    fe, wr = passes.get("FETCH_SIZE", []), passes.get("WRITE_SIZE", [])
    n = min(len(fe), len(wr))
    rows = list(range(n))[-int(last_n):]
    tot = collections.defaultdict(float)
    for i in rows:
        name = fe[i]["name"].split("(")[0].replace("void ", "")[:60]
        f, w = fe[i]["v"] * 2048, wr[i]["v"] * 1024
        tot[name] += f + w
        print("%4d %-60s fetch %10.1f MB write %10.1f MB" % (i, name, f / 1e6, w / 1e6))
    print("totals over the listed dispatches:")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("  %-60s %10.1f MB" % (k, v / 1e6))


if __name__ == "__main__":
    main(*sys.argv[1:])
