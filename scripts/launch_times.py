"""Per-launch durations of zb:: kernels from a rocprofv3 kernel_trace.csv (in launch order)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    name = r["Kernel_Name"]
    if "zb::" not in name and "k_" not in name:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print("%10.3f ms  %s" % (d, name[:110]))
