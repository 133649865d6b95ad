"""Copy/compute overlap of the host log path (bench.py --host-io, 'host' mode: zbhip_log_copy_async) from a
rocprofv3 --kernel-trace --memory-copy-trace run: the device-to-host copy intervals against the kernel
intervals, summed where both run.  Usage: python scripts/hostio_overlap.py <rocprofv3 output dir>."""
import csv
import glob
import sys


def intervals(path, kind):
    out = []
    for f in glob.glob(path + "/**/*%s*.csv" % kind, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row))
    return sorted(out, key=lambda t: t[0])


def union(iv):
    merged = []
    for a, b, _ in iv:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    return merged


def overlap(u, v):
    i = j = tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        tot += max(0, b - a)
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


d = sys.argv[1]
allk = intervals(d, "kernel_trace")
# the log copies: the runtime's blit kernels of more than 20 ms (a window's ~4.1 GB into pinned memory;
# the memory-copy trace does not list them), and the partition's own zb:: kernels
copies = [k for k in allk if k[2]["Kernel_Name"].startswith("__amd_rocclr_copyBuffer") and k[1] - k[0] > 20_000_000]
kern = [k for k in allk if k[2]["Kernel_Name"].startswith(("zb::", "void zb::"))]
ku, cu = union(kern), union(copies)
ct = sum(b - a for a, b in cu)
kt = sum(b - a for a, b in ku)
ov = overlap(ku, cu)
per = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # log bytes per window (bench.py host_io)
print("log copies (blit kernels > 20 ms): %d, %.1f ms busy%s, streams %s" % (
    len(copies), ct / 1e6, ", %.1f GB/s while copying" % (per * len(copies) / max(ct, 1)) if per else "",
    sorted({c[2]["Stream_Id"] for c in copies})))
print("zb:: kernels: %d launches, %.1f ms busy, streams %s" % (len(kern), kt / 1e6, sorted({k[2]["Stream_Id"] for k in kern})))
print("zb:: kernel time overlapped by a log copy: %.1f ms (%.0f %%)" % (ov / 1e6, 100.0 * ov / max(kt, 1)))
