"""Per-batch timeline of a rocprofv3 kernel trace (kernel_trace.csv): per kernel name its mean
duration, and the mean gap from the previous kernel's end on the same queue."""
import csv
import glob
import sys
from collections import defaultdict


def short(n):
    for k in ("k_closure_join", "k_bundles<1,", "k_bundles<16,", "k_publish", "k_gather", "k_scatter"):
        if k in n:
            return k.rstrip("<,")
    return n[:40]


rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "0")))
rows.sort()
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
last_end = {}
for s, e, k, q in rows:
    dur[k] += e - s
    cnt[k] += 1
    if q in last_end:
        gap[k] += max(0, s - last_end[q])
    last_end[q] = e
span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0
print(f"kernels={len(rows)} span_us={span:.1f}")
for k in sorted(cnt, key=lambda x: -dur[x]):
    print(f"{k:20s} n={cnt[k]:6d} mean_dur_us={dur[k] / cnt[k] / 1e3:8.2f} mean_gap_before_us={gap[k] / cnt[k] / 1e3:8.2f}")
