"""Per-step GPU timeline of the last steps of a rocprofv3 kernel + memory-copy trace (csv): each
kernel / copy with its start relative to the step's first merge kernel, duration and queue."""
import csv
import glob
import sys

d = sys.argv[1]
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(kt)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r.get("Queue_Id", "")))
mc = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
for f in mc:
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", ""), ""))
rows.sort()
marks = [i for i, r in enumerate(rows) if "k_dj_locate_prefix" in r[2]]
for s in marks[-6:-1]:
    t0 = rows[s][0]
    nxt = [m for m in marks if m > s][0]
    print("---- step", (rows[nxt][0] - t0) / 1e3, "us")
    for r in rows[s:nxt]:
        if r[2].startswith("void at::") or "elementwise" in r[2]:
            continue
        print(f"{(r[0] - t0) / 1e3:8.1f} {(r[1] - r[0]) / 1e3:7.1f}  {r[3]:>3} {r[2]}")
