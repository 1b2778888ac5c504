"""Where a host-buffer batch's time goes, from a rocprofv3 trace with --kernel-trace and
--memory-copy-trace: per kernel and per copy direction the mean duration and count, and the
busy fraction of the copy engines and of the kernels over the traced span."""
import csv
import glob
import sys
from collections import defaultdict


def intervals(pattern, key):
    out = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), key(r)))
    return sorted(out)


def busy(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(d):
    k = intervals(f"{d}/**/*kernel_trace.csv", lambda r: r["Kernel_Name"][:32])
    c = intervals(f"{d}/**/*memory_copy_trace.csv", lambda r: r.get("Direction", r.get("Operation", "copy")))
    allv = sorted(k + c)
    span = (allv[-1][1] - allv[0][0]) if allv else 1
    for name, iv in (("kernels", k), ("copies", c)):
        agg = defaultdict(lambda: [0, 0])
        for s, e, n in iv:
            agg[n][0] += e - s
            agg[n][1] += 1
        print(f"{name}: busy {busy(iv) / span:.2%} of {span / 1e3:.0f} us")
        for n, (t, m) in sorted(agg.items(), key=lambda x: -x[1][0])[:8]:
            print(f"   {n:34s} n={m:6d} mean_us={t / m / 1e3:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
