"""Per-dispatch means of every counter collected under <out>/p*/ for the check kernels."""
import csv
import glob
import json
import sys
from collections import defaultdict

KEYS = ("k_closure_join", "k_bundles<1,", "k_bundles<16,")


def main(out):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((k for k in KEYS if k in r["Kernel_Name"]), None)
            if k is None:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    res = {k: {c: v / max(1, len(disp[k][c])) for c, v in cs.items()} for k, cs in tot.items()}
    for k, cs in res.items():
        if cs.get("TCP_TCC_READ_REQ_sum"):
            cs["avg_l2_read_latency_cycles"] = cs.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / cs["TCP_TCC_READ_REQ_sum"]
        if cs.get("TCP_UTCL1_REQUEST_sum"):
            cs["utcl1_miss_rate"] = cs.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / cs["TCP_UTCL1_REQUEST_sum"]
        if cs.get("TCC_HIT_sum", 0) + cs.get("TCC_MISS_sum", 0):
            cs["l2_hit_rate"] = cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
