"""Summarise a rocprofv3 --pmc counter_collection.csv: mean counter value per launch for the
engine's kernels (gck::*). Usage: python tools/pmc_summary.py <counter_collection.csv>"""
import csv
import sys
from collections import defaultdict


def main(path):
    acc = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "gck::" not in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            acc[short][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[short].add(r["Dispatch_Id"])
            meta[short] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"],
                           r["SGPR_Count"], r["Scratch_Size"])
    for k, ctr in acc.items():
        n = len(launches[k])
        g, wg, lds, vg, sg, scr = meta[k]
        print(f"{k}: launches={n} grid={g} wg={wg} lds={lds} vgpr={vg} sgpr={sg} scratch={scr}")
        for c in sorted(ctr):
            print(f"   {c:28s} {ctr[c] / n:16.1f} per launch")


if __name__ == "__main__":
    main(sys.argv[1])
