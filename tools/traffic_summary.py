"""Per-batch HBM bytes of the bundle kernels from tools/pmc_traffic.sh output.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (rocprofv3 derived counters). On gfx950
FETCH_SIZE reports half the bytes of wide reads (MI355X_MICROARCH.md §HBM), so it is doubled;
for this kernel's narrow random reads the factor is uncalibrated (the raw values are kept)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    tot, launches = defaultdict(float), defaultdict(set)
    for f in glob.glob(path, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "k_bundles" not in r["Kernel_Name"]:
                continue
            k = "k_bundles<1>" if "k_bundles<1," in r["Kernel_Name"] else "k_bundles<16>"
            tot[k] += float(r["Counter_Value"])
            launches[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(launches[k]) * 1024 for k in tot}  # bytes per launch


def main(out):
    fetch = per_kernel(f"{out}/fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(f"{out}/write/**/*counter_collection.csv", "WRITE_SIZE")
    res = {"fetch_bytes_raw": fetch, "write_bytes": write}
    res["hbm_bytes_per_batch"] = int(sum(2 * v for v in fetch.values()) + sum(write.values()))
    res["correction"] = "FETCH_SIZE x2 (gfx950) + WRITE_SIZE; both kernels of one batch"
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
