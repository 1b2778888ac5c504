"""Per-batch HBM bytes of the check kernels, from `tools/gpu.sh profile` output.

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (rocprofv3 derived counters). MI355X_MICROARCH.md
§HBM establishes FETCH_SIZE = 1/2 of the bytes for wide streaming reads only; tools/gather_probe
measures random aligned reads of 4, 16, 32 and 64 B from a table 16x the Infinity Cache (known
bytes): every one of them is reported as 64 B — one memory-side line per access, whatever its
width. For these kernels, whose reads are random and at most 64 B, raw FETCH_SIZE is therefore the
HBM line traffic itself (factor 1, the 64-B calibration point), and no x2 correction applies."""
import csv
import glob
import json
import sys
from collections import defaultdict


def kernel_key(name):
    if "k_closure_join" in name:
        return "k_closure_join"
    if "k_label_join" in name:
        return "k_label_join"
    if "k_bundles<1," in name:
        return "k_bundles<1>"
    if "k_bundles<16," in name:
        return "k_bundles<16>"
    if "k_publish" in name:
        return "k_publish"
    if "k_gather<" in name:
        return "k_gather<" + name.split("k_gather<")[1].split(">")[0] + ">"
    return None


def per_kernel(path, counter):
    tot, launches = defaultdict(float), defaultdict(set)
    for f in glob.glob(path, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_key(r["Kernel_Name"])
            if k is None:
                continue
            tot[k] += float(r["Counter_Value"])
            launches[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(launches[k]) * 1024 for k in tot}, {k: len(v) for k, v in launches.items()}


def kernel_stats(out):
    rows = {}
    for f in glob.glob(f"{out}/kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Name"])
            if k:
                rows[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                           "total_ms": float(r["TotalDurationNs"]) / 1e6}
    return rows


def main(out):
    gf, _ = per_kernel(f"{out}/gfetch/**/*counter_collection.csv", "FETCH_SIZE")
    gw, _ = per_kernel(f"{out}/gwrite/**/*counter_collection.csv", "WRITE_SIZE")
    lanes = 1 << 24
    calib = {}
    for k, v in gf.items():
        width = int(k[len("k_gather<"):-1])
        calib[width] = {"fetch_reported": v, "read_bytes": lanes * width, "factor": lanes * width / v if v else None,
                        "write_reported": gw.get(k), "write_bytes": lanes * 4}
    fetch, n_fetch = per_kernel(f"{out}/fetch/**/*counter_collection.csv", "FETCH_SIZE")
    write, n_write = per_kernel(f"{out}/write/**/*counter_collection.csv", "WRITE_SIZE")
    stage_a = [k for k in ("k_closure_join", "k_label_join", "k_bundles<1>") if k in fetch]
    factor = (calib.get(64) or {}).get("factor") or 1.0  # one 64-B line per random access
    raw = sum(fetch[k] for k in stage_a)
    # the random-line ceiling of the same box: tools/gather_probe's random aligned reads per second
    # (G accesses/s per width; median of its repeats) — the joins' bound (bench.py roofline_line)
    rates = defaultdict(list)
    for f in glob.glob(f"{out}/gather_plain.jsonl"):
        for line in open(f):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            rates[str(r["width"])].append(r["lanes"] / (r["ms"] * 1e-3) / 1e9)
    ceiling = {w: round(sorted(v)[len(v) // 2], 2) for w, v in rates.items()}
    res = {
        "line_ceiling": ceiling,
        "calibration": calib,
        "fetch_bytes_raw_per_launch": fetch, "write_bytes_per_launch": write, "launches": n_fetch,
        "fetch_factor_used": factor,
        "hbm_bytes_per_batch": int(raw * factor + sum(write.get(k, 0) for k in stage_a)),
        "hbm_bytes_per_batch_raw": int(raw + sum(write.get(k, 0) for k in stage_a)),
        "kernels": stage_a,
        "kernel_stats": kernel_stats(out),
        "correction": "FETCH_SIZE x the gather_probe factor at 64 B (random reads of 4-64 B all count one "
                      "64-B line: FETCH_SIZE is the line traffic) + WRITE_SIZE, summed over the stage-A kernels "
                      "of one batch",
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
