"""Timeline of the last --last batches of a rocprofv3 kernel trace (the timed region of a bench.py
run with --no-profile --host-steps 0 --no-oracle, whose final launches are the timed batches):
per engine kernel launch its start / end relative to the first one, duration and queue, and the
span of the whole group, so that fill / drain and gaps between batches can be read off.

    python tools/trace_gaps.py <kernel_trace.csv> [--last 20] [--kernel k_label_join]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--kernel", default="k_label_join")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if "gck::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    heads = [i for i, r in enumerate(rows) if args.kernel in r["Kernel_Name"]]
    if not heads:
        print(json.dumps({"error": f"no {args.kernel} launches"}))
        return
    first = heads[-args.last] if len(heads) >= args.last else heads[0]
    sel = rows[first:]
    t0 = int(sel[0]["Start_Timestamp"])
    out = []
    for r in sel:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gck::", "")
        out.append({"k": name, "start_us": round(s / 1e3, 2), "end_us": round(e / 1e3, 2),
                    "dur_us": round((e - s) / 1e3, 2), "queue": r.get("Queue_Id"), "stream": r.get("Stream_Id")})
    span = max(o["end_us"] for o in out)
    busy = sum(o["dur_us"] for o in out if args.kernel in o["k"])
    print(json.dumps({"launches": len(out), "span_us": span, f"{args.kernel}_sum_us": round(busy, 2),
                      "timeline": out}, indent=0))


if __name__ == "__main__":
    main()
