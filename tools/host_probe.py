"""host_probe.py — the timeline of host-buffer batches (BASELINE.md:40-41's step: items H2D, kernels,
results D2H) against device-resident ones, on the config-4 graph.

Per phase, through the compiled submit/wait loop (libgck_driver.so): lone batches (1 in flight, the
median of the per-batch submit and wait durations and of the whole batch), and the rate at 8 in
flight. Run it alone, or under `rocprofv3 --kernel-trace --stats` to see the joins' own durations.

    python3 tools/host_probe.py --tuples 1e9 [--inflight 8] [--batches 400]
"""
import argparse
import ctypes
import json
import os
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e9)
    ap.add_argument("--config", default="nested")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--inflight", type=int, default=8)
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--lone", type=int, default=40)
    ap.add_argument("--phases", default="host,device")
    args = ap.parse_args()
    import torch
    import bench
    from gochugaru_amd.engine import Engine, ITEM_DTYPE, _driver

    dev = torch.device("cuda", 0)
    wl_args = types.SimpleNamespace(config=args.config, tuples=args.tuples, partitioned=False, scale=args.scale,
                                    batch=args.batch, churn=0.001)
    WL = bench.Workload(wl_args, dev)
    eng = Engine(device=0, workspaces=max(2, args.inflight), max_batch=args.batch)
    eng.load_schema(WL.schema)
    eng.begin_snapshot(1)
    keep = []
    WL.load(eng, keep)
    torch.cuda.synchronize()
    eng.commit_snapshot()
    n_rot = 32
    rot = [WL.checks(args.batch, 1000 + k) for k in range(n_rot)]
    outs = [(torch.zeros(args.batch, dtype=torch.uint8, device=dev),
             torch.zeros(args.batch, dtype=torch.int32, device=dev)) for _ in range(n_rot)]
    pins = []
    for b in rot:
        a = eng.host_array(args.batch, ITEM_DTYPE)
        a[:] = b.cpu().numpy().view(ITEM_DTYPE).reshape(-1)
        pins.append((a, eng.host_array(args.batch, np.uint8), eng.host_array(args.batch, np.int32)))
    torch.cuda.synchronize()
    out = {"config": args.config, "tuples": eng.tuple_count, "batch": args.batch}

    def run(kind, n_batches, depth, trace):
        ks = [j % n_rot for j in range(n_batches)]
        if kind == "host":
            run_ = eng.prepare_batches([pins[k][0].ctypes.data for k in ks], [pins[k][1].ctypes.data for k in ks],
                                       [pins[k][2].ctypes.data for k in ks], args.batch, depth, host=True)
        else:
            run_ = eng.prepare_batches([rot[k].data_ptr() for k in ks], [outs[k][0].data_ptr() for k in ks],
                                       [outs[k][1].data_ptr() for k in ks], args.batch, depth,
                                       [0] * len(ks), engine_streams=True)
        stamps = np.zeros(2 * n_batches, dtype=np.float64)
        if trace:
            _driver().gckd_set_trace(stamps.ctypes.data_as(ctypes.c_void_p), n_batches)
        dt = run_.run()
        _driver().gckd_set_trace(None, 0)
        return dt, stamps

    for kind in args.phases.split(","):
        run(kind, 16, args.inflight, False)  # warm
        dt, st = run(kind, args.lone + 3, 1, True)
        sub, wt = st[0::2], st[1::2]
        prev_end = np.concatenate([[0.0], wt[:-1]])
        per = (wt - prev_end)[3:]
        s_d = (sub - prev_end)[3:]
        w_d = (wt - sub)[3:]
        eng.reset_stats()
        dt8, _ = run(kind, args.batches, args.inflight, False)
        stt = eng.stats()
        out[kind] = {"lone_batch_us_median": round(float(np.median(per)) * 1e6, 2),
                     "lone_submit_us_median": round(float(np.median(s_d)) * 1e6, 2),
                     "lone_wait_us_median": round(float(np.median(w_d)) * 1e6, 2),
                     "lone_checks_per_s": round(args.batch / float(np.median(per)), 1),
                     "inflight": args.inflight, "batches": args.batches,
                     "pipelined_checks_per_s": round(args.batches * args.batch / dt8, 1),
                     "pipelined_us_per_batch": round(dt8 / args.batches * 1e6, 2),
                     "aql_batches": int(stt["aql_batches"]), "label_checks": int(stt["label_checks"]),
                     "slot_checks": int(stt["slot_checks"])}
        print(json.dumps({kind: out[kind]}), file=sys.stderr, flush=True)
    same = all((pins[k][1] == outs[k][0].cpu().numpy()).all() and (pins[k][2] == outs[k][1].cpu().numpy()).all()
               for k in range(n_rot)) if "host" in out and "device" in out else None
    out["host_equals_device"] = same
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
