"""Snapshot ingest timing on the config-4 graph shape: (1) interned-tuple
ingest — gck_tuple records in a shuffled (export-stream) order through gck_add_tuples +
gck_commit_snapshot (host radix sort into CSRs, upload, derived device indexes); (2) the on-disk
snapshot cache — gck_save_snapshot, then gck_load_snapshot_file into a fresh engine. The three
engines (device-prebuilt CSRs, tuple ingest, file load) answer the same 64K batch identically.

Usage (GPU box): python tools/ingest_bench.py --tuples 1e8 [--file /tmp/snap.gck]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e8)
    ap.add_argument("--file", default="/tmp/gck_ingest_bench.gck")
    ap.add_argument("--file-only", action="store_true", help="only the snapshot file (save from the prebuilt engine)")
    args = ap.parse_args()
    import torch
    from gochugaru_amd.engine import ELLIPSIS, TUPLE_DTYPE, Engine
    from tests import synth
    from tests.test_gpu_scale import load_engine, run

    G = synth.build(args.tuples, device="cuda")
    items = synth.checks(G, 65536, seed=31)
    ref = load_engine(G)
    p0, e0 = run(ref, items)
    if args.file_only:
        t0 = time.perf_counter()
        ref.save_snapshot(args.file)
        t_save = time.perf_counter() - t0
        n = int(ref.tuple_count)
        ref.close()
        f = Engine(device=0)
        f.load_schema(synth.SCHEMA)
        t0 = time.perf_counter()
        f.load_snapshot_file(args.file)
        torch.cuda.synchronize()
        t_load = time.perf_counter() - t0
        p2, e2 = run(f, items)
        f.close()
        size = os.path.getsize(args.file)
        os.remove(args.file)
        same = bool((p0 == p2).all() and (e0 == e2).all())
        print(json.dumps({"workload": "config4-deep-nested-groups", "tuples": n,
                          "snapshot_file": {"bytes": size, "save_s": round(t_save, 2), "load_s": round(t_load, 2),
                                            "load_tuples_per_s": round(n / t_load)},
                          "same_results_64k": same}))
        assert same
        return
    ref.close()

    H = synth.host_arrays(G)
    parts = []
    for (off, nbr, rel, st, sr) in ((H["mem_user_off"], H["mem_user_nbr"], synth.R_MEMBER, synth.T_USER, ELLIPSIS),
                                    (H["mem_group_off"], H["mem_group_nbr"], synth.R_MEMBER, synth.T_GROUP, synth.R_MEMBER),
                                    (H["viewer_off"], H["viewer_nbr"], synth.R_VIEWER, synth.T_GROUP, synth.R_MEMBER)):
        rows = np.repeat(np.arange(len(off) - 1, dtype=np.uint32), np.diff(off.astype(np.int64)))
        t = np.zeros(len(rows), dtype=TUPLE_DTYPE)
        t["resource_type"] = synth.T_DOC if rel == synth.R_VIEWER else synth.T_GROUP
        t["relation"], t["resource_id"] = rel, rows
        t["subject_type"], t["subject_relation"], t["subject_id"] = st, sr, nbr
        parts.append(t)
    tuples = np.concatenate(parts)
    del parts
    tuples = tuples[np.random.default_rng(5).permutation(len(tuples))]

    e = Engine(device=0)
    e.load_schema(synth.SCHEMA)
    e.reserve_objects(synth.T_USER, G.n_users)
    e.reserve_objects(synth.T_GROUP, G.n_groups)
    e.reserve_objects(synth.T_DOC, G.n_docs)
    t0 = time.perf_counter()
    e.begin_snapshot(1)
    for k in range(0, len(tuples), 1 << 24):  # export pages
        e.add_tuples(tuples[k:k + (1 << 24)])
    t_add = time.perf_counter() - t0
    e.commit_snapshot()
    torch.cuda.synchronize()
    t_ingest = time.perf_counter() - t0
    p1, e1 = run(e, items)

    t0 = time.perf_counter()
    e.save_snapshot(args.file)
    t_save = time.perf_counter() - t0
    size = os.path.getsize(args.file)
    e.close()
    f = Engine(device=0)
    f.load_schema(synth.SCHEMA)
    t0 = time.perf_counter()
    f.load_snapshot_file(args.file)
    torch.cuda.synchronize()
    t_load = time.perf_counter() - t0
    p2, e2 = run(f, items)
    n = int(f.tuple_count)
    f.close()
    os.remove(args.file)
    same = bool((p0 == p1).all() and (e0 == e1).all() and (p0 == p2).all() and (e0 == e2).all())
    print(json.dumps({
        "workload": "config4-deep-nested-groups", "tuples": n,
        "tuple_ingest": {"add_s": round(t_add, 2), "total_s": round(t_ingest, 2),
                         "tuples_per_s": round(n / t_ingest)},
        "snapshot_file": {"bytes": size, "save_s": round(t_save, 2), "load_s": round(t_load, 2),
                          "load_tuples_per_s": round(n / t_load)},
        "same_results_64k": same}))
    assert same


if __name__ == "__main__":
    main()
