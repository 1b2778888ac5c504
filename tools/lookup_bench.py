"""LookupResources / LookupSubjects timing on a bench workload (config 4 by default): the time
of one lookup sweeping every candidate object on the device, and candidates/s."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from gochugaru_amd.engine import ELLIPSIS, Engine
    from tests import synth
    dev = torch.device("cuda", 0)
    G = synth.build(args.tuples, device=dev)
    e = Engine(device=0)
    e.load_schema(synth.SCHEMA)
    e.reserve_objects(synth.T_USER, G.n_users)
    e.reserve_objects(synth.T_GROUP, G.n_groups)
    e.reserve_objects(synth.T_DOC, G.n_docs)
    e.begin_snapshot(1)
    keep = []
    for rel, st, sr, n_rows, off, nbr in G.csrs():
        off32 = off.to(torch.int32).contiguous()
        keep.append(off32)
        e.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    torch.cuda.synchronize()
    e.commit_snapshot()
    items = synth.checks(G, 16, seed=3).view(torch.int32).reshape(16, 5).cpu().numpy()
    out = {"docs": G.n_docs, "users": G.n_users, "resources": [], "subjects": []}
    for k in range(args.reps):
        user = int(items[k, 3])
        t0 = time.perf_counter()
        ids, _ = e.lookup_resources(synth.T_DOC, synth.R_VIEW, synth.T_USER, ELLIPSIS, user)
        dt = time.perf_counter() - t0
        out["resources"].append({"user": user, "found": int(len(ids)), "ms": round(dt * 1e3, 2),
                                 "candidates_per_s": round(G.n_docs / dt)})
        doc = int(items[k, 1])
        t0 = time.perf_counter()
        ids, _ = e.lookup_subjects(synth.T_DOC, doc, synth.R_VIEW, synth.T_USER)
        dt = time.perf_counter() - t0
        out["subjects"].append({"doc": doc, "found": int(len(ids)), "ms": round(dt * 1e3, 2),
                                "candidates_per_s": round(G.n_users / dt)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
