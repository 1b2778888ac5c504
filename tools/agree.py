"""Debug tool: GPU vs C-oracle agreement on the config-4 graph, per engine variant.

    python tools/agree.py [--tuples 1e9] [--batches 8] [--variants default,nobidir,wide]

Prints one JSON line per variant: mismatches per batch, the first mismatched items, and
whether two runs of the same batch agree with each other (determinism).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "default": {},
    "nobidir": {"bidir": False},
    "wide": {"wide_only": True},
    "nohash": {"membership_hash": False},
    "nogiant": {"giant_stage": False},
    "bidir-one": {"bidir_both": 1},
    "bundle-1": {"bundle_checks": 1},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e9)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--variants", default="default,nobidir")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--seed0", type=int, default=5000)
    ap.add_argument("--bench-like", action="store_true",
                    help="bench.py's CPU-baseline loop: new items/outputs per batch, no host sync between")
    args = ap.parse_args()
    import torch

    from gochugaru_amd.engine import Engine
    from oracle import corc
    from oracle import spicedb_ref as ref
    from tests import synth

    dev = torch.device("cuda", 0)
    G = synth.build(args.tuples, device=dev)
    H = synth.host_arrays(G)
    ids = corc.Ids(ref.Schema(synth.SCHEMA))
    idx = {(synth.R_MEMBER, synth.T_USER, synth.ELLIPSIS, False): 0,
           (synth.R_MEMBER, synth.T_GROUP, synth.R_MEMBER, False): 1,
           (synth.R_VIEWER, synth.T_GROUP, synth.R_MEMBER, False): 2}
    prog = corc.encode_program(ids, idx)
    tab = corc.make_csr_table([(H["mem_user_off"], H["mem_user_nbr"], None, None, G.n_groups),
                               (H["mem_group_off"], H["mem_group_nbr"], None, None, G.n_groups),
                               (H["viewer_off"], H["viewer_nbr"], None, None, G.n_docs)])
    batches = []
    for k in range(args.batches):
        it = synth.checks(G, args.batch, seed=args.seed0 + k)
        hi = it.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
        cp, ce, _ = corc.check(prog, tab, hi, threads=16)
        batches.append((it, hi, cp, ce))
    print(json.dumps({"graph_tuples": G.n_tuples, "batches": args.batches}), flush=True)
    for name in args.variants.split(","):
        eng = Engine(device=0, profile=args.profile, **VARIANTS[name])
        eng.load_schema(synth.SCHEMA)
        eng.reserve_objects(synth.T_USER, G.n_users)
        eng.reserve_objects(synth.T_GROUP, G.n_groups)
        eng.reserve_objects(synth.T_DOC, G.n_docs)
        eng.begin_snapshot(1)
        keep = []
        for rel, st, sr, n_rows, off, nbr in G.csrs():
            off32 = off.to(torch.int32).contiguous()
            nbr32 = nbr.contiguous()
            keep.append((off32, nbr32))
            eng.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr32.data_ptr(), nbr32.numel(), device=True)
        torch.cuda.synchronize()
        eng.commit_snapshot()
        del keep
        if args.bench_like:
            stream = torch.cuda.current_stream(dev).cuda_stream
            items0 = synth.checks(G, args.batch, seed=1000)
            p0 = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
            e0 = torch.zeros(args.batch, dtype=torch.int32, device=dev)
            for _ in range(23):
                eng.check_bulk_device(items0.data_ptr(), args.batch, p0.data_ptr(), e0.data_ptr(), stream=stream)
            torch.cuda.synchronize()
            for trial in range(3):
                outs = []
                for k in range(args.batches):
                    it = synth.checks(G, args.batch, seed=args.seed0 + k)
                    pk = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
                    ek = torch.zeros(args.batch, dtype=torch.int32, device=dev)
                    eng.check_bulk_device(it.data_ptr(), args.batch, pk.data_ptr(), ek.data_ptr(), stream=stream)
                    outs.append((it, pk, ek))
                torch.cuda.synchronize()
                bad_b = {}
                for k, ((_, hi, cp, ce), (it, pk, ek)) in enumerate(zip(batches, outs)):
                    gp, ge = pk.cpu().numpy(), ek.cpu().numpy()
                    nb = int(((gp != cp) | (ge != ce)).sum())
                    if nb:
                        bad_b[k] = [nb, int((gp == 0).sum())]
                print(json.dumps({"variant": name, "bench_like_trial": trial, "bad_batches": bad_b}), flush=True)
        per, samples, nondet = [], [], 0
        t0 = time.time()
        for it, hi, cp, ce in batches:
            outs = []
            for rep in range(2):
                p = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
                e = torch.zeros(args.batch, dtype=torch.int32, device=dev)
                eng.check_bulk_device(it.data_ptr(), args.batch, p.data_ptr(), e.data_ptr(),
                                      stream=torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                outs.append((p.cpu().numpy(), e.cpu().numpy()))
            nondet += int(((outs[0][0] != outs[1][0]) | (outs[0][1] != outs[1][1])).sum())
            gp, ge = outs[0]
            bad = np.nonzero((gp != cp) | (ge != ce))[0]
            per.append(int(len(bad)))
            for i in bad[: max(0, 6 - len(samples))]:
                samples.append({"res": int(hi[i]["resource_id"]), "subj": int(hi[i]["subject_id"]),
                                "gpu": [int(gp[i]), int(ge[i])], "oracle": [int(cp[i]), int(ce[i])]})
        st = eng.stats()
        print(json.dumps({"variant": name, "mismatches": sum(per),
                          "mismatch_per_batch": {k: v for k, v in enumerate(per) if v}, "nondeterministic": nondet,
                          "samples": samples, "secs": round(time.time() - t0, 1),
                          "deferred": st["deferred"], "deferred_wide": st["deferred_wide"],
                          "bidir_checks": st["bidir_checks"]}), flush=True)
        eng.close()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
