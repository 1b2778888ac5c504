"""Watch-batch application latency on the config-4 graph (VERDICT r2 "next" 5):
load the nested-group graph at --tuples, apply --batches Watch batches of --churn x tuples each
(user memberships, group nesting, document viewers; batch --cycle-at closes a cycle in the
hierarchy), time every gck_apply_updates call, and after each batch check one 64K batch on the
device (throughput, and how many checks the one-round stages answered). With --verify the batch
is compared with the C oracle over the host-side state (tests/synth.py NestedChurn).

    python tools/watch_bench.py --tuples 1e9 --batches 3 --cycle-at 2 [--verify]
"""
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
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--churn", type=float, default=0.001)
    ap.add_argument("--cycle-at", type=int, default=-1, help="batch index that closes a hierarchy cycle")
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--mix", default="all", choices=["all", "members", "nesting"],
                    help="all: memberships / nesting / viewers 90/5/5 %%; members: memberships and viewers only "
                         "(95/0/5: the hierarchy unchanged); nesting: nesting only")
    args = ap.parse_args()
    import numpy as np
    import torch
    from oracle import corc
    from tests import synth
    from tests.test_gpu_scale import load_engine, run

    t0 = time.time()
    G = synth.build(args.tuples, device="cuda")
    C = synth.NestedChurn(G, seed=7)
    items = synth.checks(G, 65536, seed=31)
    e = load_engine(G)
    print(f"[watch] loaded {G.n_tuples} tuples in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    out = {"tuples": G.n_tuples, "churn": args.churn, "mix": args.mix, "batches": []}

    def measure(tag):
        e.reset_stats()
        torch.cuda.synchronize()
        t = time.perf_counter()
        gp, ge = run(e, items)
        dt = time.perf_counter() - t
        st = e.stats()
        rec = {"batch": tag, "check_ms": round(dt * 1e3, 3), "one_round_checks": int(st["closure_checks"]),
               "slot_checks": int(st["slot_checks"]), "deferred": int(st["deferred"])}
        if args.verify:
            prog, tab = C.oracle()
            hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
            cp, ce, _ = corc.check(prog, tab, hi, threads=threads)
            rec["oracle_mismatches"] = int(((gp != cp) | (ge != ce)).sum())
            rec["max_depth_errors"] = int((ce == 1).sum())
        return rec

    out["batches"].append(measure("initial"))
    n_up = int(G.n_tuples * args.churn)
    for b in range(args.batches):
        share = {"all": (0.9, 0.05, 0.05), "members": (0.95, 0.0, 0.05), "nesting": (0.0, 1.0, 0.0)}[args.mix]
        ups = C.batch(n_up, cycle=(b == args.cycle_at), share=share)
        torch.cuda.synchronize()
        t = time.perf_counter()
        e.apply_updates(2 + b, ups)
        torch.cuda.synchronize()
        apply_s = time.perf_counter() - t
        rec = measure(b)
        rec["updates"] = int(len(ups))
        rec["apply_s"] = round(apply_s, 3)
        rec["cycle"] = b == args.cycle_at
        out["batches"].append(rec)
        print(f"[watch] {rec}", file=sys.stderr, flush=True)
    print(json.dumps(out))
    e.close()


if __name__ == "__main__":
    main()
