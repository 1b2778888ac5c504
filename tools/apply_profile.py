"""Profile Watch-batch application on the config-5 graph: load, then apply --batches update
batches of --churn x tuples each, timing every gck_apply_updates call (run under
rocprofv3 --hip-trace --kernel-trace --stats to see where the time goes)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--churn", type=float, default=0.001)
    args = ap.parse_args()
    import torch
    from gochugaru_amd.engine import Engine
    from tests import synth_configs as S
    dev = torch.device("cuda", 0)
    M = S.Mixed(args.scale, device=dev)
    e = Engine(device=0)
    e.load_schema(M.W.schema)
    for t, n in M.W.counts.items():
        e.reserve_objects(M.W.t(t), n)
    e.begin_snapshot(1)
    cav = e.add_caveat_instance("only_on_tuesday", "")
    keep = []

    def loader(rid, st, sr, n_rows, off, nbr):
        off32 = off.to(torch.int32).contiguous()
        keep.append((off32, nbr))
        e.load_csr(rid, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    M.load(e, loader, cav)
    torch.cuda.synchronize()
    e.commit_snapshot()
    n_up = max(1, int(M.W.n_tuples * args.churn))
    batches = [M.churn(n_up, cav) for _ in range(args.batches)]
    ts = []
    for k, u in enumerate(batches):
        t0 = time.perf_counter()
        e.apply_updates(2 + k, u)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"updates_per_batch": n_up, "apply_ms": [round(t, 3) for t in ts],
                      "median_ms": sorted(ts)[len(ts) // 2]}))


if __name__ == "__main__":
    main()
