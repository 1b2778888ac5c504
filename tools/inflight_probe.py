"""Throughput of config-4 device batches vs batches in flight, repeated in one process (variance
check): python tools/inflight_probe.py [--tuples 1e9] [--reps 3] [--batches 400]."""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tuples", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--depths", default="1,2,3,4,6,8")
    ap.add_argument("--closure", type=int, default=1)
    ap.add_argument("--n", type=int, default=65536, help="checks per batch (small: the host cost per batch)")
    ap.add_argument("--split", action="store_true", help="time submit and wait calls separately first")
    ap.add_argument("--host", action="store_true", help="pinned host buffers (gck_host_alloc) instead of HBM")
    ap.add_argument("--native", action="store_true", help="the compiled submit/wait loop (libgck_driver.so)")
    ap.add_argument("--both", action="store_true", help="python and native loops alternately in this process")
    ap.add_argument("--engine-streams", action="store_true", help="GCK_SUBMIT_ENGINE_STREAM")
    ap.add_argument("--rot", type=int, default=64, help="distinct pre-generated batches rotated through")
    ap.add_argument("--workspaces", type=int, default=0, help="engine workspaces (0 = the largest depth)")
    ap.add_argument("--queues", type=int, default=0, help="GPU_MAX_HW_QUEUES (0 = default)")
    args = ap.parse_args()
    if args.queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.queues)
    import torch
    from gochugaru_amd.engine import Engine
    from tests import synth
    dev = torch.device("cuda", 0)
    G = synth.build(args.tuples, device=dev)
    depths = [int(x) for x in args.depths.split(",")]
    eng = Engine(device=0, workspaces=args.workspaces or max(depths), closure=bool(args.closure))
    eng.load_schema(synth.SCHEMA)
    eng.reserve_objects(synth.T_USER, G.n_users)
    eng.reserve_objects(synth.T_GROUP, G.n_groups)
    eng.reserve_objects(synth.T_DOC, G.n_docs)
    eng.begin_snapshot(1)
    keep = []
    for rel, st, sr, n_rows, off, nbr in G.csrs():
        off32 = off.to(torch.int32).contiguous()
        keep.append((off32, nbr))
        eng.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    torch.cuda.synchronize()
    eng.commit_snapshot()
    n = args.n
    R = args.rot
    rot = [synth.checks(G, n, seed=3000 + k) for k in range(R)]
    outs = [(torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.int32, device=dev))
            for _ in range(R)]
    streams = [torch.cuda.Stream(dev) for _ in range(max(depths))]
    torch.cuda.synchronize()
    if args.host:
        from gochugaru_amd.engine import ITEM_DTYPE
        import numpy as np
        hrot = []
        for b in rot[:16]:
            a = eng.host_array(n, ITEM_DTYPE)
            a[:] = b.cpu().numpy().view(ITEM_DTYPE).reshape(-1)
            hrot.append((a, eng.host_array(n, np.uint8), eng.host_array(n, np.int32)))

    cursor = [0]

    def run(depth, nb, native=args.native):
        if native:
            ks = [(cursor[0] + k) % R for k in range(nb)]
            cursor[0] += nb
            eng.run_device_batches([rot[j].data_ptr() for j in ks], [outs[j][0].data_ptr() for j in ks],
                                   [outs[j][1].data_ptr() for j in ks], n, depth,
                                   [streams[k % depth].cuda_stream for k in range(nb)],
                                   engine_streams=args.engine_streams)
            return
        if args.host:
            q = collections.deque()
            for k in range(nb):
                if len(q) >= depth:
                    q.popleft().wait()
                q.append(eng.submit_into(*hrot[k % len(hrot)]))
            while q:
                q.popleft().wait()
            return
        q = collections.deque()
        for k in range(nb):
            if len(q) >= depth:
                q.popleft().wait()
            j = (cursor[0] + k) % R
            q.append(eng.submit(rot[j].data_ptr(), n, outs[j][0].data_ptr(), outs[j][1].data_ptr(), device=True,
                                stream=streams[k % depth].cuda_stream, engine_stream=args.engine_streams))
        cursor[0] += nb
        while q:
            q.popleft().wait()

    def split(depth, nb):  # host seconds inside submit / wait calls
        q = collections.deque()
        ts = tw = 0.0
        pc = time.perf_counter
        for k in range(nb):
            if len(q) >= depth:
                t = pc()
                q.popleft().wait()
                tw += pc() - t
            j = k % 64
            t = pc()
            q.append(eng.submit(rot[j].data_ptr(), n, outs[j][0].data_ptr(), outs[j][1].data_ptr(), device=True,
                                stream=streams[k % depth].cuda_stream))
            ts += pc() - t
        while q:
            q.popleft().wait()
        return ts, tw

    if args.split:
        for d in depths:
            split(d, 20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ts, tw = split(d, args.batches)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"inflight {d}: {dt / args.batches * 1e6:.2f} us/batch, submit {ts / args.batches * 1e6:.2f} us, "
                  f"wait {tw / args.batches * 1e6:.2f} us", flush=True)
    for r in range(args.reps):
        for d in depths:
            for native in ([False, True] if args.both else [args.native]):
                run(d, 20, native)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(d, args.batches, native)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(f"rep {r} inflight {d} {'native' if native else 'python'}: {args.batches * n / dt / 1e6:8.1f} M "
                      f"checks/s  {dt / args.batches * 1e3:.4f} ms/batch", flush=True)
    st = eng.stats()
    print("closure_checks", st["closure_checks"], "bundles", st["bundles"])
    eng.close()


if __name__ == "__main__":
    main()
