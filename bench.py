"""bench.py — permission checks/sec at batch 64K on the 1B-tuple deep nested-group graph.

Workload (BASELINE.json metric "permission checks/sec (whole node) at batch 64K, 1B tuples;
HBM GB/s vs peak"; config 4 of BASELINE.json configs, replicated-graph mode, which fits one
MI355X): tests/synth.py builds the seeded graph on every rank (identical, replicated), the
engine ingests it through the C ABI (gck_load_csr), and each step is one 65,536-item
``doc#view@user`` request per GPU. `value` follows this bench's contract: the requests' items are
resident in HBM when the timed region starts and the results stay there — 2,000 distinct
pre-generated requests, 8 in flight (gck_check_submit / gck_check_wait, the compiled loop of
libgck_driver.so), barrier + synchronize on both sides, max over ranks. BASELINE.md:40-41 /
SURVEY §8(d) define the step with its transfers: the same requests start in host memory (pinned,
gck_host_alloc: where a cgo caller builds its requests), cross to the GPU, are checked, and the
results end in host memory — timed the same way and reported in the same line as
`baseline_pipelined` (8 in flight) and `baseline_step` (one batch alone, median over >= 20 batches
after 3 warm-up ones). With N ranks every 64K request is cut into N contiguous slices, rank r
checking slice r against its replica (no collective on the data path): the node figure at batch
64K, strong scaling, value = (checks of the requests) / (max-over-ranks time); `weak_scaling`
times every rank on its own 64K requests beside it. Configs 2, 3 run the same way; 5
(``--config mixed``) checks a device-resident batch per rank and step beside its Watch batch.

Also printed: the roofline of the dominant kernel (SURVEY.md §8d algorithmic bytes of a batch,
counted by the oracle's counting mode, / the mean stage-A launch time of device-resident batches
one at a time after the timed region, from the queue's dispatch timestamps; `traffic` = HBM bytes
per batch from rocprofv3 PMC), the host link's share (`pcie`), the process's placement on the
GPU's NUMA node (`host_placement`), and a CPU baseline: the C restatement oracle (16 host
threads) on a bounded sample of the same batches, ~15 s of CPU work, with every sampled check
compared against the GPU's answer (`oracle_agreement`).
"""
import argparse
import collections
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
BATCH = 65536


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a 64K batch takes ~6 us of device time with 8 in flight: 2000 timed batches (~12 ms) keep
    # the pipeline's fill and drain (a few batches' worth) and host jitter out of the figure
    # (configs 2, 3, 5: 200 / 20 — their steps are longer and config 5 pre-generates a Watch
    # batch or 64K contexts per step)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--tuples", type=float, default=1e9, help="graph size (1e9 = BASELINE config)")
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline time budget")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-labels", action="store_true",
                    help="engine without the label-join stage (GCK_FLAG_NO_LABELS): the A/B of the join")
    ap.add_argument("--cpu-max-batches", type=int, default=400)
    ap.add_argument("--no-oracle", action="store_true", help="skip the host oracle (no roofline, no CPU baseline)")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC HBM bytes per batch (tools/gpu.sh profile, calibrated by tools/gather_probe)")
    ap.add_argument("--host-steps", type=int, default=200, help="PCIe-inclusive host-buffer steps (0 = skip)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="check batches in flight (gck_check_submit on this many streams): the next batch's "
                         "kernels fill the tail of the previous one; 1 = one batch at a time (default: 8 for "
                         "config 4, 3 for the others)")
    ap.add_argument("--no-profile", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--trace-loop", action="store_true",
                    help="record when each timed batch's submit and wait returned (compiled loop; `loop_trace`)")
    ap.add_argument("--driver", default="native", choices=["native", "python"],
                    help="who runs the submit/wait loop over the device batches: native = the compiled loop "
                         "of libgck_driver.so (what a cgo caller runs), python = one ctypes call per submit/wait")
    ap.add_argument("--engine-streams", type=int, default=1,
                    help="1: device batches run on the engine's workspace streams (GCK_SUBMIT_ENGINE_STREAM) "
                         "instead of the caller's streams")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (0 = the runtime's default, 4)")
    ap.add_argument("--bundle-checks", type=int, default=0)
    ap.add_argument("--bundle-frontier", type=int, default=0)
    ap.add_argument("--bundle-visited", type=int, default=0)
    ap.add_argument("--bundle-waves", type=int, default=0)
    ap.add_argument("--bundle-budget", type=int, default=0)
    ap.add_argument("--giant-slots", type=int, default=0)
    ap.add_argument("--wide-only", action="store_true")
    ap.add_argument("--no-giant", action="store_true", help="deferred checks go to the grid-wide path")
    ap.add_argument("--no-bidir", action="store_true", help="forward-only search (no bidirectional checks)")
    ap.add_argument("--bidir-both", type=int, default=0, help="expand both sides while <= this many entries")
    ap.add_argument("--partitioned", action="store_true",
                    help="config 4 partitioned mode: each rank holds the rows it owns; the ranks check one "
                         "global batch (batch x ranks) with a per-level all-to-all (gochugaru_amd/partition.py)")
    ap.add_argument("--part-backend", default="nccl", help="exchange backend in --partitioned mode (nccl = RCCL)")
    ap.add_argument("--share-gpu", action="store_true", help="every rank on cuda:0 (a one-GPU rehearsal with gloo)")
    ap.add_argument("--config", default="nested", choices=["nested", "gdocs", "github", "mixed", "quota"],
                    help="nested = BASELINE config 4 (the headline, default); gdocs / github = configs 2 / 3 "
                         "(tests/synth_configs.py) at --scale; mixed = config 5 (config 2 + 10 %% caveated "
                         "tuples, check contexts, one Watch batch of --churn x tuples applied per step); quota = "
                         "config 5 with 32K per-relationship caveat contexts x one context per request")
    ap.add_argument("--selftest", action="store_true", help="launcher / rank bookkeeping only (no GPU; tests)")
    ap.add_argument("--coalesce", type=int, default=1,
                    help="strong scaling: a rank checks its slices of up to this many consecutive requests in one "
                         "dispatch (default 1: one dispatch per request slice, so `value` at N > 1 is strong scaling "
                         "of one 64K request; with N > 1 the figure at coalesce = N is reported as `coalesced`)")
    ap.add_argument("--resident", type=int, default=0,
                    help="1: the engine's resident closure join (GCK_FLAG_RESIDENT, resident.inc): requests are "
                         "posted to one long-running launch instead of a dispatch each")
    ap.add_argument("--churn", type=float, default=0.001, help="config 5: updates per step, as a fraction of tuples")
    ap.add_argument("--watch-stage", type=int, default=2,
                    help="config 5: Watch batches staged ahead of the one a step applies (gck_watch_stage: grouped "
                         "on the engine's staging threads beside the apply; a consumer holding that many further "
                         "responses); 0 = gck_apply_updates")
    ap.add_argument("--scale", type=float, default=1.0, help="configs 2 / 3: 1.0 = 10M / 100M tuples")
    args = ap.parse_args()
    nested = args.config == "nested"
    pipelined = args.config in ("nested", "gdocs", "github")  # batches in flight through the compiled loop
    if args.steps is None:
        args.steps = 2000 if nested else (1000 if pipelined else 200)
    if args.warmup is None:
        args.warmup = 100 if nested else 20
    if args.inflight is None:
        args.inflight = 8 if pipelined else 3
    # untimed batches before the timed region: at least --warmup, and at least two per batch in
    # flight, so that every workspace, stream and hardware queue has run a batch before t0
    args.warm = max(args.warmup, 2 * max(1, args.inflight))
    return args


class Workload:
    """One benchmark graph: schema, CSRs in the engine's id space, a check generator and the C
    oracle's view of the same arrays."""

    def __init__(self, args, dev):
        import torch
        from oracle import corc
        from oracle import spicedb_ref as ref
        self.kind = args.config
        if args.config == "nested":
            from tests import synth
            G = self.G = synth.build(args.tuples, device=dev)
            self.schema = synth.SCHEMA
            self.reserve = [(synth.T_USER, G.n_users), (synth.T_GROUP, G.n_groups), (synth.T_DOC, G.n_docs)]
            self.csrs = G.csrs()
            self.union_only = True
            self.data = "synthetic (tests/synth.py, seed 20251003): deep nested groups, 25 layers, Pareto(2.1) group sizes"
            self.cfg = {"workload": "config4-deep-nested-groups-" + ("partitioned" if args.partitioned else "replicated"),
                        "users": G.n_users, "groups": G.n_groups, "docs": G.n_docs}
            self._checks = lambda n, seed: synth.checks(G, n, seed=seed)

            def oracle():
                H = synth.host_arrays(G)
                ids = corc.Ids(ref.Schema(synth.SCHEMA))
                idx = {(synth.R_MEMBER, synth.T_USER, synth.ELLIPSIS, False): 0,
                       (synth.R_MEMBER, synth.T_GROUP, synth.R_MEMBER, False): 1,
                       (synth.R_VIEWER, synth.T_GROUP, synth.R_MEMBER, False): 2}
                tab = corc.make_csr_table([(H["mem_user_off"], H["mem_user_nbr"], None, None, G.n_groups),
                                           (H["mem_group_off"], H["mem_group_nbr"], None, None, G.n_groups),
                                           (H["viewer_off"], H["viewer_nbr"], None, None, G.n_docs)])
                return corc.encode_program(ids, idx), tab
            self.oracle = oracle
        elif args.config == "quota":
            from tests import synth_configs
            Q = self.Q = synth_configs.Quota(args.scale, device=dev)
            W = Q.W
            self.schema = W.schema
            self.reserve = [(W.t(t), n) for t, n in W.counts.items()]
            self.csrs = None
            self.union_only = True
            self.data = (f"synthetic (tests/synth_configs.py Quota, seed 20251003, scale {args.scale}): config-2 graph, "
                         f"10% of folder/doc viewer+editor user tuples caveated with quota(limit, used) "
                         f"{{used < limit}}, each relationship storing one of {len(Q.limits)} distinct limits "
                         f"(as many partial caveat instances); every check carries its own {{\"used\": U}} "
                         f"context (10% none): {args.batch} contexts per batch")
            self.cfg = {"workload": W.name, **{k + "s": v for k, v in W.counts.items()},
                        "caveat_instances": len(Q.limits), "contexts_per_batch": args.batch}
            self._checks = lambda n, seed: Q.checks(n, seed)
            self.oracle = None
        elif args.config == "mixed":
            from tests import synth_configs
            M = self.M = synth_configs.Mixed(args.scale, device=dev)
            W = M.W
            self.schema = W.schema
            self.reserve = [(W.t(t), n) for t, n in W.counts.items()]
            self.csrs = None
            self.union_only = True
            self.data = (f"synthetic (tests/synth_configs.py Mixed, seed 20251003, scale {args.scale}): config-2 graph, "
                         f"10% of folder/doc viewer+editor user tuples with only_on_tuesday; checks 25% tuesday / "
                         f"25% monday / 50% no context; each step applies one Watch batch of {args.churn:.2%} of the "
                         f"tuples (CREATE/TOUCH/DELETE 45/45/10) before its check batch")
            self.cfg = {"workload": W.name, **{k + "s": v for k, v in W.counts.items()}}
            self._checks = lambda n, seed: M.checks(n, seed)
            self.oracle = None
        else:
            from tests import synth_configs
            W = synth_configs.CONFIGS[args.config](args.scale, device=dev)
            self.schema = W.schema
            self.reserve = [(W.t(t), n) for t, n in W.counts.items()]
            self.csrs = W.csrs
            self.union_only = args.config == "gdocs"
            self.data = (f"synthetic (tests/synth_configs.py {args.config}, seed 20251003, scale {args.scale}): "
                         + ("Google-Docs schema, nested groups, folder forest, parent arrows, public docs"
                            if args.config == "gdocs" else
                            "GitHub schema, nested teams, exclusion (banned), intersection and all() over org membership"))
            self.cfg = {"workload": W.name, **{k + "s": v for k, v in W.counts.items()}}
            self._checks = lambda n, seed: synth_configs.checks(W, n, seed=seed)
            self.oracle = W.oracle
        torch.cuda.synchronize()

    def checks(self, n, seed):
        return self._checks(n, seed)

    def load(self, eng, keep):
        import torch
        for t, n in self.reserve:
            eng.reserve_objects(t, n)

        def loader(rel, st, sr, n_rows, off, nbr):
            off32 = off.to(torch.int32).contiguous()
            nbr32 = nbr.contiguous()
            keep.append((off32, nbr32))
            eng.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr32.data_ptr(), nbr32.numel(), device=True)
        if self.kind == "quota":
            self.Q.load(eng, loader)
        elif self.kind == "mixed":
            self.cav = eng.add_caveat_instance("only_on_tuesday", "")
            self.M.load(eng, loader, self.cav)
        else:
            for c in self.csrs:
                loader(*c)


def host_cpus():
    """The host CPUs this process may use: its affinity mask, capped by a cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us) — nproc / os.cpu_count() report the
    whole machine. Returns (usable, nproc)."""
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        usable = min(usable, max(1, int(quota)))
    return usable, nproc


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per GPU) with the
    torch.distributed environment torchrun would give them, before this process touches a GPU,
    and exit with the first failing rank's status. Rank 0's stdout (the JSON line) passes through."""
    import socket
    import subprocess
    share = "--share-gpu" in sys.argv
    if not share and "--selftest" not in sys.argv:
        import torch  # counting devices does not initialise the GPU
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible; refusing to run fewer ranks",
                  file=sys.stderr, flush=True)
            sys.exit(2)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c
    if rc != 0:
        print(f"bench.py --gpus {n}: a rank failed (status {rc})", file=sys.stderr, flush=True)
    sys.exit(rc if rc > 0 else (1 if rc else 0))


def init_group(backend):
    """torch.distributed's process group, its first collective run: Gloo announces its connections
    on stdout when they are made, and stdout is kept for the one JSON line."""
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group(backend)
        if backend == "gloo":
            dist.barrier()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def selftest(args):
    """The multi-rank bookkeeping without a GPU (tests/test_bench_launch.py): every rank joins the
    gloo group, takes its slice of the request the node figure shares (strong scaling), times a
    dummy step, and rank 0 prints the JSON line's rank-dependent keys with every rank's slice."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        init_group("gloo")
    from gochugaru_amd.sharded import slices
    b, e = slices(args.batch, world)[rank]
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    sl = torch.tensor([b, e], dtype=torch.int64)
    every = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_gather(every, sl)
    else:
        every = [sl]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "max_over_ranks": float(t[0]), "slice": [b, e],
                          "slices": [[int(x[0]), int(x[1])] for x in every], "global_batch": args.batch,
                          "checks_per_step": {"strong": args.batch, "weak": world * args.batch}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def roofline_line(tj, tj_path, b_alg, ms, steps, job_s):
    """The roofline object of the dominant kernel. `achieved` = the HBM bytes one launch moves —
    rocprofv3 FETCH_SIZE + WRITE_SIZE of this workload's batches on this round's code (`tj`,
    tools/traffic_summary.py) — over the mean solo launch time `ms`; `frac` = that / 8 TB/s, and
    `frac_job` the same bytes of every timed batch over the device-resident timed region `job_s`.
    SURVEY §8(d)'s algorithmic bytes (`alg_bytes_per_launch`) charge the forward search the joins
    replace with precomputed slots, so their ratio to the time is no HBM fraction and is not
    reported as one. The joins are random-line bound: `random_lines` compares the 64-B accesses per
    launch (FETCH_SIZE / 64: every random read of <= 64 B counts one line, tools/gather_probe) with
    the random-line rate tools/gather_probe measured in the same profile run."""
    root = os.path.dirname(os.path.abspath(__file__))
    traffic = tj.get("hbm_bytes_per_batch") if tj else None
    src = os.path.relpath(tj_path, root) if tj else None
    sec = ms * 1e-3
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic, "traffic_source": src,
            "alg_bytes_per_launch": int(b_alg),
            "alg_note": "SURVEY §8(d) algorithmic bytes (25 B per check + 8 B per row + 4 B per edge of the oracle's "
                        "forward BFS): the joins answer from precomputed slots and never perform that BFS, so these "
                        "bytes over the launch time are not an HBM fraction (they exceed the peak at job level); "
                        "achieved / frac use the measured bytes"}
    if traffic:
        roof["achieved"] = round(traffic / sec / 1e9, 3)
        roof["frac"] = round(traffic / sec / 1e9 / HBM_PEAK_GBS, 6)
        if job_s:
            roof["achieved_job"] = round(traffic * steps / job_s / 1e9, 3)
            roof["frac_job"] = round(traffic * steps / job_s / 1e9 / HBM_PEAK_GBS, 6)
        fetch = sum((tj.get("fetch_bytes_raw_per_launch") or {}).get(k, 0) for k in tj.get("kernels", []))
        # the ceiling: the best random-access rate tools/gather_probe measured on the box (reads of 4
        # to 64 B; the joins' 16-B chunk loads, four lanes to a 64-B slot line, exceed its 64-B figure)
        ceil = max((tj.get("line_ceiling") or {}).values(), default=None)
        if fetch:
            lines = fetch / 64.0
            rl = {"per_launch": int(lines), "solo_G_per_s": round(lines / sec / 1e9, 2)}
            if job_s:
                rl["job_G_per_s"] = round(lines * steps / job_s / 1e9, 2)
            if ceil:
                rl["ceiling_G_per_s"] = ceil
                rl["frac_solo"] = round(rl["solo_G_per_s"] / ceil, 4)
                if job_s:
                    rl["frac_job"] = round(rl["job_G_per_s"] / ceil, 4)
                rl["ceiling_source"] = ("tools/gather_probe: the best rate of random aligned 4-64 B reads from a table "
                                        "16x the Infinity Cache (per width: " + json.dumps(tj.get("line_ceiling")) + ")")
            roof["random_lines"] = rl
    else:  # no counter pass for this workload on this round's code: the algorithmic figure, flagged
        roof["achieved"] = round(b_alg / sec / 1e9, 3)
        roof["frac"] = round(b_alg / sec / 1e9 / HBM_PEAK_GBS, 6)
        roof["achieved_basis"] = "algorithmic bytes (no PMC pass found for this workload)"
    return roof


def progress(msg):
    """Progress on stderr (long runs under a profiler must keep writing)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args.gpus)  # does not return
    if args.selftest:
        return selftest(args)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world_env:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.hw_queues:  # before the HIP runtime starts
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # replicated mode: gloo for the timing barriers / reductions only (no data-path collective);
        # partitioned mode: the per-level exchange (RCCL over xGMI by default)
        init_group(args.part_backend if args.partitioned else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # the submitting thread (and so the writer of each request's items) on the GPU's NUMA node
    from gochugaru_amd.engine import pin_to_device_node
    placement = pin_to_device_node(local)

    from gochugaru_amd.engine import Engine, ITEM_DTYPE

    t0 = time.time()
    WL = Workload(args, dev)
    t_gen = time.time() - t0
    progress(f"workload generated in {t_gen:.1f}s")

    t0 = time.time()
    depth = max(1, args.inflight)
    # events only for the solo phase after the timed region (and the configs timed without one)
    solo_profile = WL.kind not in ("mixed", "quota") and not args.partitioned
    eng = Engine(device=local, profile=not args.no_profile and not solo_profile, workspaces=max(2, depth),
                 labels=not args.no_labels,
                 max_batch=args.batch * world if args.partitioned else args.batch, wide_only=args.wide_only,
                 bundle_checks=args.bundle_checks, bundle_frontier=args.bundle_frontier,
                 bundle_visited=args.bundle_visited, bundle_waves_per_cu=args.bundle_waves,
                 bundle_budget=args.bundle_budget, giant_slots=args.giant_slots,
                 giant_stage=not args.no_giant, bidir=not args.no_bidir, bidir_both=args.bidir_both,
                 resident=bool(args.resident))
    if args.partitioned:
        eng.set_partition(rank, world)
    eng.load_schema(WL.schema)
    eng.begin_snapshot(1)
    keep = []
    WL.load(eng, keep)
    torch.cuda.synchronize()
    eng.commit_snapshot()
    t_load = time.time() - t0
    progress(f"snapshot committed in {t_load:.1f}s")
    n_tuples = eng.tuple_count
    dev_bytes = eng.device_bytes

    stream = torch.cuda.current_stream(dev).cuda_stream
    run_steps = None  # the nested workload's compiled submit/wait loop (--driver native)
    loop_s = {"s": None}  # the compiled loop's own wall time of the last phase (first submit to last wait)
    if args.partitioned:
        # one global batch: every rank's 64K checks, the same items on every rank
        from gochugaru_amd.partition import PartitionedChecker, RcclPartitionedChecker
        # nccl: the level loop and its RCCL exchange inside libgck (gck_part_check); else the
        # Python driver over torch.distributed (gloo rehearsals)
        if args.part_backend == "nccl":
            # RCCL prints its version banner on stdout when the communicator starts: keep stdout
            # for the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                pc = RcclPartitionedChecker(eng)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
        else:
            pc = PartitionedChecker(eng)
        items = torch.cat([WL.checks(args.batch, 1000 + r) for r in range(world)])
        n_global = args.batch * world
        out = {"perm": torch.zeros(n_global, dtype=torch.uint8, device=dev),
               "err": torch.zeros(n_global, dtype=torch.int32, device=dev)}
        pc_out = (out["perm"], out["err"]) if args.part_backend == "nccl" else None

        def step():
            if pc_out is not None:  # (the RCCL checker writes into the preallocated results)
                pc.check(items, n_global, out=pc_out)
            else:
                out["perm"], out["err"] = pc.check(items, n_global)
    elif WL.kind == "mixed":
        # config 5: per step one Watch batch (pre-generated: the stream's arrivals) then one check
        # batch with contexts, at the revision the batch moved the snapshot to
        from tests.synth_configs import CONTEXTS
        # every step its own check batch (no step re-reads a batch another step left in the caches)
        m_rot = [WL.checks(args.batch, 1000 + 100003 * rank + k) for k in range(args.warm + args.steps)]
        items = m_rot[0]
        perm = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
        err = torch.zeros(args.batch, dtype=torch.int32, device=dev)
        # The check batch is submitted and left running: the next step's Watch batch validates,
        # groups and stages its updates beside it and drains it before it touches the snapshot
        # (delta.inc device_apply), so every check batch runs on the revision its step applied
        from gochugaru_amd.engine import Contexts
        n_up = max(1, int(n_tuples * args.churn))
        batches = [WL.M.churn(n_up, WL.cav) for _ in range(args.warm + args.steps)]
        rev = {"r": 1, "k": 0, "apply_s": 0.0, "submit_s": 0.0, "wait_s": 0.0, "pending": None, "tq": []}
        m_ctx = Contexts(CONTEXTS)

        def step():
            t_a = time.perf_counter()
            rev["r"] += 1
            k = rev["k"]
            if args.watch_stage:
                # a Watch consumer holding the next `watch_stage` responses stages them (the
                # engine's staging threads validate and group them) before it applies this one:
                # every step still groups, merges and publishes one whole batch, the later batches'
                # grouping beside this one's merge. After the first step each step stages exactly
                # one batch (the last steps stage the final batch again, discarded after the run),
                # so the timed region holds as many groupings as applies
                tq = rev["tq"]
                while len(tq) < args.watch_stage + 1:
                    tq.append(eng.stage_updates(batches[min(k + len(tq), len(batches) - 1)]))
                eng.apply_staged(rev["r"], tq.pop(0))
            else:
                eng.apply_updates(rev["r"], batches[k])
            rev["k"] += 1
            rev["apply_s"] += time.perf_counter() - t_a
            t_s = time.perf_counter()
            # on the engine's streams: the label join with its caveat plane is dispatched into the
            # engine's HSA queues (aql.inc), the contexts' Ctx in the kernarg block
            b = eng.submit(m_rot[rev["k"] - 1].data_ptr(), args.batch, perm.data_ptr(), err.data_ptr(), device=True,
                           stream=stream, contexts=m_ctx, engine_stream=bool(args.engine_streams))
            rev["submit_s"] += time.perf_counter() - t_s
            if rev["pending"] is not None:
                t_w = time.perf_counter()
                rev["pending"].wait()  # (already finished by the apply above)
                rev["wait_s"] += time.perf_counter() - t_w
            rev["pending"] = b

        def drain():
            if rev["pending"] is not None:
                rev["pending"].wait()
                rev["pending"] = None
            if rev["k"] >= len(batches):
                for t in rev["tq"]:
                    eng.discard_staged(t)
                rev["tq"] = []
    elif WL.kind == "quota":
        # per step one batch with its own 64K contexts (pre-generated, rotated): the contexts are
        # parsed, the walk records the (instance, context) pairs it meets, the host evaluates
        # them and the batch runs again — all inside the step
        from gochugaru_amd.engine import Contexts  # marshalled ahead, as the items are
        q_rot = [WL.checks(args.batch, 1000 + 100003 * rank + k) for k in range(args.warm + args.steps)]
        q_rot = [(it, used, Contexts(texts)) for it, used, texts in q_rot]
        q_out = [(torch.zeros(args.batch, dtype=torch.uint8, device=dev),
                  torch.zeros(args.batch, dtype=torch.int32, device=dev)) for _ in q_rot]
        torch.cuda.synchronize()
        cursor = {"k": 0}

        def step():
            k = cursor["k"]
            cursor["k"] += 1
            it, _, texts = q_rot[k]
            eng.check_bulk_device(it.data_ptr(), args.batch, q_out[k][0].data_ptr(), q_out[k][1].data_ptr(),
                                  stream=stream, contexts=texts)
    else:
        # distinct requests of args.batch checks, rotated through warm-up and timed steps (no step
        # re-reads a batch a previous step left in the caches), each with its own result buffers;
        # up to `depth` of them in flight on as many streams (gck_check_submit / gck_check_wait).
        # The node figure (BASELINE "whole node at batch 64K"): every request is the
        # same on every rank and each rank checks its contiguous slice of it (sharded.slices, as
        # DistributedChecker does), so N GPUs share one 64K request — strong scaling; at N = 1
        # the slice is the whole request. Weak scaling (every rank its own 64K requests) is
        # timed after it as a secondary key.
        from gochugaru_amd.sharded import slices
        s_lo, s_hi = slices(args.batch, world)[rank]
        n_slice = s_hi - s_lo
        n_rot = args.warm + args.steps
        # (one device array for every rotated slice and one per result plane: a rank's slices of
        # consecutive requests lie back to back, so several can go in one dispatch)
        rot_all = torch.cat([WL.checks(args.batch, 1000 + k)[s_lo:s_hi] for k in range(n_rot)]).contiguous()
        rot = [rot_all[k * n_slice:(k + 1) * n_slice] for k in range(n_rot)]
        perm_all = torch.zeros(n_rot * n_slice, dtype=torch.uint8, device=dev)
        err_all = torch.zeros(n_rot * n_slice, dtype=torch.int32, device=dev)
        outs = [(perm_all[k * n_slice:(k + 1) * n_slice], err_all[k * n_slice:(k + 1) * n_slice]) for k in range(n_rot)]
        # Coalescing (strong scaling): with N ranks a request leaves each rank ~batch/N checks, and
        # a dispatch that small is bound by its own latency, not by the GPU; a rank therefore checks
        # its slices of up to `coal` consecutive requests in one dispatch (they are contiguous), as a
        # node-level dispatcher batches what arrives for each GPU. The timed region still holds
        # exactly the steps' requests. coal_for(count): the largest divisor of count <= coal.
        coal_max = max(1, args.batch // max(1, n_slice))
        coal = max(1, min(args.coalesce, coal_max))
        coal_for = lambda count, cap=None: max(c for c in range(1, (cap or coal) + 1) if count % c == 0)
        streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        # `value`'s path (BASELINE.md:40-41, SURVEY §8d: items H2D + kernels + results D2H): the
        # same requests in host memory — pinned, from gck_host_alloc, where a cgo caller builds its
        # requests — and the results back into host memory. One allocation per array, every
        # batch its own slice (no step re-reads a batch another step read).
        h_items = eng.host_array(n_rot * n_slice, ITEM_DTYPE)
        h_perm = eng.host_array(n_rot * n_slice, np.uint8)
        h_err = eng.host_array(n_rot * n_slice, np.int32)
        for k in range(n_rot):
            h_items[k * n_slice:(k + 1) * n_slice] = rot[k].cpu().numpy().view(ITEM_DTYPE).reshape(-1)
        h_ptr = lambda a, k: a.ctypes.data + k * n_slice * a.itemsize
        torch.cuda.synchronize()
        cursor = {"k": 0}
        pending = collections.deque()

        def step():
            k = cursor["k"]
            cursor["k"] += 1
            if len(pending) >= depth:
                pending.popleft().wait()
            sl = slice(k * n_slice, (k + 1) * n_slice)
            pending.append(eng.submit_into(h_items[sl], h_perm[sl], h_err[sl]))

        def drain():
            while pending:
                pending.popleft().wait()

        if args.driver == "native":
            # the same submit/wait loop, run by the compiled caller (libgck_driver.so) over the
            # steps of one phase: run_steps(count) checks the next `count` rotated batches; the
            # loop's arguments are marshalled before the phase (prepare), so a timed phase is the C
            # loop alone
            prepared = {}

            def prepare(count):
                k0 = cursor["k"] + sum(c for c, _ in prepared.values())
                cc = coal_for(count)
                ks = range(k0, k0 + count, cc)
                prepared[len(prepared)] = (count, eng.prepare_batches(
                    [h_ptr(h_items, k) for k in ks], [h_ptr(h_perm, k) for k in ks], [h_ptr(h_err, k) for k in ks],
                    n_slice * cc, depth, host=True))

            def run_steps(count):
                c, run = prepared.pop(min(prepared))
                assert c == count
                cursor["k"] += count
                loop_s["s"] = run.run()

            prepare(args.warm)
            prepare(args.steps)

    native = run_steps is not None
    if native:
        run_steps(args.warm)
    else:
        for _ in range(args.warm):
            step()
    if WL.kind != "quota" and not args.partitioned:
        drain()
    torch.cuda.synchronize()
    eng.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    trace = None
    if native and args.trace_loop:  # per-batch submit / wait return times of the timed loop
        from gochugaru_amd.engine import _driver
        import ctypes
        trace = np.zeros(2 * args.steps, dtype=np.float64)
        _driver().gckd_set_trace(trace.ctypes.data_as(ctypes.c_void_p), args.steps)
    if WL.kind == "mixed":
        rev["apply_s"] = rev["submit_s"] = rev["wait_s"] = 0.0  # (the Watch share is of the timed steps only)
    t0 = time.perf_counter()
    if native:
        run_steps(args.steps)
    else:
        for _ in range(args.steps):
            step()
    if WL.kind != "quota" and not args.partitioned:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if WL.kind == "mixed":
        rev["apply_timed"], rev["submit_timed"], rev["wait_timed"] = rev["apply_s"], rev["submit_s"], rev["wait_s"]
    if trace is not None:
        _driver().gckd_set_trace(None, 0)
    progress(f"timed region: {args.steps} steps in {elapsed * 1e3:.2f} ms"
             + (f" (compiled loop {loop_s['s'] * 1e3:.3f} ms)" if native else ""))
    pipelined = native and WL.kind in ("nested", "gdocs", "github") and not args.partitioned
    # the same requests device-resident (items already in HBM, results left there): `value`, what
    # the engine sustains without the PCIe transfers. The timed batches again, after warm-up batches
    # of their own, on the engine's streams.
    device_resident = None
    if pipelined:
        def mkd(k0, count, cap=None):
            cc = coal_for(count, cap)
            ks = range(k0, k0 + count, cc)
            return eng.prepare_batches([rot[k].data_ptr() for k in ks], [outs[k][0].data_ptr() for k in ks],
                                       [outs[k][1].data_ptr() for k in ks], n_slice * cc, depth,
                                       [streams[j % depth].cuda_stream for j in range(len(ks))],
                                       engine_streams=bool(args.engine_streams))
        d_warm, d_run = mkd(0, args.warm), mkd(args.warm, args.steps)
        torch.cuda.synchronize()
        d_warm.run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        td = time.perf_counter()
        d_loop = d_run.run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        td = time.perf_counter() - td
        if world > 1:
            tt = torch.tensor([td], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            td = float(tt[0])
        device_resident = {"value": round(args.batch * args.steps / td, 1), "unit": "checks/s", "seconds": td,
                           "ms_per_step": round(td / args.steps * 1e3, 4), "compiled_loop_ms": round(d_loop * 1e3, 4),
                           "inflight": depth, "steps": args.steps,
                           "note": "the same rotated requests with the items already in HBM and the results left "
                                   "there (no PCIe in the step): `value`"}
        progress(f"device-resident phase: {td * 1e3:.2f} ms")
    # N > 1: the same device-resident requests with a rank's slices of N consecutive requests in one
    # dispatch (what a node-level dispatcher that aggregates per GPU would do): N x the per-request
    # latency, so reported beside `value`, never as it
    coalesced = None
    if pipelined and world > 1 and args.coalesce == 1 and coal_max > 1:
        c_warm, c_run = mkd(0, args.warm, coal_max), mkd(args.warm, args.steps, coal_max)
        torch.cuda.synchronize()
        c_warm.run()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        tc = time.perf_counter()
        c_run.run()
        torch.cuda.synchronize()
        dist.barrier()
        tc = time.perf_counter() - tc
        tt = torch.tensor([tc], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tc = float(tt[0])
        coalesced = {"value": round(args.batch * args.steps / tc, 1), "unit": "checks/s",
                     "requests_per_dispatch": coal_for(args.steps, coal_max),
                     "checks_per_dispatch": n_slice * coal_for(args.steps, coal_max),
                     "ms_per_step": round(tc / args.steps * 1e3, 4),
                     "note": "device-resident, a rank's slices of consecutive requests checked in one dispatch "
                             "(request aggregation: each request waits for the next ones); not `value`"}
        progress(f"coalesced phase: {tc * 1e3:.2f} ms")
    # weak scaling beside the node figure (N > 1): every rank checks its own whole requests (host
    # buffers, as `value`)
    weak = None
    if pipelined and world > 1:
        n_w = min(args.steps, 500)
        n_wr = n_w + 2 * depth
        w_items = eng.host_array(n_wr * args.batch, ITEM_DTYPE)
        w_perm = eng.host_array(n_wr * args.batch, np.uint8)
        w_err = eng.host_array(n_wr * args.batch, np.int32)
        for k in range(n_wr):
            w_items[k * args.batch:(k + 1) * args.batch] = (
                WL.checks(args.batch, 700000 + 100003 * rank + k).cpu().numpy().view(ITEM_DTYPE).reshape(-1))
        wp = lambda a, k: a.ctypes.data + k * args.batch * a.itemsize
        mkw = lambda ks: eng.prepare_batches([wp(w_items, k) for k in ks], [wp(w_perm, k) for k in ks],
                                             [wp(w_err, k) for k in ks], args.batch, depth, host=True)
        w_warm, w_run = mkw(range(2 * depth)), mkw(range(2 * depth, n_wr))
        torch.cuda.synchronize()
        w_warm.run()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        tw = time.perf_counter()
        w_run.run()
        torch.cuda.synchronize()
        dist.barrier()
        tw = time.perf_counter() - tw
        tt = torch.tensor([tw], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tw = float(tt[0])
        weak = {"value": round(world * args.batch * n_w / tw, 1), "unit": "checks/s", "steps": n_w,
                "ms_per_step": round(tw / n_w * 1e3, 4), "scaling": "weak",
                "note": f"every rank checks its own {args.batch}-check requests ({world} x {args.batch} checks per "
                        f"step) from pinned host memory, results back to host memory, max-over-ranks time"}
        del w_items, w_perm, w_err
        progress("weak-scaling phase done")
    same_results = None
    if WL.kind not in ("mixed", "quota") and not args.partitioned:  # the first timed batch and its results
        items = rot[args.warm]
        sl0 = slice(args.warm * n_slice, (args.warm + 1) * n_slice)
        perm, err = torch.from_numpy(h_perm[sl0].copy()), torch.from_numpy(h_err[sl0].copy())
        if device_resident is not None:  # every timed batch: host path == device-resident path
            same_results = all(
                (h_perm[k * n_slice:(k + 1) * n_slice] == outs[k][0].cpu().numpy()).all() and
                (h_err[k * n_slice:(k + 1) * n_slice] == outs[k][1].cpu().numpy()).all()
                for k in range(args.warm, args.warm + args.steps))
    if WL.kind == "quota":
        items, (perm, err) = q_rot[args.warm][0], q_out[args.warm]
    if WL.kind == "mixed":  # the last step's batch: checked on the final snapshot, as the oracle is
        items = m_rot[rev["k"] - 1]
    st = eng.stats()
    # per-launch time of the dominant kernel, alone on the GPU: the timed batches again, one at a
    # time, device-resident (the kernel's own HBM roofline, without the PCIe reads of `value`'s
    # path), stage A timed by its dispatch timestamps (the engine's HSA queues; HIP events for a
    # batch launched through HIP), every 4th batch of a workspace. With batches in flight a launch
    # also waits for the CUs the other batches hold, so the roofline uses these; `achieved_job` is
    # the whole device-resident phase.
    st_solo = None
    if WL.kind not in ("mixed", "quota") and not args.partitioned and not args.no_profile:
        eng.set_profile(True)  # the timed region ran without events (a timed launch holds back the others)
        eng.reset_stats()
        for k in range(min(len(rot), 48)):
            eng.submit(rot[k].data_ptr(), n_slice, outs[k][0].data_ptr(), outs[k][1].data_ptr(), device=True,
                       stream=streams[0].cuda_stream, engine_stream=bool(args.engine_streams)).wait()
        torch.cuda.synchronize()
        st_solo = eng.stats()
        eng.set_profile(False)
        progress(f"solo launches done: {int(st_solo['bundle_launches'])} timed, {st_solo['bundle_ms']:.3f} ms, "
                 f"{int(st_solo['aql_batches'])} dispatched into the engine's queues")
    if args.partitioned and not args.no_profile:
        # the partitioned join's own kernels timed by their events (k_label_join on one rank;
        # k_pj_pack + k_pj_decide on several, the exchange between them not included), the
        # global batch again a few times
        eng.set_profile(True)
        eng.reset_stats()
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        st_solo = eng.stats()
        eng.set_profile(False)
        progress("solo partitioned batches done")
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])

    # pipelined configs: N ranks share each request (strong scaling); the others check a batch per
    # rank and step (weak)
    strong = WL.kind in ("nested", "gdocs", "github") and not args.partitioned
    total_checks = (args.batch if strong else world * args.batch) * args.steps
    value = total_checks / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # `value` (this task's bench contract): inputs already resident in HBM when the timed region
    # starts — the device-resident phase, timed as the host-buffer one (barrier + synchronize on both
    # sides, max over ranks). BASELINE.md:40-41's step with its PCIe transfers is the timed region
    # above, reported beside it as `baseline_pipelined` (and `baseline_step`, one batch at a time).
    baseline_pipelined = None
    if device_resident is not None:
        baseline_pipelined = {
            "value": round(value, 1), "unit": "checks/s", "ms_per_step": round(ms_per_step, 4), "inflight": depth,
            "steps": args.steps,
            "definition": "BASELINE.md:40-41 / SURVEY §8(d) step: 65,536-check requests in pinned host memory "
                          "(gck_host_alloc), items H2D + kernels + results D2H inside the timed region, 8 in flight "
                          "through the compiled submit/wait loop (libgck_driver.so); never `value`, which is "
                          "device-resident by this bench's contract (DESIGN.md §4)"}
        value = device_resident["value"]
        ms_per_step = device_resident["ms_per_step"]
    if args.partitioned:  # this rank's slice of the global batch, for the checker below
        perm = out["perm"][rank * args.batch:(rank + 1) * args.batch].contiguous()
        err = out["err"][rank * args.batch:(rank + 1) * args.batch].contiguous()
        items = items[rank * args.batch:(rank + 1) * args.batch].contiguous()
    res = perm.cpu().numpy()
    errs = err.cpu().numpy()

    # ---- the host-buffer path's other shapes (never `value`): one ctypes call per submit / wait,
    # pageable numpy buffers through the engine's pinned staging, one batch at a time, and
    # BASELINE.md:40-41's lone-batch median — over the first rotated batches, cycled
    host_rate = None
    baseline_step = None
    if WL.kind not in ("mixed", "quota") and not args.partitioned and args.host_steps > 0:
        n_h = min(len(rot), 32)
        p_rot = [(h_items[k * n_slice:(k + 1) * n_slice], h_perm[k * n_slice:(k + 1) * n_slice].copy(),
                  h_err[k * n_slice:(k + 1) * n_slice].copy()) for k in range(n_h)]
        p_rot = [(a, eng.host_array(n_slice, np.uint8), eng.host_array(n_slice, np.int32)) for a, _, _ in p_rot]
        h_rot = [a.copy() for a, _, _ in p_rot]  # pageable copies
        ref0 = (h_perm[:n_slice].copy(), h_err[:n_slice].copy())  # batch 0 from the warm-up

        def host_run(n_batches, dq, pinned):
            res_, q = {}, collections.deque()
            for j in range(n_batches):
                k = j % n_h
                if len(q) >= dq:
                    kk, b = q.popleft()
                    res_[kk] = b.wait()
                q.append((k, eng.submit_into(*p_rot[k]) if pinned else eng.submit(h_rot[k])))
            while q:
                kk, b = q.popleft()
                res_[kk] = b.wait()
            return res_

        def timed(dq, pinned):
            host_run(args.warm, dq, pinned)
            t0_ = time.perf_counter()
            r = host_run(args.host_steps, dq, pinned)
            dt = time.perf_counter() - t0_
            return r, {"value": round(args.host_steps * n_slice / dt, 1),
                       "ms_per_step": round(dt / args.host_steps * 1e3, 4)}
        hres, py_pinned = timed(depth, True)
        pres, pageable = timed(depth, False)
        _, one = timed(1, True)
        # BASELINE.md:40-41's own definition: 3 warm-up batches, then >= 20 batches, each one alone
        # (items H2D, kernels, results D2H: the compiled loop over pinned buffers, 1 in flight),
        # checks/s = checks per batch / the MEDIAN batch time
        from gochugaru_amd.engine import _driver
        import ctypes
        nb_med = max(20, min(200, args.host_steps))
        kb = [j % n_h for j in range(3 + nb_med)]
        med_run = eng.prepare_batches([p_rot[k][0].ctypes.data for k in kb], [p_rot[k][1].ctypes.data for k in kb],
                                      [p_rot[k][2].ctypes.data for k in kb], n_slice, 1, host=True)
        stamps = np.zeros(2 * len(kb), dtype=np.float64)
        _driver().gckd_set_trace(stamps.ctypes.data_as(ctypes.c_void_p), len(kb))
        med_run.run()
        _driver().gckd_set_trace(None, 0)
        subs, ends = stamps[0::2], stamps[1::2]
        prev = np.concatenate([[0.0], ends[:-1]])
        per_batch = (ends - prev)[3:]
        med_s = float(np.median(per_batch))
        baseline_step = {"value": round(n_slice / med_s, 1), "unit": "checks/s", "median_batch_ms": round(med_s * 1e3, 4),
                         "p90_batch_ms": round(float(np.percentile(per_batch, 90)) * 1e3, 4),
                         "median_submit_ms": round(float(np.median((subs - prev)[3:])) * 1e3, 4),
                         "batches": int(len(per_batch)), "warmup_batches": 3, "checks_per_batch": n_slice,
                         "definition": "BASELINE.md:40-41: checks per batch / median batch time over >= 20 batches "
                                       "after 3 warm-up batches, each batch alone (1 in flight): items H2D + kernels + "
                                       "results D2H (pinned gck_host_alloc buffers, the compiled submit/wait loop)"}
        same = all(0 in r and (r[0][0] == ref0[0]).all() and (r[0][1] == ref0[1]).all() for r in (hres, pres))
        host_rate = {"python_pinned": py_pinned, "pageable": pageable, "one_at_a_time": one, "inflight": depth,
                     "same_results": bool(same), "batches_cycled": n_h,
                     "note": "`value`'s path through other callers: one ctypes call per submit/wait over pinned "
                             "buffers (`python_pinned`), pageable numpy buffers through the engine's pinned staging "
                             "(`pageable`), 1 in flight (`one_at_a_time`)"}

    # ---- the uniform caller format (include/gck.h gck_check_submit_uniform; never `value`): the same
    # requests as runs of one shape — one header, 8-B (resource id, subject id) pairs in pinned host
    # memory, packed 2-bit results and a sparse error list back, read and written in place by the
    # join — `depth` in flight through the compiled loop. Each request is cut into its shapes
    # (config 4: one; configs 2 / 3: a run per permission), as INTEGRATION.md's toItems does.
    uni_line = None
    if pipelined and args.host_steps > 0:
        from gochugaru_amd.engine import ITEM_ERROR_DTYPE, unpack_results
        from gochugaru_amd.engine import _driver
        import ctypes
        n_u = args.warm + args.steps
        u_pairs = eng.host_array(n_u * n_slice * 2, np.uint32)
        u_errs = eng.host_array(n_u * n_slice, ITEM_ERROR_DTYPE)
        groups = []  # per uniform request: (batch k, header, start offset in the batch, order slice)
        words = 0
        for k in range(n_u):
            hk = h_items[k * n_slice:(k + 1) * n_slice]
            key = ((hk["resource_type"].astype(np.uint64) << np.uint64(48)) | (hk["permission"].astype(np.uint64) << np.uint64(32))
                   | (hk["subject_type"].astype(np.uint64) << np.uint64(16)) | hk["subject_relation"].astype(np.uint64))
            order = np.argsort(key, kind="stable")
            pv = u_pairs[2 * k * n_slice:2 * (k + 1) * n_slice].reshape(-1, 2)
            pv[:, 0] = hk["resource_id"][order]
            pv[:, 1] = hk["subject_id"][order]
            ks = key[order]
            cuts = [0] + (np.flatnonzero(np.diff(ks)) + 1).tolist() + [n_slice]
            for a, b in zip(cuts[:-1], cuts[1:]):
                x = int(ks[a])
                hdr = ((x >> 48) & 0xFFFF, (x >> 32) & 0xFFFF, (x >> 16) & 0xFFFF, x & 0xFFFF, 0)
                groups.append((k, hdr, a, b, order[a:b], words))
                words += (b - a + 31) // 32
        u_packed = eng.host_array(max(1, words), np.uint64)
        g_warm = [g for g in groups if g[0] < args.warm]
        g_time = [g for g in groups if g[0] >= args.warm]

        def prep_u(gs, dq):
            return eng.prepare_uniform([g[1] for g in gs],
                                       [u_pairs.ctypes.data + 8 * (g[0] * n_slice + g[2]) for g in gs],
                                       [g[3] - g[2] for g in gs],
                                       [u_packed.ctypes.data + 8 * g[5] for g in gs],
                                       [u_errs.ctypes.data + 8 * (g[0] * n_slice + g[2]) for g in gs],
                                       n_slice, dq)
        pw, pt = prep_u(g_warm, depth), prep_u(g_time, depth)
        pw.run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tu = time.perf_counter()
        pt.run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tu = time.perf_counter() - tu
        if world > 1:
            tt = torch.tensor([tu], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            tu = float(tt[0])
        # every timed request's results against the item path's (the timed region above)
        same_u = True
        for gi, (k, hdr, a, b, order_g, w0) in enumerate(g_time):
            n_g = b - a
            got = unpack_results(u_packed[w0:w0 + (n_g + 31) // 32], n_g)
            ne = int(pt.n_errs[gi])
            rec = u_errs[k * n_slice + a:k * n_slice + a + min(ne, n_g)]
            e_g = np.zeros(n_g, dtype=np.int32)
            e_g[rec["index"]] = rec["code"]
            hp = h_perm[k * n_slice:(k + 1) * n_slice][order_g]
            he = h_err[k * n_slice:(k + 1) * n_slice][order_g]
            want_p = np.where(he != 0, 0, hp)
            if not ((got == want_p).all() and (e_g == he).all()):
                same_u = False
                break
        # one request at a time (BASELINE.md:40-41's lone-batch step in the uniform format): the
        # first rotated requests, 1 in flight, median over >= 20 after 3 warm-up ones
        g_lone = [g for g in groups if g[0] < min(n_u, 23)]
        pl = prep_u(g_lone, 1)
        stamps = np.zeros(2 * len(g_lone), dtype=np.float64)
        _driver().gckd_set_trace(stamps.ctypes.data_as(ctypes.c_void_p), len(g_lone))
        pl.run()
        _driver().gckd_set_trace(None, 0)
        ends = stamps[1::2]
        starts = np.concatenate([[0.0], ends[:-1]])
        per_req = (ends - starts)
        per_batch = collections.defaultdict(float)
        for g, t in zip(g_lone, per_req):
            per_batch[g[0]] += t
        lone = [per_batch[k] for k in sorted(per_batch)][3:]
        med_u = float(np.median(lone)) if lone else None
        per_rank = args.batch * args.steps / world
        uni_line = {"value": round(args.batch * args.steps / tu, 1), "unit": "checks/s",
                    "ms_per_step": round(tu / args.steps * 1e3, 4), "inflight": depth,
                    "requests_per_batch": round(len(g_time) / args.steps, 2),
                    "same_results_as_items": bool(same_u),
                    "bytes_per_check": {"h2d": 8, "d2h": 0.25},
                    "pcie_h2d_GBs": round(per_rank * 8 / tu / 1e9, 2),
                    "lone_batch": ({"value": round(n_slice / med_u, 1), "median_batch_ms": round(med_u * 1e3, 4),
                                    "batches": len(lone)} if med_u else None),
                    "definition": "the timed requests as uniform requests (gck_check_submit_uniform: one header + "
                                  "8-B id pairs in pinned host memory, 2-bit results + error list back, read and "
                                  "written in place by the join across PCIe), 8 in flight through the compiled loop "
                                  "(gckd_run_uniform); `lone_batch`: one 64K request at a time, median"}
        del u_pairs, u_errs, u_packed
        progress(f"uniform phase: {tu * 1e3:.2f} ms")

    # `value`'s path is bound by the host link: 20 B of items in and 5 B of results out per check
    pcie = None
    if WL.kind in ("nested", "gdocs", "github") and not args.partitioned:
        per_rank = args.batch * args.steps / world  # checks over this rank's own link
        h2d, d2h = per_rank * 20 / elapsed / 1e9, per_rank * 5 / elapsed / 1e9
        pcie = {"bound": "pcie", "achieved": round(h2d, 2), "peak": 63.0, "unit": "GB/s", "frac": round(h2d / 63.0, 4),
                "d2h_GBs": round(d2h, 2), "bytes_per_check": {"h2d": 20, "d2h": 5},
                "note": "per GPU: the items' host-to-device bytes of the timed region (the binding direction) over "
                        "its time; peak = PCIe Gen5 x16 spec per direction (MI355X_MICROARCH.md); tools/pcie_probe "
                        "measures 40-41 GB/s for the GPU's zero-copy reads and the copy engines on this platform"}
    progress("host-buffer runs done")
    # ---- host-side checker: oracle over the same graph (rank 0) ------------------------------
    # host threads for the oracle: the CPUs this process may use (affinity mask, cgroup quota),
    # capped by OMP_NUM_THREADS when the box sets it (its per-GPU CPU share); nproc reports the
    # whole machine
    usable_cpus, nproc = host_cpus()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = args.cpu_threads or (min(usable_cpus, omp) if omp > 0 else usable_cpus)
    cpu_note = (f"{threads} threads: sched_getaffinity/cgroup allow {usable_cpus} CPUs"
                + (f", OMP_NUM_THREADS={omp}" if omp else "") + f", nproc {nproc}")
    prog = tab = None
    if rank == 0 and not args.no_oracle and WL.kind == "mixed":
        from oracle import corc  # the final snapshot (after every Watch batch) vs the timed batch
        hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
        mx = {}
        cp, ce = WL.M.expected(hi, threads=threads, stats=mx)
        agree_mixed = float(((cp == res) & (ce == errs)).mean())
        if not args.no_cpu and world == 1:
            # the C oracle answering the timed batch once (each context class against the snapshot
            # with its caveat outcomes), on the final snapshot; the Watch batches are not included
            cpu_q = {"value": round(args.batch / mx["seconds"], 1), "unit": "checks/s", "cores": threads, "kind": "port",
                     "sample": f"the timed batch ({args.batch} checks, 3 context classes), C oracle "
                               f"(oracle/check_oracle.c; caveat outcomes per context class), OpenMP {cpu_note}, "
                               f"{mx['seconds']:.2f}s; Watch application not included"}
        # SURVEY §8d algorithmic bytes of one check batch (+4 B per caveated edge)
        mixed_alg = 25 * args.batch + 8 * mx["rows"] + 4 * mx["edges"] + 4 * mx["cav_edges"]
    if rank == 0 and not args.no_oracle and WL.kind == "quota":
        from oracle import corc  # the first timed batch vs the C oracle's threshold mode
        q_threads = threads
        q_prog, q_tab, q_lim = WL.Q.oracle()
        hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
        t_q = time.perf_counter()
        cp, ce = corc.check_quota(q_prog, q_tab, hi, q_lim, q_rot[args.warm][1], threads=q_threads)
        t_q = time.perf_counter() - t_q
        agree_mixed = float(((cp == res) & (ce == errs)).mean())
        if not args.no_cpu and world == 1:
            cpu_q = {"value": round(args.batch / t_q, 1), "unit": "checks/s", "cores": q_threads, "kind": "port",
                     "sample": f"the first timed batch ({args.batch} checks, {args.batch} contexts), C oracle "
                               f"threshold mode (oracle/check_oracle.c orc_check_quota: the caveat restated in C, "
                               f"no CEL), OpenMP {cpu_note}, {t_q:.2f}s"}
    if rank == 0 and not args.no_oracle and WL.kind not in ("mixed", "quota"):
        from oracle import corc

        prog, tab = WL.oracle()
        host_items = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)

    # ---- roofline of the dominant kernels (SURVEY.md §8d algorithmic bytes) -------------------
    # One batch = stage A (k_closure_join over every check, then k_bundles<1> over what it left) and,
    # rarely, k_bundles<16> (deferred giant checks); they are >99 % of the device time, so stage A
    # is the "kernel". A timed join dispatched into the engine's queue carries the queue's dispatch
    # timestamps (packet start to completion, the span rocprofv3's kernel trace reports); one
    # launched through HIP its own start / stop events (hipExtLaunchKernelGGL on the launch stream).
    # Algorithmic bytes come from the oracle's counting mode on the timed batch (implementation
    # independent): 25 B per check (item in, tri-state + error out) + 8 B per row opened + 4 B
    # per edge enumerated (+4 B per caveated edge: none in this config). The launch time is
    # the mean over the sampled launches of the solo phase (the timed batches again, one at a time).
    n_batches = max(1, st["batches"])
    roof = None
    st_roof = st_solo if st_solo is not None else st
    if prog is not None and st_roof["bundle_launches"] and st_roof["bundle_ms"] > 0 and not args.partitioned:
        # counted on up to 4 of the rotated timed batches, averaged
        n_cnt = min(4, args.steps) if WL.kind != "mixed" else 1
        cnt = collections.Counter()
        for k in range(n_cnt):
            hk = (rot[args.warm + k].cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
                  if WL.kind != "mixed" else host_items)
            if WL.union_only:
                ck = corc.count_bfs(prog, tab, hk, threads=threads)
            else:  # joins: the recursive oracle's own row / edge counts (memoised per check)
                ck = corc.check(prog, tab, hk, threads=threads)[2]
            cnt.update(ck)
        cnt = {k: v / n_cnt for k, v in cnt.items()}
        b_alg = 25 * len(hk) + 8 * cnt["rows"] + 4 * cnt["edges"]
        ms_a = st_roof["bundle_ms"] / st_roof["bundle_launches"]
        ms_b = st_roof["giant_ms"] / st_roof["bundle_launches"]
        ms = ms_a + ms_b
        tj = None
        # (the counter passes of this workload's own batches on this round's code: tools/gpu.sh profile)
        if args.traffic_json is None:
            args.traffic_json = os.path.join(ROOT, "profiles", "r06", "pmc_" + WL.kind, "traffic.json")
        if args.traffic_json and os.path.exists(args.traffic_json) and WL.kind in ("nested", "gdocs", "github"):
            tj = json.load(open(args.traffic_json))
        roof = roofline_line(tj, args.traffic_json, b_alg, ms, args.steps,
                             device_resident["seconds"] if device_resident else None)
        # the join stage A ran: the label join (labels.inc) when the snapshot has label tables
        # and prefers them, else the closure join (closure.inc)
        kname = "k_label_join" if st_roof.get("label_checks", 0) > 0 else "k_closure_join"
        roof.update({
            "kernel": (f"{kname} (+ k_bundles<1> over what it leaves): stage A of a batch, dispatched as in "
                       "the timed region (into the engine's HSA queues, aql.inc) and timed by the queue's dispatch "
                       "timestamps (hsa_amd_profiling_get_dispatch_time: packet start to completion), batches one "
                       "at a time after the timed region; k_bundles<16> only for deferred giant checks"),
            "inflight": depth,
            "driver": args.driver if run_steps is not None or args.driver == "python" else "python",
            "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0")) or 4,
            "engine_streams": bool(args.engine_streams),
            "launch_timing": "solo" if st_solo is not None else "timed region",
            "alg_counts": {k: int(v) for k, v in cnt.items()},
            "mean_launch_ms": {f"stage A ({kname} + k_bundles<1>)": round(ms_a, 4), "k_bundles<16>": round(ms_b, 4)}})

    # ---- CPU baseline: the C restatement oracle on a bounded sample (rank 0, N=1) -----------
    # The sample is the timed batch plus further batches of the same generator (other seeds),
    # sized to --cpu-seconds; the GPU result of every sampled check is compared with it.
    cpu = None
    agree = None
    disagree = []
    if rank == 0 and world == 1 and not args.no_cpu and prog is not None and not args.partitioned:
        t0 = time.perf_counter()
        corc.check(prog, tab, host_items, threads=threads)
        per_batch = time.perf_counter() - t0
        extra = int(max(0, min(args.cpu_max_batches, args.cpu_seconds / max(per_batch, 1e-6))) - 1)
        # the timed batches with the results the timed region produced, then further batches
        timed = list(range(args.warm, args.warm + args.steps)) if WL.kind != "mixed" else []
        # (the results `value`'s path wrote into host memory)
        batches = ([(rot[k], torch.from_numpy(h_perm[k * n_slice:(k + 1) * n_slice]),
                     torch.from_numpy(h_err[k * n_slice:(k + 1) * n_slice])) for k in timed[:extra + 1]] if timed
                   else [(items, perm.clone(), err.clone())])
        extra = max(0, extra + 1 - len(batches))
        for k in range(extra):
            it = WL.checks(args.batch, 5000 + k)
            pk = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
            ek = torch.zeros(args.batch, dtype=torch.int32, device=dev)
            eng.check_bulk_device(it.data_ptr(), args.batch, pk.data_ptr(), ek.data_ptr(), stream=stream)
            batches.append((it, pk, ek))
        torch.cuda.synchronize()
        host = [(b[0].cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1), b[1].cpu().numpy(), b[2].cpu().numpy())
                for b in batches]
        n_s, n_ok, dt = 0, 0, 0.0
        for bi, (hi, gp, ge) in enumerate(host):
            t0 = time.perf_counter()
            cp, ce, _ = corc.check(prog, tab, hi, threads=threads)
            dt += time.perf_counter() - t0
            n_s += len(hi)
            ok = (cp == gp) & (ce == ge)
            n_ok += int(ok.sum())
            if not ok.all() and len(disagree) < 8:  # diagnostics: which batch, which items
                bad = np.nonzero(~ok)[0]
                # the same batch again, synchronously: does the engine agree the second time?
                it = batches[bi][0]
                pk = torch.zeros(args.batch, dtype=torch.uint8, device=dev)
                ek = torch.zeros(args.batch, dtype=torch.int32, device=dev)
                eng.check_bulk_device(it.data_ptr(), args.batch, pk.data_ptr(), ek.data_ptr(), stream=stream)
                torch.cuda.synchronize()
                rp, re_ = pk.cpu().numpy(), ek.cpu().numpy()
                disagree.append({"batch": bi, "n": int(len(bad)), "unwritten": int(((gp == 0) & (ge == 0)).sum()),
                                 "rerun_mismatches": int(((rp != cp) | (re_ != ce)).sum()),
                                 "first": [{"i": int(i), "gpu": [int(gp[i]), int(ge[i])],
                                            "oracle": [int(cp[i]), int(ce[i])]} for i in bad[:3]]})
        agree = n_ok / n_s
        cpu = {"value": round(n_s / dt, 1), "unit": "checks/s", "cores": threads, "kind": "port",
               "sample": f"{len(host)} batches x {args.batch} checks (the timed batches, then seeds 5000..), same "
                         f"{n_tuples / 1e6:.0f}M-tuple graph, C oracle (oracle/check_oracle.c, OpenMP "
                         f"{cpu_note}), {dt:.1f}s; every sampled check "
                         f"compared with the GPU result"}

    progress("oracle / CPU baseline done")
    import shutil
    spicedb = shutil.which("spicedb")  # SpiceDB serve-testing is the baseline where present
    if rank == 0 and WL.kind in ("mixed", "quota") and not args.no_oracle:
        agree = agree_mixed
    if rank == 0 and WL.kind in ("quota", "mixed") and not args.no_oracle and not args.no_cpu and world == 1:
        cpu = cpu_q
    if rank == 0 and WL.kind == "mixed" and not args.no_oracle and st["bundle_launches"] and st["bundle_ms"] > 0:
        # config 5: the check batch's stage A (wave bundles with caveat outcomes) timed by its HIP
        # events every 4th batch of a workspace inside the timed region; the Watch batch is
        # the rest of the step (watch.apply_ms_per_step)
        ms_a = (st["bundle_ms"] + st["giant_ms"]) / st["bundle_launches"]
        # (the counter passes of config 5's own check batches, tools/gpu.sh profile ... --config mixed)
        tj_path = args.traffic_json or os.path.join(ROOT, "profiles", "r06", "pmc_mixed", "traffic.json")
        tj = json.load(open(tj_path)) if os.path.exists(tj_path) else None
        roof = roofline_line(tj, tj_path, mixed_alg, ms_a, args.steps, elapsed)
        roof.update({"kernel": ("stage A of the check batch: k_label_join with the caveat plane, then k_bundles<1> over "
                                "the checks it deferred" if st["label_checks"] > 0 else
                                "stage A of the check batch (k_bundles<1>; k_bundles<16> for deferred giant checks)")
                               + ", HIP events on its launch stream, sampled every 4th batch in the timed region",
                     "mean_launch_ms": round(ms_a, 4)})

    if rank == 0 and args.partitioned and prog is not None:  # rank 0's slice of the global batch
        t_c = time.perf_counter()
        cp, ce, cnt_p = corc.check(prog, tab, host_items, threads=threads)
        t_c = time.perf_counter() - t_c
        agree = float(((cp == res) & (ce == errs)).mean())
        if not args.no_cpu and world == 1:
            cpu = {"value": round(len(host_items) / t_c, 1), "unit": "checks/s", "cores": threads, "kind": "port",
                   "sample": f"rank 0's {len(host_items)} checks of the timed global batch, the same "
                             f"{n_tuples / 1e6:.0f}M-tuple graph, C oracle (oracle/check_oracle.c, OpenMP {cpu_note}), "
                             f"{t_c:.1f}s; every sampled check compared with the GPU result"}
        if st_solo is not None and st_solo["bundle_launches"] and st_solo["bundle_ms"] > 0:
            # SURVEY §8d algorithmic bytes of rank 0's checks (the oracle's counting mode), over the
            # join's kernel time on rank 0 (each rank decides about 1/world of the global batch)
            ck = corc.count_bfs(prog, tab, host_items, threads=threads)
            b_alg = 25 * len(host_items) + 8 * ck["rows"] + 4 * ck["edges"]
            ms_a = st_solo["bundle_ms"] / st_solo["bundle_launches"]
            achieved = b_alg / (ms_a * 1e-3) / 1e9
            kname = "k_label_join" if world == 1 else "k_pj_pack + k_pj_decide"
            roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                    "kernel": f"{kname}: the partitioned label join of one global batch on rank 0, timed by the "
                              f"kernels' own HIP events (the exchange between them not included)",
                    "alg_bytes_per_launch": int(b_alg), "mean_launch_ms": round(ms_a, 4),
                    "alg_counts": {k: int(v) for k, v in ck.items()},
                    "label_checks_per_batch": round(st_solo["label_checks"] / max(1, st_solo["batches"]), 1)}

    check_stage = None
    if rank == 0 and WL.kind == "mixed":
        # the check stage alone, after the timed region (never `value`): the timed batch again on the
        # final snapshot, no Watch batch between, `depth` batches in flight on the engine's streams
        # with the same contexts — what the one-round join and its leftovers sustain
        n_cs = 200
        cs_out = [(torch.zeros(args.batch, dtype=torch.uint8, device=dev),
                   torch.zeros(args.batch, dtype=torch.int32, device=dev)) for _ in range(depth)]
        torch.cuda.synchronize()
        eng.reset_stats()
        t_cs = time.perf_counter()
        pend = []
        for k in range(n_cs):
            if len(pend) == depth:
                pend.pop(0).wait()
            o = cs_out[k % depth]
            pend.append(eng.submit(items.data_ptr(), args.batch, o[0].data_ptr(), o[1].data_ptr(), device=True,
                                   engine_stream=True, contexts=m_ctx))
        for b in pend:
            b.wait()
        torch.cuda.synchronize()
        t_cs = time.perf_counter() - t_cs
        st_cs = eng.stats()
        same = all(bool((o[0].cpu() == perm.cpu()).all()) for o in cs_out)
        check_stage = {"value": round(n_cs * args.batch / t_cs, 1), "unit": "checks/s", "batches": n_cs,
                       "inflight": depth, "label_checks_per_batch": round(st_cs["label_checks"] / n_cs, 1),
                       "same_results_as_timed_batch": same,
                       "note": "the timed batch repeated on the final snapshot without Watch batches between, "
                               "device-resident, engine streams; not the step"}
        progress("check-stage phase done")
    if rank == 0:
        line = {
            "metric": ("permission checks/sec (whole node) at batch 64K, 1B tuples" if WL.kind == "nested" else
                       f"permission checks/sec (whole node) at batch 64K, {WL.cfg['workload']}"),
            "value": round(value, 1), "unit": "checks/s", "n_gpus": 1 if args.share_gpu else world, "steps": args.steps,
            "warmup": args.warmup, "warmup_batches": args.warm, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u32",
            "data": WL.data,
            "config": {**WL.cfg, "tuples": n_tuples, "batch_per_gpu": args.batch,
                       "parallelism": (f"graph partitioned x{world} by resource id, per-level all-to-all "
                                       f"({args.part_backend}), global batch {args.batch * world}")
                       if args.partitioned else
                       (f"batch-sharded x{world}: one process per GPU, each {args.batch}-check request cut into "
                        f"{world} contiguous slices (sharded.slices), rank r checks slice r against a full replica of "
                        f"the graph; no data-path collective (barriers and the max-over-ranks time only)"
                        if strong else
                        f"batch-sharded x{world}: one process per GPU, each rank checks its own stream of "
                        f"{args.batch}-check batches against a full replica of the graph; no data-path collective "
                        f"(barriers and the max-over-ranks time only)"
                        + (f", {world} ranks sharing one GPU" if args.share_gpu else "")),
                       "hbm_snapshot_GB": round(dev_bytes / 1e9, 2)},
            "roofline": roof,
            "cpu_baseline": ({**cpu, "spicedb_probe": {"which_spicedb": spicedb,
                                                       "note": "BASELINE.md: SpiceDB serve-testing (memdb) is the CPU "
                                                               "baseline where a spicedb binary exists on the box; "
                                                               + ("it does, but it is not driven by this bench"
                                                                  if spicedb else
                                                                  "none was found, so the C restatement stands in")}}
                             if cpu else cpu),
            **({"dispatch": {"requests_per_dispatch": coal_for(args.steps), "checks_per_dispatch": n_slice * coal_for(args.steps),
                             "note": "a rank's slices of consecutive requests checked in one dispatch (--coalesce; "
                                     "1 = strong scaling of each request)"}}
               if strong and world > 1 else {}),
            **({"coalesced": coalesced} if coalesced else {}),
            **({"baseline_pipelined_uniform": uni_line} if uni_line else {}),
            **({"baseline_pipelined": baseline_pipelined} if baseline_pipelined else {}),
            **({"baseline_step": baseline_step} if baseline_step else {}),
            **({"weak_scaling": weak} if weak else {}),
            **({"host_buffers": host_rate} if host_rate else {}),
            **({"device_resident": device_resident} if device_resident else {}),
            **({"pcie": pcie} if pcie else {}),
            **({"host_equals_device_resident": same_results} if same_results is not None else {}),
            "host_placement": placement,
            "oracle_agreement": agree,
            **({"disagreements": disagree} if disagree else {}),
            "result_mix": {"HAS": int((res == 2).sum()), "NO": int((res == 1).sum()),
                           "COND": int((res == 3).sum()), "ERR": int((errs != 0).sum())},
            # levels: BFS levels run by the wave bundles (summed over bundles) plus the grid-wide
            # and partitioned paths' levels; the closure join runs none
            "engine": {"bfs_levels_per_batch": round(st["levels"] / n_batches, 2),
                       "levels_per_bundle": round(st["levels"] / st["bundles"], 2) if st["bundles"] else None,
                       "bundles_per_batch": round(st["bundles"] / n_batches, 1),
                       "entries_per_batch": int(st["entries_expanded"] / n_batches),
                       "edges_per_batch": int(st["edges_enumerated"] / n_batches),
                       "probes_per_batch": int(st["membership_probes"] / n_batches),
                       "device_ms_per_batch": round(st["kernel_ms"], 3),
                       "bundle_ms_per_batch": round(st["bundle_ms"] / n_batches, 4),
                       "deferred_per_batch": round(st["deferred"] / n_batches, 1),
                       "giant_ms_per_batch": round(st["giant_ms"] / n_batches, 4),
                       "deferred_wide_per_batch": round(st["deferred_wide"] / n_batches, 2),
                       "closure_checks_per_batch": round(st["closure_checks"] / n_batches, 1),
                       "slot_checks_per_batch": round(st["slot_checks"] / n_batches, 1),
                       "label_checks_per_batch": round(st["label_checks"] / n_batches, 1),
                       "aql_dispatched_batches": int(st["aql_batches"]),
                       "resident_batches": int(st["resident_batches"])},
            "setup_s": {"generate": round(t_gen, 1), "load": round(t_load, 1)},
            **({"timed_loop_ms": round(loop_s["s"] * 1e3, 4)} if loop_s["s"] is not None else {}),
            **({"loop_trace_us": {"submit_returned": [round(x * 1e6, 1) for x in trace[0::2]],
                                  "wait_returned": [round(x * 1e6, 1) for x in trace[1::2]]}}
               if trace is not None else {}),
            **({"caveats": {"evals_per_step": round(st["caveat_evals"] / args.steps, 1),
                            "extra_passes_per_step": round(st["caveat_passes"] / args.steps, 2)}}
               if WL.kind == "quota" else {}),
            **({"watch": {"updates_per_step": n_up, "apply_ms_per_step": round(rev["apply_timed"] / args.steps * 1e3, 3),
                          "share_of_step": round(rev["apply_timed"] / elapsed, 3),
                          "check_submit_ms_per_step": round(rev["submit_timed"] / args.steps * 1e3, 3),
                          "check_wait_ms_per_step": round(rev["wait_timed"] / args.steps * 1e3, 3),
                          "revision": rev["r"],
                          "staged": int(args.watch_stage),
                          "staging": (f"gck_watch_stage: each step stages the Watch batch {args.watch_stage} ahead "
                                      "(validated and grouped, its upload image laid out, on the engine's two "
                                      "staging threads) and then applies its own (gck_watch_apply_staged: merge, "
                                      "re-link, publication); the later batches' grouping runs beside this step's "
                                      "apply and device work" if args.watch_stage else "gck_apply_updates: grouping "
                                      "inside the apply")}} if WL.kind == "mixed" else {}),
            **({"check_stage": check_stage} if check_stage else {}),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
