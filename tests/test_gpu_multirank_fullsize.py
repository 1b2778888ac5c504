"""The multi-rank protocols at BASELINE.json's full sizes, rehearsed on the one-GPU test box:
ranks in separate spawned processes sharing cuda:0 over gloo (RCCL refuses two ranks on one
GPU; the 8-GPU node runs the same engine code over RCCL).

* config 4 partitioned by resource id (the export stream each rank filters is
  client/client.go:472-499) at 1e9 tuples over 2 ranks: one 64K batch through the partitioned
  label join, bit-exact against the C oracle on every rank, every check decided by the join on
  both ranks, and each rank's load peak at most 0.6x the replicated engine's (each rank alone in
  its own process: the device's free memory before the engine and after its commit);
* config 3 replicated and batch-sharded at 1e8 tuples over 2 ranks (DistributedChecker): each
  rank checks its contiguous slice of one 64K request, and the gathered slices equal one engine's
  answer to the whole request (client/client.go:238-284: one request = one Check)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from gochugaru_amd import engine as E

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 65536


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _part_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from gochugaru_amd.partition import PartitionedChecker
    from tests import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G = synth.build(1e9, device=torch.device("cuda", 0))
        items = synth.checks(G, N, seed=4246)
        e = E.Engine(device=0, max_batch=N * world)
        e.set_partition(rank, world)
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
        n_tuples = G.n_tuples
        del keep, G  # (the engine holds its own copies: only the items stay)
        torch.cuda.empty_cache()
        pc = PartitionedChecker(e)
        e.reset_stats()
        perm, err = pc.check(items, N)
        st = e.stats()
        np.save(os.path.join(out_dir, f"perm{rank}.npy"), perm.cpu().numpy())
        np.save(os.path.join(out_dir, f"err{rank}.npy"), err.cpu().numpy())
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump({"label_checks": int(st["label_checks"]), "levels": int(st["levels"]),
                       "tuples": e.tuple_count, "graph_tuples": n_tuples, "device_bytes": e.device_bytes,
                       "transport": pc.transport.calls}, f)
        e.close()
    finally:
        dist.destroy_process_group()


_LOAD_PROBE = r"""
import json, sys, torch
sys.path.insert(0, {root!r})
from gochugaru_amd import engine as E
from tests import synth
torch.cuda.set_device(0)
G = synth.build(1e9, device="cuda")
offs = [(rel, st, sr, n_rows, off.to(torch.int32).contiguous(), nbr) for rel, st, sr, n_rows, off, nbr in G.csrs()]
torch.cuda.synchronize()
free0 = torch.cuda.mem_get_info(0)[0]
e = E.Engine(device=0, workspaces=1)
if {world} > 1:
    e.set_partition({rank}, {world})
e.load_schema(synth.SCHEMA)
e.reserve_objects(synth.T_USER, G.n_users); e.reserve_objects(synth.T_GROUP, G.n_groups); e.reserve_objects(synth.T_DOC, G.n_docs)
e.begin_snapshot(1)
for rel, st, sr, n_rows, off, nbr in offs:
    e.load_csr(rel, st, sr, n_rows, off.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
e.commit_snapshot()
torch.cuda.synchronize()
free1 = torch.cuda.mem_get_info(0)[0]
print(json.dumps({{"peak": free0 - free1, "device_bytes": e.device_bytes, "tuples": e.tuple_count}}))
"""


def _load_probe(rank, world):
    code = _LOAD_PROBE.format(root=ROOT, rank=rank, world=world)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
def test_config4_1e9_partitioned_two_ranks(tmp_path):
    import torch.multiprocessing as mp

    from oracle import corc
    from tests import synth
    from tests.test_gpu_fullsize import THREADS, _diff, _oracle
    mp.spawn(_part_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    perms = [np.load(tmp_path / f"perm{r}.npy") for r in range(2)]
    errs = [np.load(tmp_path / f"err{r}.npy") for r in range(2)]
    assert np.array_equal(perms[0], perms[1]) and np.array_equal(errs[0], errs[1])
    G = synth.build(1e9, device=torch.device("cuda", 0))
    items = synth.checks(G, N, seed=4246)
    _, prog, tab = _oracle(G)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    cp, ce, _ = corc.check(prog, tab, hi, threads=THREADS)
    first, n_bad = _diff(perms[0], errs[0], cp, ce)
    assert n_bad == 0, first
    assert 0.3 < np.mean(cp == 2) < 0.7
    # every check decided by the partitioned label join, on both ranks; neither holds the graph
    assert all(o["label_checks"] == N for o in outs), [o["label_checks"] for o in outs]
    assert all(o["tuples"] < o["graph_tuples"] for o in outs), outs
    del G, items
    torch.cuda.empty_cache()
    # each rank's load alone in its process: at most 0.6x the replicated engine's peak
    rep = _load_probe(0, 1)
    parts = [_load_probe(r, 2) for r in range(2)]
    print(json.dumps({"replicated": rep, "ranks": parts, "check": outs}))
    for p in parts:
        assert p["peak"] <= 0.6 * rep["peak"], (p, rep)


def _shard_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from gochugaru_amd.sharded import DistributedChecker
    from tests import synth_configs as S
    from tests.test_gpu_fullsize import load_config

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = S.CONFIGS["github"](1.0, device=torch.device("cuda", 0))
        items = S.checks(W, N, seed=4247).cpu().numpy().view(E.ITEM_DTYPE).reshape(-1).copy()
        e = load_config(W)
        del W
        torch.cuda.empty_cache()
        dc = DistributedChecker(e)
        perm, err = dc.check_slice(items)
        b, en = dc.my_slice(N)
        perm_all, err_all = dc.gather(N, perm, err)
        if rank == 0:  # one engine, the whole request
            p1, e1 = e.check_bulk(items)
            np.save(os.path.join(out_dir, "one_perm.npy"), p1)
            np.save(os.path.join(out_dir, "one_err.npy"), e1)
        np.save(os.path.join(out_dir, f"all_perm{rank}.npy"), perm_all)
        np.save(os.path.join(out_dir, f"all_err{rank}.npy"), err_all)
        with open(os.path.join(out_dir, f"s{rank}.json"), "w") as f:
            json.dump({"slice": [b, en], "tuples": e.tuple_count}, f)
        e.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_config3_1e8_sharded_two_ranks(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_shard_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    sl = [json.load(open(tmp_path / f"s{r}.json")) for r in range(2)]
    assert sl[0]["slice"] == [0, N // 2] and sl[1]["slice"] == [N // 2, N]
    assert sl[0]["tuples"] > 9e7
    one_p, one_e = np.load(tmp_path / "one_perm.npy"), np.load(tmp_path / "one_err.npy")
    for r in range(2):  # the gathered slices, on every rank, equal the single engine's answer
        assert np.array_equal(np.load(tmp_path / f"all_perm{r}.npy"), one_p)
        assert np.array_equal(np.load(tmp_path / f"all_err{r}.npy"), one_e)
    assert (one_p == 2).sum() > N // 20 and (one_p == 1).sum() > N // 4
