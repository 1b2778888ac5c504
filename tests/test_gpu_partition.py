"""Partitioned graphs on the GPU (include/gck.h gck_part_*, gochugaru_amd/csrc/partition.inc):
ranks that each hold only the rows of the objects they own check a global batch together through
the exchange driver (gochugaru_amd/partition.py). On the one-GPU test box the ranks share cuda:0
and exchange over gloo (host-staged); on a multi-GPU node the same driver uses RCCL.
Bar: every rank returns the single-GPU engine's / the oracle's results bit-exactly."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, family, seed, out_dir, backend):
    import torch.distributed as dist

    from gochugaru_amd.partition import PartitionedChecker

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        if family == "synth":
            from tests import synth
            G = synth.build(seed, device=torch.device("cuda", 0))
            e = E.Engine(device=0)
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
            d_items = synth.checks(G, 4096, seed=77)
            n = 4096
        else:
            schema, tuples, checks = gen.FAMILIES[family](seed)
            e = E.Engine(device=0)
            e.set_partition(rank, world)
            e.load_schema(schema)
            e.load_snapshot_text(1, "\n".join(tuples))
            items = e.make_items([parse_check(c) for c in checks])
            d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
            n = len(items)
        pc = PartitionedChecker(e)
        perm, err = pc.check(d_items, n, now_us=gen.NOW_US)
        with pytest.raises(E.GckError):  # a partitioned engine refuses single-rank checks
            e.check_bulk(np.zeros(1, dtype=E.ITEM_DTYPE))
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump({"perm": perm.cpu().tolist(), "err": err.cpu().tolist(), "levels": pc.levels,
                       "tuples": e.tuple_count}, f)
        e.close()
    finally:
        dist.destroy_process_group()


def _run(tmp_path, world, family, seed, backend="gloo"):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), family, seed, str(tmp_path), backend), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for o in outs[1:]:
        assert o["perm"] == outs[0]["perm"] and o["err"] == outs[0]["err"]
    return outs


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("family,seed", [("nested", 1), ("gdocs", 2), ("gdocs_deep", 3)])
def test_partitioned_matches_oracle(tmp_path, world, family, seed):
    outs = _run(tmp_path, world, family, seed)
    schema, tuples, checks = gen.FAMILIES[family](seed)
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    got = list(zip(outs[0]["perm"], outs[0]["err"]))
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]


def test_partitioned_scale_matches_replicated(tmp_path):
    """The config-4 graph shape at 2e6 tuples split over 2 ranks vs the single-GPU engine."""
    from tests import synth
    from tests.test_gpu_scale import load_engine, run
    outs = _run(tmp_path, 2, "synth", 2e6)
    G = synth.build(2e6, device=torch.device("cuda", 0))
    e = load_engine(G)
    p, x = run(e, synth.checks(G, 4096, seed=77))
    e.close()
    assert outs[0]["perm"] == p.tolist() and outs[0]["err"] == x.tolist()
    assert sum(1 for v in p if v == E.PERM_HAS) > 1000


def test_partitioned_rejects_joins():
    schema, tuples, checks = gen.github(1)
    e = E.Engine(device=0)
    e.set_partition(0, 2)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    d = torch.zeros(20, dtype=torch.uint8, device="cuda")
    with pytest.raises(E.GckError) as ei:
        e.part_begin(d.data_ptr(), 1)
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    e.close()


@pytest.mark.parametrize("family,seed", [("nested", 1), ("gdocs", 2), ("gdocs_deep", 3)])
def test_rccl_loop_single_rank_matches_oracle(family, seed):
    """gck_part_check: the level loop with its RCCL exchange inside libgck (grouped send / receive
    of counts and entries, in-place all-reduce MAX of the flags). The one-GPU test box can only
    hold a one-rank communicator (RCCL refuses two ranks on one GPU: "Duplicate GPU detected"),
    so this runs the whole RCCL path with world 1; the multi-rank exchange protocol itself is
    covered by the gloo tests above and tests/test_partition_cpu.py."""
    from gochugaru_amd.partition import RcclPartitionedChecker
    schema, tuples, checks = gen.FAMILIES[family](seed)
    e = E.Engine(device=0)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    pc = RcclPartitionedChecker(e)
    perm, err = pc.check(d_items, len(items), now_us=gen.NOW_US)
    got = list(zip(perm.cpu().tolist(), err.cpu().tolist()))
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]
    perm2, err2 = pc.check(d_items, len(items), now_us=gen.NOW_US)  # the communicator is reused
    assert perm2.cpu().tolist() == perm.cpu().tolist() and err2.cpu().tolist() == err.cpu().tolist()
    e.close()


def test_partitioned_steps_refuse_a_swapped_snapshot():
    """A Watch batch between gck_part_begin and a later step swaps the device snapshot: the step
    fails with GCK_E_STATE instead of running on other (or freed) arrays; a new begin works."""
    schema, tuples, checks = gen.FAMILIES["gdocs"](1)
    e = E.Engine(device=0)
    e.set_partition(0, 1)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks[:64]])
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    e.part_begin(d_items.data_ptr(), len(items))
    e.apply_updates_text(2, "TOUCH " + tuples[0])
    with pytest.raises(E.GckError) as ei:
        e.part_expand()
    assert ei.value.code == E.GCK_E_STATE
    e.part_begin(d_items.data_ptr(), len(items))
    e.part_expand()
    e.close()
