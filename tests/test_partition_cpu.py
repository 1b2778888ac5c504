"""Partitioned checks, multi-process on the CPU: the exchange driver (gochugaru_amd/partition.py)
over gloo with world_size 2 and 3, each rank a CPU model of the engine's gck_part_* protocol
(tests/part_model.py). Every rank must return the same results, equal to the single-process
oracle (oracle/spicedb_ref.py). The same driver runs the HIP engine in tests/test_gpu_partition.py.
"""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gochugaru_amd import engine as E
from gochugaru_amd.partition import PartitionedChecker
from tests import gen, part_model
from tests.helpers import oracle_for, parse_check, to_oracle_item


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, family, seed, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        schema, tuples, checks = gen.FAMILIES[family](seed)
        items = [to_oracle_item(parse_check(c)) for c in checks]
        m = part_model.ModelRank(schema, tuples, items, rank, world)
        pc = PartitionedChecker(m)
        perm, err = pc.check(torch.zeros(len(items) * 20, dtype=torch.uint8), len(items))
        res = {"perm": perm.tolist(), "err": err.tolist(), "levels": pc.levels,
               "local_tuples": m.store.count}
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("family,seed", [("nested", 1), ("gdocs", 2), ("gdocs_deep", 3)])
def test_partitioned_driver_matches_oracle(tmp_path, world, family, seed):
    mp.spawn(_worker, args=(world, _free_port(), family, seed, str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for o in outs[1:]:
        assert o["perm"] == outs[0]["perm"] and o["err"] == outs[0]["err"] and o["levels"] == outs[0]["levels"]
    schema, tuples, checks = gen.FAMILIES[family](seed)
    assert sum(o["local_tuples"] for o in outs) == len(set(tuples))  # the graph is split, not copied
    ck = oracle_for(schema, tuples)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    got = list(zip(outs[0]["perm"], outs[0]["err"]))
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]


def test_owner_hash_matches_library():
    """tests/part_model.owner restates part_owner; the library's gck_partition_owner is the
    product's (host side of the same inline function the kernels use)."""
    for world in (1, 2, 3, 8):
        for obj in list(range(0, 2000, 7)) + [2**31, 2**32 - 3]:
            want = 0 if world == 1 else part_model.owner(obj, world)
            assert E.partition_owner(obj, world) == want
