"""Replicated-graph sharding on the CPU (gochugaru_amd/sharded.py): the slicing, and the
one-process-per-GPU protocol over gloo with world_size 2 and 3 — every rank checks its contiguous
slice of one global request (the checker here is the oracle, as a stand-in engine on a box without
a GPU) and the gathered answer is the single-process answer in request order."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from gochugaru_amd.sharded import DistributedChecker, slices
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item


def test_slices_cover_in_order():
    for n in (0, 1, 5, 64, 65536, 65537):
        for g in (1, 2, 3, 8):
            s = slices(n, g)
            assert len(s) == g and s[0][0] == 0 and s[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(s, s[1:]))
            assert max(e - b for b, e in s) - min(e - b for b, e in s) <= 1


class _OracleChecker:
    """A stand-in engine: check_bulk over oracle items (test infrastructure only)."""

    def __init__(self, family, seed):
        schema, tuples, checks = gen.FAMILIES[family](seed)
        self.ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
        self.items = [to_oracle_item(parse_check(c)) for c in checks]

    def check_bulk(self, idx):
        res = [self.ck.check(self.items[int(i)]) for i in idx]
        return (np.array([r[0] for r in res], dtype=np.uint8), np.array([r[1] for r in res], dtype=np.int32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, family, seed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _OracleChecker(family, seed)
        dc = DistributedChecker(c)
        n = len(c.items)
        idx = np.arange(n)  # the global request: item indices (the same on every rank)
        p, e = dc.check_slice(idx)
        pa, ea = dc.gather(n, p, e)
        np.save(os.path.join(out, f"r{rank}.npy"), np.stack([pa.astype(np.int64), ea.astype(np.int64)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_slices_gather_in_request_order(world, tmp_path):
    family, seed = "github", 2
    mp.spawn(_worker, args=(world, _free_port(), family, seed, str(tmp_path)), nprocs=world, join=True)
    c = _OracleChecker(family, seed)
    want_p, want_e = c.check_bulk(np.arange(len(c.items)))
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        assert np.array_equal(got[0], want_p) and np.array_equal(got[1], want_e)
