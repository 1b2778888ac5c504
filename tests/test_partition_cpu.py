"""Partitioned checks, the host side on the CPU (no GPU): the owner function the engine and its
tests share, and the exchange a partitioned engine runs its batches over — the gck_transport
callbacks of gochugaru_amd/partition.py GlooTransport (all-to-all of byte blocks in rank order, an
element-wise MAX all-reduce) — driven through their C function pointers exactly as libgck's
partition.inc calls them, with world_size 2 and 3 over gloo. The engine's own use of the transport
(the label join's records, the level loop's entries / query and join records / flag planes) is
covered on the GPU by tests/test_gpu_partition.py."""
import ctypes
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gochugaru_amd import engine as E


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    from gochugaru_amd.partition import GlooTransport

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = GlooTransport(device=False)
        c = t.c
        # rank r sends (r * 16 + d + 1) bytes to rank d != r, each byte = 10 r + d; nothing to itself
        sb = [0 if d == rank else rank * 16 + d + 1 for d in range(world)]
        rb = [0 if s == rank else s * 16 + rank + 1 for s in range(world)]
        send = np.concatenate([np.full(sb[d], 10 * rank + d, dtype=np.uint8) for d in range(world)])
        recv = np.zeros(sum(rb), dtype=np.uint8)
        U64 = ctypes.c_uint64 * world
        rc = c.alltoallv(None, send.ctypes.data, U64(*sb), recv.ctypes.data, U64(*rb), None)
        # an empty exchange (every block 0) still completes on every rank
        rc0 = c.alltoallv(None, send.ctypes.data, U64(*[0] * world), recv.ctypes.data, U64(*[0] * world), None)
        buf = np.array([(rank * 37 + k) % 251 for k in range(301)], dtype=np.uint8)
        rc2 = c.allreduce_max_u8(None, buf.ctypes.data, len(buf), None)
        json.dump({"rc": [rc, rc0, rc2], "recv": recv.tolist(), "max": buf.tolist(), "error": t.error},
                  open(os.path.join(out_dir, f"r{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_transport_routes_blocks_and_reduces(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        o = json.load(open(tmp_path / f"r{r}.json"))
        assert o["rc"] == [0, 0, 0], o["error"]
        want = []
        for s in range(world):
            if s != r:
                want += [10 * s + r] * (s * 16 + r + 1)
        assert o["recv"] == want
        assert o["max"] == [max((q * 37 + k) % 251 for q in range(world)) for k in range(301)]


def test_owner_matches_library():
    """gck_partition_owner is the engine's part_owner (id mod world; gck_internal.hpp), which the
    partitioned slots also index by (id / world)."""
    for world in (1, 2, 3, 8):
        for obj in list(range(0, 2000, 7)) + [2**31, 2**32 - 3]:
            assert E.partition_owner(obj, world) == (0 if world == 1 else obj % world)


def _owner_name(type_id: int, name: str, world: int) -> int:
    """The name's owner restated (include/gck.h gck_partition_owner_name): FNV-1a 64 over the type
    id (2 bytes, little endian) and the name's bytes, a murmur-style finaliser, mod world."""
    m = (1 << 64) - 1
    h = 1469598103934665603
    for b in bytes([type_id & 0xFF, type_id >> 8]) + name.encode():
        h = ((h ^ b) * 1099511628211) & m
    h ^= h >> 33
    h = (h * 0xff51afd7ed558ccd) & m
    h ^= h >> 33
    return h % world if world > 1 else 0


def test_owner_of_a_name_matches_library():
    """Ownership by name (hash(type, id) mod G), decided before any interning: the
    library's function equals its restatement, and spreads names evenly over the ranks."""
    lib = E.load_library()
    names = [f"user{k}" for k in range(4000)] + ["", "*", "doc:x", "üñí", "a" * 300]
    for world in (1, 2, 3, 8):
        for t in (0, 1, 7, 300):
            for nm in names[:50] + names[-5:]:
                b = nm.encode()
                assert lib.gck_partition_owner_name(t, b, len(b), world) == _owner_name(t, nm, world), (t, nm, world)
        counts = np.bincount([E.partition_owner_name(2, nm, world) for nm in names[:4000]], minlength=world)
        assert counts.min() > 0.8 * 4000 / world, counts
