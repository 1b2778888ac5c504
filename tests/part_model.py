"""TEST INFRASTRUCTURE — a CPU model of one rank of a partitioned engine (the gck_part_* protocol
of include/gck.h, device side in gochugaru_amd/csrc/partition.inc), so that the host exchange
driver (gochugaru_amd/partition.py) can run world_size>1 over gloo on a machine without a GPU.

The model restates the level-synchronous evaluation the engine runs (union
schemas): every (check, node, object) is expanded once, at its minimal depth, on the rank that
owns the object; pushes for objects another rank owns go to that rank's outbox; found /
conditional / depth-error / alive flags are exchanged as 0/1 byte planes. Its answers are
compared with the single-process oracle (oracle/spicedb_ref.py), which pins both the protocol
and the driver. The buffers the driver passes are CPU tensors, addressed through data_ptr()
exactly as the real engine addresses device memory.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Tuple

import numpy as np
import torch

from oracle import spicedb_ref as ref

ENTRY = np.dtype([("q", "<u4"), ("obj", "<u4"), ("node", "<u2"), ("depth", "u1"), ("cond", "u1")])
assert ENTRY.itemsize == 12


def owner(obj: int, world: int) -> int:
    """part_owner (gochugaru_amd/csrc/gck_internal.hpp)."""
    h = (obj * 2654435761) & 0xFFFFFFFF
    h ^= h >> 16
    return h % world


def _view(ptr: int, dtype, n: int) -> np.ndarray:
    nbytes = np.dtype(dtype).itemsize * n
    buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n)


class Ids:
    """Global interning shared by every rank: (type, name) -> dense id; nodes = (type, rel)."""

    def __init__(self, schema: ref.Schema, tuples: List[ref.Tuple_], items: List[ref.Item]):
        names: Dict[str, set] = {t: set() for t in schema.defs}
        for t in tuples:
            names[t.resource_type].add(t.resource_id)
            if t.subject_id != ref.WILDCARD:
                names[t.subject_type].add(t.subject_id)
        for it in items:
            names.setdefault(it.resource_type, set()).add(it.resource_id)
            names.setdefault(it.subject_type, set()).add(it.subject_id)
        self.id = {(t, n): i for t, ns in names.items() for i, n in enumerate(sorted(ns))}
        self.name = {(t, i): n for (t, n), i in self.id.items()}
        self.nodes = [(d, r) for d in schema.defs for r in schema.defs[d].relations]
        self.node = {n: i for i, n in enumerate(self.nodes)}


class ModelRank:
    """Implements Engine.part_* for one rank (union schemas, no caveats)."""

    torch_device = torch.device("cpu")

    def __init__(self, schema_text: str, tuples: List[str], items: List[ref.Item], rank: int, world: int,
                 max_depth: int = 50):
        self.schema = ref.Schema(schema_text)
        tps = [ref.parse_tuple(t) for t in tuples]
        self.ids = Ids(self.schema, tps, items)
        self.part_rank, self.part_world = rank, world
        self.max_depth = max_depth
        self.store = ref.TupleStore(t for t in tps
                                    if owner(self.ids.id[(t.resource_type, t.resource_id)], world) == rank)
        self.items = items

    # ---- protocol ---------------------------------------------------------------------------
    # the label join (gck_part_join_*): the model has no label tables, so it sends no records and
    # decides nothing — every check goes through the level loop, as on an engine without them
    def part_join_pack(self, d_items: int, n: int, d_send: int, cap: int, stream=None) -> np.ndarray:
        return np.zeros(self.part_world, dtype=np.uint64)

    def part_join_decide(self, d_items: int, n: int, d_recv: int, n_recv: int, d_perm: int, d_err: int, stream=None):
        assert n_recv == 0

    def part_begin(self, d_items: int, n: int, now_us: int = 0, stream=None):
        assert n == len(self.items)
        self.n, self.level = n, 0
        self.flags = np.zeros((n, 3), dtype=bool)  # found Y, found C, error
        self.done = np.zeros(n, dtype=bool)
        self.result = np.zeros(n, dtype=np.uint8)
        self.err = np.zeros(n, dtype=np.int32)
        self.last_alive = np.zeros(n, dtype=np.int64)
        self.visited = set()
        self.frontier: List[Tuple] = []
        self.next: List[Tuple] = []
        self.out: List[List[Tuple]] = [[] for _ in range(self.part_world)]
        ck = ref.Checker(self.schema, ref.TupleStore())
        for q, it in enumerate(self.items):
            e = ck.validate(it)
            if e:
                self.done[q], self.err[q] = True, e
                continue
            root = self.ids.id[(it.resource_type, it.resource_id)]
            if owner(root, self.part_world) == self.part_rank:
                self.frontier.append((q, root, self.ids.node[(it.resource_type, it.permission)], 0, 0))

    def _push(self, q, obj, node, depth, cond):
        if cond and (q, node, 0, obj) in self.visited:
            return
        key = (q, node, cond, obj)
        if key in self.visited:
            return
        self.visited.add(key)
        d = owner(obj, self.part_world)
        (self.next if d == self.part_rank else self.out[d]).append((q, obj, node, depth, cond))
        self.last_alive[q] = self.level + 1

    def _expand(self, q, obj, node, depth, cond):
        it = self.items[q]
        typ, rel = self.ids.nodes[node]
        oname = self.ids.name[(typ, obj)]
        subj = (it.subject_type, it.subject_id, it.subject_relation or ref.ELLIPSIS)
        if (typ, oname, rel) == subj:
            self.flags[q, 1 if cond else 0] = True
            return
        if depth >= self.max_depth:
            self.flags[q, 2] = True
            return
        r = self.schema.relation(typ, rel)
        if not r.is_permission:
            for t in self.store.get(typ, oname, rel):
                if t.subject_type == subj[0] and ((t.subject_id == ref.WILDCARD and t.subject_relation == ref.ELLIPSIS
                                                   and subj[2] == ref.ELLIPSIS)
                                                  or (t.subject_id == subj[1] and t.subject_relation == subj[2])):
                    self.flags[q, 1 if cond else 0] = True
                elif t.subject_relation != ref.ELLIPSIS:
                    self._push(q, self.ids.id[(t.subject_type, t.subject_id)],
                               self.ids.node[(t.subject_type, t.subject_relation)], depth + 1, cond)
            return
        self._eval(r.expr, q, typ, obj, oname, depth, cond)

    def _eval(self, e, q, typ, obj, oname, depth, cond):
        if e.op == "union":
            for c in e.children:
                self._eval(c, q, typ, obj, oname, depth, cond)
        elif e.op == "computed":
            self._push(q, obj, self.ids.node[(typ, e.name)], depth + 1, cond)
        elif e.op == "arrow":
            assert e.func == "any"
            for t in self.store.get(typ, oname, e.tupleset):
                if self.schema.relation(t.subject_type, e.name) is not None:
                    self._push(q, self.ids.id[(t.subject_type, t.subject_id)],
                               self.ids.node[(t.subject_type, e.name)], depth + 1, cond)
        elif e.op != "nil":
            raise ValueError("partitioned checks support union schemas only")

    def part_expand(self) -> np.ndarray:
        self.next, self.out = [], [[] for _ in range(self.part_world)]
        for q, obj, node, depth, cond in self.frontier:
            if not self.done[q]:
                self._expand(q, obj, node, depth, cond)
        return np.array([len(o) for o in self.out], dtype=np.uint64)

    def part_pack(self, d_send: int, cap: int):
        flat = [x for o in self.out for x in o]
        assert len(flat) <= cap
        _view(d_send, ENTRY, len(flat))[:] = np.array(flat, dtype=ENTRY)

    def part_ingest(self, d_recv: int, n_recv: int, d_flags: int):
        for e in _view(d_recv, ENTRY, n_recv).tolist():
            q, obj, node, depth, cond = (int(x) for x in e)
            assert owner(obj, self.part_world) == self.part_rank
            if not self.done[q]:
                self._push(q, obj, node, depth, cond)
        n = self.n
        fl = _view(d_flags, np.uint8, 4 * n + 1)
        fl[:n], fl[n:2 * n], fl[2 * n:3 * n] = self.flags[:, 0], self.flags[:, 1], self.flags[:, 2]
        fl[3 * n:4 * n] = self.last_alive > self.level
        fl[4 * n] = 0

    def part_resolve(self, d_flags: int) -> int:
        n = self.n
        fl = _view(d_flags, np.uint8, 4 * n + 1).astype(bool)
        self.flags |= np.stack([fl[:n], fl[n:2 * n], fl[2 * n:3 * n]], axis=1)
        self.last_alive[fl[3 * n:4 * n]] = self.level + 1
        for q in range(n):
            if self.done[q]:
                continue
            if self.flags[q, 0]:
                self.done[q], self.result[q] = True, ref.HAS
            elif self.last_alive[q] <= self.level:
                self.done[q] = True
                if self.flags[q, 2]:
                    self.err[q] = ref.ITEM_ERR_MAX_DEPTH
                else:
                    self.result[q] = ref.COND if self.flags[q, 1] else ref.NO
        self.frontier = self.next
        self.level += 1
        return int(sum(1 for q in range(n) if not self.done[q] and self.last_alive[q] > self.level - 1))

    def part_finish(self, d_perm: int, d_err: int):
        assert self.done.all()
        _view(d_perm, np.uint8, self.n)[:] = np.where(self.err != 0, 0, self.result)
        _view(d_err, np.int32, self.n)[:] = self.err
