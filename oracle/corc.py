"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C restatement (oracle/check_oracle.c ->
oracle/libgck_oracle.so) plus an independent numpy CSR builder and program encoder.

The program encoder works from the oracle's own schema parser (spicedb_ref.Schema), and the
CSR builder from the oracle's own tuple store, so that nothing here shares code with the
product's C++ compiler/builder (gochugaru_amd/csrc). Relation ids follow the same public
numbering as the C ABI (definition order), so the two can be fed the same interned items.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import spicedb_ref as ref

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libgck_oracle.so")

ELLIPSIS = 0xFFFF
WILDCARD = 0xFFFFFFFF
ABSENT = 0xFFFFFFFE

OP_UNION, OP_INTER, OP_EXCL, OP_NIL, OP_COMP, OP_ARROW = 1, 2, 3, 4, 5, 6

ITEM_DTYPE = np.dtype([
    ("resource_type", "<u2"), ("permission", "<u2"), ("resource_id", "<u4"),
    ("subject_type", "<u2"), ("subject_relation", "<u2"), ("subject_id", "<u4"),
    ("context_slot", "<u4"),
])


class _CSR(C.Structure):
    _fields_ = [("off", C.c_void_p), ("nbr", C.c_void_p), ("cav", C.c_void_p),
                ("exp", C.c_void_p), ("n_rows", C.c_uint32), ("pad", C.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} missing: run `make -C oracle`")
        l = C.CDLL(LIB)
        l.orc_check.restype = C.c_int
        l.orc_check.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int64, C.c_int,
                                C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        l.orc_check_quota.restype = C.c_int
        l.orc_check_quota.argtypes = l.orc_check.argtypes + [C.c_void_p, C.c_void_p, C.c_uint32]
        l.orc_count_bfs.restype = C.c_int
        l.orc_count_bfs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int,
                                    C.c_void_p]
        _lib = l
    return _lib


class Ids:
    """Public numbering shared with the C ABI: types and relations in definition order."""

    def __init__(self, schema: ref.Schema):
        self.schema = schema
        self.types = list(schema.defs)
        self.type_id = {t: i for i, t in enumerate(self.types)}
        self.rels: List[Tuple[str, str]] = []
        self.rel_id: Dict[Tuple[str, str], int] = {}
        for t in self.types:
            for r in schema.defs[t].relations:
                self.rel_id[(t, r)] = len(self.rels)
                self.rels.append((t, r))

    def kinds(self, typ: str, rel: str) -> List[Tuple[int, int]]:
        """Distinct (subject type, subject relation) kinds of a relation, in schema order."""
        out = []
        for a in self.schema.relation(typ, rel).allowed:
            k = (self.type_id[a.type],
                 ELLIPSIS if a.relation == ref.ELLIPSIS else self.rel_id[(a.type, a.relation)])
            if k not in out:
                out.append(k)
        return out


def encode_program(ids: Ids, csr_index: Dict[Tuple[int, int, int, bool], int]) -> np.ndarray:
    """[n_types, n_rels, rel_off[n_rels], records...] (see check_oracle.c)."""
    recs: List[List[int]] = []
    for (t, r) in ids.rels:
        rel = ids.schema.relation(t, r)
        tid = ids.type_id[t]
        rid = ids.rel_id[(t, r)]
        if not rel.is_permission:
            rec = [tid, 0, 0]
            for (st, sr) in ids.kinds(t, r):
                rec += [st, sr, csr_index.get((rid, st, sr, False), -1), csr_index.get((rid, st, sr, True), -1)]
                rec[2] += 1
        else:
            rec = [tid, 1, 0] + _encode_expr(ids, t, rel.expr)
        recs.append(rec)
    n_rels = len(recs)
    head = 2 + n_rels
    offs, pos = [], head
    for rec in recs:
        offs.append(pos)
        pos += len(rec)
    out = [len(ids.types), n_rels] + offs
    for rec in recs:
        out += rec
    return np.asarray(out, dtype=np.int32)


def _encode_expr(ids: Ids, t: str, e: ref.Expr) -> List[int]:
    if e.op in ("union", "intersect", "exclude"):
        op = {"union": OP_UNION, "intersect": OP_INTER, "exclude": OP_EXCL}[e.op]
        out = [op, len(e.children)]
        for c in e.children:
            out += _encode_expr(ids, t, c)
        return out
    if e.op == "nil":
        return [OP_NIL]
    if e.op == "computed":
        return [OP_COMP, ids.rel_id[(t, e.name)]]
    if e.op == "arrow":
        ts = ids.rel_id[(t, e.tupleset)]
        targets = []
        for (st, _sr) in ids.kinds(t, e.tupleset):
            stn = ids.types[st]
            tr = ids.rel_id.get((stn, e.name), -1)
            if (st, tr) not in [(a, b) for a, b in zip(targets[::2], targets[1::2])]:
                targets += [st, tr]
        return [OP_ARROW, ts, 1 if e.func == "all" else 0, len(targets) // 2] + targets
    raise ValueError(e.op)


class Store:
    """Independent CSR build (numpy) of an oracle TupleStore, in the oracle's own id space."""

    def __init__(self, schema: ref.Schema, tuples: Sequence[ref.Tuple_]):
        self.ids = Ids(schema)
        self.names: Dict[int, Dict[str, int]] = {i: {} for i in range(len(self.ids.types))}
        store = ref.TupleStore(tuples)  # TOUCH semantics: last write wins
        self.caveats: List[Tuple[str, tuple]] = [("", ())]
        rows = []
        for (rt, rid, rel), lst in sorted(store.index.items()):
            for tp in lst:
                rows.append(tp)
        for tp in rows:
            self.intern(tp.resource_type, tp.resource_id)
            if tp.subject_id != ref.WILDCARD:
                self.intern(tp.subject_type, tp.subject_id)
        groups: Dict[Tuple[int, int, int, bool], List[Tuple[int, int, int, int]]] = {}
        for tp in rows:
            rid = self.ids.rel_id[(tp.resource_type, tp.relation)]
            st = self.ids.type_id[tp.subject_type]
            sr = ELLIPSIS if tp.subject_relation == ref.ELLIPSIS else self.ids.rel_id[(tp.subject_type, tp.subject_relation)]
            ext = tp.caveat is not None or tp.expires_at is not None
            cav = 0
            if tp.caveat:
                self.caveats.append((tp.caveat, tp.caveat_context or ()))
                cav = len(self.caveats) - 1
            exp = 0 if tp.expires_at is None else max(1, int(round(tp.expires_at * 1e6)))
            obj = self.names[self.ids.type_id[tp.resource_type]][tp.resource_id]
            sid = WILDCARD if tp.subject_id == ref.WILDCARD else self.names[st][tp.subject_id]
            groups.setdefault((rid, st, sr, ext), []).append((obj, sid, cav, exp))
        self.csr_index: Dict[Tuple[int, int, int, bool], int] = {}
        self.arrays = []
        for key in sorted(groups):
            rid = key[0]
            n_rows = len(self.names[self.ids.type_id[self.ids.rels[rid][0]]])
            g = np.array(sorted(groups[key]), dtype=np.int64).reshape(-1, 4)
            counts = np.bincount(g[:, 0], minlength=n_rows)
            off = np.zeros(n_rows + 1, dtype=np.uint32)
            off[1:] = np.cumsum(counts)
            nbr = g[:, 1].astype(np.uint32)
            cav = g[:, 2].astype(np.uint32) if key[3] else None
            exp = g[:, 3].astype(np.int64) if key[3] else None
            self.csr_index[key] = len(self.arrays)
            self.arrays.append((off, nbr, cav, exp, n_rows))
        self.program = encode_program(self.ids, self.csr_index)

    def intern(self, typ: str, oid: str) -> int:
        d = self.names[self.ids.type_id[typ]]
        if oid not in d:
            d[oid] = len(d)
        return d[oid]

    def items(self, checks: Sequence[ref.Item]) -> np.ndarray:
        out = np.zeros(len(checks), dtype=ITEM_DTYPE)
        for i, it in enumerate(checks):
            rt = self.ids.type_id.get(it.resource_type, 0xFFFF)
            st = self.ids.type_id.get(it.subject_type, 0xFFFF)
            out[i]["resource_type"] = rt
            out[i]["subject_type"] = st
            out[i]["permission"] = self.ids.rel_id.get((it.resource_type, it.permission), 0xFFFE)
            sr = it.subject_relation or ref.ELLIPSIS
            out[i]["subject_relation"] = ELLIPSIS if sr == ref.ELLIPSIS else self.ids.rel_id.get((it.subject_type, sr), 0xFFFE)
            out[i]["resource_id"] = self.names.get(rt, {}).get(it.resource_id, ABSENT)
            out[i]["subject_id"] = (WILDCARD if it.subject_id == ref.WILDCARD
                                    else self.names.get(st, {}).get(it.subject_id, ABSENT))
        return out

    def csr_table(self):
        return make_csr_table(self.arrays)


def make_csr_table(arrays):
    """arrays: list of (off, nbr, cav|None, exp|None, n_rows) numpy arrays."""
    tab = (_CSR * max(1, len(arrays)))()
    keep = []
    for i, (off, nbr, cav, exp, n_rows) in enumerate(arrays):
        off = np.ascontiguousarray(off, dtype=np.uint32)
        nbr = np.ascontiguousarray(nbr, dtype=np.uint32)
        keep += [off, nbr]
        tab[i].off = off.ctypes.data
        tab[i].nbr = nbr.ctypes.data
        if cav is not None:
            cav = np.ascontiguousarray(cav, dtype=np.uint32)
            exp = np.ascontiguousarray(exp, dtype=np.int64)
            keep += [cav, exp]
            tab[i].cav = cav.ctypes.data
            tab[i].exp = exp.ctypes.data
        tab[i].n_rows = int(n_rows)
    return tab, keep


def check(program: np.ndarray, csr_table, items: np.ndarray, now_us: int = 0, max_depth: int = 50,
          threads: int = 1):
    """Returns (perm u8[n], err i32[n], counters {rows, probes, edges})."""
    tab, _keep = csr_table
    items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
    program = np.ascontiguousarray(program, dtype=np.int32)
    n = len(items)
    perm = np.zeros(n, dtype=np.uint8)
    err = np.zeros(n, dtype=np.int32)
    ctr = np.zeros(3, dtype=np.uint64)
    lib().orc_check(program.ctypes.data, C.addressof(tab), items.ctypes.data, n, now_us, max_depth,
                    threads, perm.ctypes.data, err.ctypes.data, ctr.ctypes.data)
    return perm, err, dict(rows=int(ctr[0]), probes=int(ctr[1]), edges=int(ctr[2]))


def check_quota(program: np.ndarray, csr_table, items: np.ndarray, limits: np.ndarray, used: np.ndarray,
                now_us: int = 0, max_depth: int = 50, threads: int = 1):
    """check() with threshold caveats: caveated edge k holds while the check's value
    used[context_slot - 1] is below limits[k] (INT64_MIN: an evaluation error; slot 0:
    unresolved). Returns (perm, err)."""
    tab, _keep = csr_table
    items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
    program = np.ascontiguousarray(program, dtype=np.int32)
    limits = np.ascontiguousarray(limits, dtype=np.int64)
    used = np.ascontiguousarray(used, dtype=np.int64)
    n = len(items)
    perm = np.zeros(n, dtype=np.uint8)
    err = np.zeros(n, dtype=np.int32)
    lib().orc_check_quota(program.ctypes.data, C.addressof(tab), items.ctypes.data, n, now_us, max_depth,
                          threads, perm.ctypes.data, err.ctypes.data, None, limits.ctypes.data,
                          used.ctypes.data, len(used))
    return perm, err


def count_bfs(program: np.ndarray, csr_table, items: np.ndarray, threads: int = 1):
    """SURVEY §8d counting rule (union-only programs)."""
    tab, _keep = csr_table
    items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
    program = np.ascontiguousarray(program, dtype=np.int32)
    ctr = np.zeros(5, dtype=np.uint64)
    rc = lib().orc_count_bfs(program.ctypes.data, C.addressof(tab), items.ctypes.data, len(items),
                             threads, ctr.ctypes.data)
    if rc != 0:
        raise ValueError("count_bfs needs a union-only program")
    return dict(rows=int(ctr[0]), probes=int(ctr[1]), edges=int(ctr[2]), expanded=int(ctr[3]),
                levels=int(ctr[4]))
