"""Seeded synthetic workload at BASELINE.json scale (bench + scale parity tests).

Config 4 of BASELINE.json / SURVEY.md §8d — "deep nested-group hierarchy (depth 20+,
power-law fan-out), 1B tuples", schema::

    definition user {}
    definition group { relation member: user | group#member }
    definition doc   { relation viewer: group#member   permission view = viewer }

Generator (all vectorised in torch, on the GPU for the 1B case):

* groups in ``layers`` = 25 layers (group->group depth 24); layer sizes grow geometrically
  (x1.3 per layer); every group below layer 0 gets one parent in the layer above, chosen with
  a skewed draw ``floor(n_above * u**2)`` so that child counts (fan-out) are heavy-tailed;
  2 % of groups get a second parent (a DAG, still acyclic: edges only go one layer down);
* direct user members per group: Pareto(alpha=2.1) sizes, capped at 1M, each group's members a
  sorted random subset of a random window of the user id space (strictly increasing gaps);
* docs: 1-3 viewer groups each, uniform over all groups;
* checks: ``doc#view@user``, half sampled from positive reachable pairs (doc -> viewer group
  -> 0..24 random descents, uniform, stopping at a leaf group -> a random member), half uniform
  (doc, user) pairs: positive answers come from every depth of the DAG, down to 24 group hops.

Returns CSR arrays in the engine's id space (types user=0, group=1, doc=2; relations
member=0, viewer=1, view=2) — the same arrays feed the HIP engine (``gck_load_csr``) and the
C oracle (``oracle/corc.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict

import numpy as np
import torch

SCHEMA = """
definition user {}
definition group {
  relation member: user | group#member
}
definition doc {
  relation viewer: group#member
  permission view = viewer
}
"""

T_USER, T_GROUP, T_DOC = 0, 1, 2
R_MEMBER, R_VIEWER, R_VIEW = 0, 1, 2
ELLIPSIS = 0xFFFF


@dataclass
class Graph:
    n_users: int
    n_groups: int
    n_docs: int
    layer_start: torch.Tensor       # int64[layers+1]
    # CSRs (int32 tensors interpreted as uint32; offsets int64 while building)
    mem_user_off: torch.Tensor
    mem_user_nbr: torch.Tensor
    mem_group_off: torch.Tensor
    mem_group_nbr: torch.Tensor
    viewer_off: torch.Tensor
    viewer_nbr: torch.Tensor

    @property
    def n_tuples(self) -> int:
        return int(self.mem_user_nbr.numel() + self.mem_group_nbr.numel() + self.viewer_nbr.numel())

    def csrs(self):
        """(relation, subject type, subject relation, n_rows, offsets, neighbours)."""
        return [
            (R_MEMBER, T_USER, ELLIPSIS, self.n_groups, self.mem_user_off, self.mem_user_nbr),
            (R_MEMBER, T_GROUP, R_MEMBER, self.n_groups, self.mem_group_off, self.mem_group_nbr),
            (R_VIEWER, T_GROUP, R_MEMBER, self.n_docs, self.viewer_off, self.viewer_nbr),
        ]


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def _offsets(counts: torch.Tensor) -> torch.Tensor:
    off = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
    off[1:] = torch.cumsum(counts.to(torch.int64), 0)
    return off


def _segment_ids(off: torch.Tensor, total: int) -> torch.Tensor:
    """row id of every element of a CSR with offsets `off`."""
    n = off.numel() - 1
    counts = off[1:] - off[:-1]
    return torch.repeat_interleave(torch.arange(n, device=off.device), counts, output_size=total)


def sizes_for(target_tuples: float):
    """Scale the config so that the tuple count is ~target (1e9 = the BASELINE config)."""
    scale = target_tuples / 1e9
    n_users = max(1000, int(200e6 * scale))
    n_groups = max(256, int(8e6 * scale))
    n_docs = max(256, int(30e6 * scale))
    return n_users, n_groups, n_docs


def build(target_tuples: float = 1e9, seed: int = 20251003, device="cuda", layers: int = 25,
          alpha: float = 2.1, member_cap: int = 1_000_000) -> Graph:
    n_users, n_groups, n_docs = sizes_for(target_tuples)
    gen = _gen(device, seed)
    # ---- layers ---------------------------------------------------------------------
    r = 1.3
    w = np.array([r ** l for l in range(layers)])
    sizes = np.maximum(1, np.floor(n_groups * w / w.sum())).astype(np.int64)
    sizes[-1] += n_groups - sizes.sum()
    layer_start = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int64, device=device)
    ls = layer_start.tolist()
    # ---- group -> subgroup edges (parent row lists its children) ---------------------
    parents, children = [], []
    for l in range(1, layers):
        n_above, n_here = sizes[l - 1], sizes[l]
        kids = torch.arange(ls[l], ls[l + 1], device=device)
        u = torch.rand(n_here, generator=gen, device=device)
        par = ls[l - 1] + torch.floor(n_above * u * u).to(torch.int64).clamp_(max=n_above - 1)
        parents.append(par)
        children.append(kids)
        second = torch.rand(n_here, generator=gen, device=device) < 0.02
        if second.any():
            u2 = torch.rand(int(second.sum()), generator=gen, device=device)
            par2 = ls[l - 1] + torch.floor(n_above * u2).to(torch.int64).clamp_(max=n_above - 1)
            parents.append(par2)
            children.append(kids[second])
    par = torch.cat(parents)
    kid = torch.cat(children)
    key = par * (n_groups + 1) + kid
    key = torch.unique(key)  # sorted, drops duplicate (parent, child) pairs
    par, kid = key // (n_groups + 1), key % (n_groups + 1)
    mem_group_off = _offsets(torch.bincount(par, minlength=n_groups))
    mem_group_nbr = kid.to(torch.int32)
    # ---- direct user members: Pareto sizes, sorted strictly increasing ids ----------
    non_user = n_docs * 2 + mem_group_nbr.numel()
    mean = max(2.0, (target_tuples - non_user) / n_groups)
    x_m = mean * (alpha - 1) / alpha
    u = torch.rand(n_groups, generator=gen, device=device, dtype=torch.float64)
    sz = torch.floor(x_m * torch.pow(1.0 - u, -1.0 / alpha)).clamp_(1, min(member_cap, n_users))
    sz = sz.to(torch.int64)
    off = _offsets(sz)
    total = int(off[-1])
    row = _segment_ids(off, total)
    max_gap = torch.clamp(n_users // sz, min=1)                     # per row: s * gap <= U
    gaps = 1 + torch.floor(torch.rand(total, generator=gen, device=device) *
                           max_gap[row].to(torch.float32)).to(torch.int64).clamp_(max=max_gap[row] - 1)
    csum = torch.cumsum(gaps, 0)
    row_base = torch.zeros(n_groups, dtype=torch.int64, device=device)
    row_base[1:] = csum[off[1:-1] - 1]
    within = csum - row_base[row]                                     # 1..sum per row
    span = torch.zeros(n_groups, dtype=torch.int64, device=device)
    span = within[off[1:] - 1]
    start = torch.floor(torch.rand(n_groups, generator=gen, device=device, dtype=torch.float64) *
                        (n_users - span).clamp(min=0).to(torch.float64)).to(torch.int64)
    ids = start[row] + within - 1
    del gaps, csum, within, row
    mem_user_nbr = ids.to(torch.int32)
    del ids
    # ---- docs ---------------------------------------------------------------------------
    k = 1 + torch.floor(torch.rand(n_docs, generator=gen, device=device) * 3).to(torch.int64)
    voff = _offsets(k)
    vtot = int(voff[-1])
    vrow = _segment_ids(voff, vtot)
    vg = torch.floor(torch.rand(vtot, generator=gen, device=device, dtype=torch.float64) * n_groups).to(torch.int64)
    vkey = torch.unique(vrow * n_groups + vg)
    vrow, vg = vkey // n_groups, vkey % n_groups
    viewer_off = _offsets(torch.bincount(vrow, minlength=n_docs))
    viewer_nbr = vg.to(torch.int32)
    return Graph(n_users, n_groups, n_docs, layer_start, off, mem_user_nbr, mem_group_off,
                 mem_group_nbr, viewer_off, viewer_nbr)


def checks(G: Graph, n: int = 65536, seed: int = 7, positive_frac: float = 0.5,
           max_descend: int = 24) -> torch.Tensor:
    """Check items (gck_item records, 20 B each) as a uint8 tensor [n, 20] on G's device."""
    dev = G.viewer_nbr.device
    gen = _gen(dev, seed)
    n_pos = int(n * positive_frac)
    # positive: doc -> one of its viewer groups -> descend -> random member
    docs = torch.floor(torch.rand(n, generator=gen, device=dev) * G.n_docs).to(torch.int64)
    vo = G.viewer_off
    deg = (vo[docs + 1] - vo[docs])
    pick = vo[docs] + torch.floor(torch.rand(n, generator=gen, device=dev) * deg.to(torch.float32)).to(torch.int64).clamp_(max=deg - 1)
    grp = G.viewer_nbr[pick.clamp(min=0)].to(torch.int64)
    go = G.mem_group_off
    steps = torch.floor(torch.rand(n, generator=gen, device=dev) * (max_descend + 1)).to(torch.int64)
    for s in range(max_descend):
        d = go[grp + 1] - go[grp]
        move = (steps > s) & (d > 0)
        ch = go[grp] + torch.floor(torch.rand(n, generator=gen, device=dev) * d.to(torch.float32)).to(torch.int64).clamp_(max=(d - 1).clamp(min=0))
        grp = torch.where(move, G.mem_group_nbr[ch.clamp(max=G.mem_group_nbr.numel() - 1)].to(torch.int64), grp)
    uo = G.mem_user_off
    ud = uo[grp + 1] - uo[grp]
    up = uo[grp] + torch.floor(torch.rand(n, generator=gen, device=dev) * ud.to(torch.float32)).to(torch.int64).clamp_(max=(ud - 1).clamp(min=0))
    pos_user = G.mem_user_nbr[up].to(torch.int64)
    rnd_user = torch.floor(torch.rand(n, generator=gen, device=dev, dtype=torch.float64) * G.n_users).to(torch.int64)
    is_pos = torch.arange(n, device=dev) < n_pos
    user = torch.where(is_pos, pos_user, rnd_user)
    perm = torch.randperm(n, generator=gen, device=dev)
    docs, user = docs[perm], user[perm]
    items = torch.zeros(n, 5, dtype=torch.int32, device=dev)
    # (resource_type | permission << 16), resource_id, (subject_type | subject_relation << 16), subject_id, ctx
    items[:, 0] = T_DOC | (R_VIEW << 16)
    items[:, 1] = docs.to(torch.int32)
    items[:, 2] = (T_USER | (ELLIPSIS << 16)) - (1 << 32) if (T_USER | (ELLIPSIS << 16)) >= 2 ** 31 else (T_USER | (ELLIPSIS << 16))
    items[:, 3] = user.to(torch.int32)
    return items.view(torch.uint8).reshape(n, 20)


def host_arrays(G: Graph) -> Dict[str, np.ndarray]:
    """uint32 host copies of every CSR (offsets narrowed to uint32)."""
    out = {}
    for name in ("mem_user_off", "mem_user_nbr", "mem_group_off", "mem_group_nbr", "viewer_off", "viewer_nbr"):
        t = getattr(G, name)
        if t.dtype == torch.int64:
            t = t.to(torch.int32)
        out[name] = t.cpu().numpy().view(np.uint32)
    return out


class NestedChurn:
    """Watch churn on the config-4 graph (client/client.go:370-413 UpdatesSinceRevision: CREATE /
    TOUCH / DELETE of relationships) with the graph's state kept on the host as sorted
    (object << 32 | subject) keys per relation kind, so that the C oracle can check any revision.
    Updates hit all three kinds: user memberships, group nesting (acyclic: a parent in a higher
    layer) and document viewers; `cycle=True` adds one nesting edge from a deep descendant back up
    to a group above it, which closes a cycle in the hierarchy."""

    KINDS = [(R_MEMBER, T_USER, ELLIPSIS), (R_MEMBER, T_GROUP, R_MEMBER), (R_VIEWER, T_GROUP, R_MEMBER)]

    def __init__(self, G: Graph, seed: int = 99):
        self.G = G
        self.rng = np.random.default_rng(seed)
        H = host_arrays(G)
        self.rows = {R_MEMBER: G.n_groups, R_VIEWER: G.n_docs}
        self.layer_start = G.layer_start.cpu().numpy()
        self.keys = {}
        for kind, (o, nb) in zip(self.KINDS, (("mem_user_off", "mem_user_nbr"), ("mem_group_off", "mem_group_nbr"),
                                              ("viewer_off", "viewer_nbr"))):
            off, nbr = H[o].astype(np.int64), H[nb].astype(np.uint64)
            row = np.repeat(np.arange(off.size - 1, dtype=np.uint64), np.diff(off))
            self.keys[kind] = (row << np.uint64(32)) | nbr  # rows ascending, sorted within: sorted

    def _layer_of(self, g):
        return np.searchsorted(self.layer_start, g, side="right") - 1

    def batch(self, n: int, cycle: bool = False, share=(0.9, 0.05, 0.05)):
        """n updates split over memberships / nesting / viewers by `share` (a 0 share: none of
        that kind, e.g. (0.95, 0, 0.05) leaves the hierarchy as it is)."""
        from gochugaru_amd.engine import UPDATE_CREATE, UPDATE_DELETE, UPDATE_DTYPE, UPDATE_TOUCH
        rng, G = self.rng, self.G
        out = []
        for kind, frac in zip(self.KINDS, share):
            rel, st, sr = kind
            if frac <= 0 and not (cycle and kind == (R_MEMBER, T_GROUP, R_MEMBER)):
                continue
            k = max(1, int(n * frac))
            keys = self.keys[kind]
            ops = rng.choice([UPDATE_CREATE, UPDATE_TOUCH, UPDATE_DELETE], size=k, p=[0.45, 0.45, 0.10])
            n_new = int((ops == UPDATE_CREATE).sum())
            rows = rng.integers(0, self.rows[rel], n_new)
            if kind == (R_MEMBER, T_USER, ELLIPSIS):
                subj = rng.integers(0, G.n_users, n_new)
            elif kind == (R_MEMBER, T_GROUP, R_MEMBER):
                # a parent in a higher layer than the child: the hierarchy stays acyclic
                lay = self._layer_of(rows)
                deeper = lay + 1 < self.layer_start.size - 1
                lo = self.layer_start[np.minimum(lay + 1, self.layer_start.size - 2)]
                subj = lo + (rng.random(n_new) * (G.n_groups - lo)).astype(np.int64)
                subj = np.where(deeper, subj, -1)
            else:
                subj = rng.integers(0, G.n_groups, n_new)
            new = (rows.astype(np.uint64) << np.uint64(32)) | subj.astype(np.uint64)
            new = new[subj >= 0]
            old = keys[rng.integers(0, keys.size, k - n_new)] if keys.size else np.zeros(0, np.uint64)
            ukeys = np.concatenate([new, old])
            uops = np.concatenate([ops[ops == UPDATE_CREATE][: new.size], ops[ops != UPDATE_CREATE]])
            if cycle and kind == (R_MEMBER, T_GROUP, R_MEMBER):
                ukeys, uops = self._with_cycle(ukeys, uops)
            ukeys, first = np.unique(ukeys, return_index=True)
            uops = uops[first]
            # host state: drop every updated key, insert the upserts (both sides sorted: O(n) copies)
            pos = np.searchsorted(keys, ukeys)
            hit = (pos < keys.size) & (keys[np.minimum(pos, max(keys.size - 1, 0))] == ukeys)
            keep = np.ones(keys.size, dtype=bool)
            keep[pos[hit]] = False
            kept = keys[keep]
            up = uops != UPDATE_DELETE
            ins = ukeys[up]
            self.keys[kind] = np.insert(kept, np.searchsorted(kept, ins), ins)
            u = np.zeros(ukeys.size, dtype=UPDATE_DTYPE)
            u["op"] = uops
            t = u["tuple"]
            t["resource_type"] = T_GROUP if rel == R_MEMBER else T_DOC
            t["relation"] = rel
            t["resource_id"] = ukeys >> np.uint64(32)
            t["subject_type"] = st
            t["subject_relation"] = sr
            t["subject_id"] = ukeys & np.uint64(0xFFFFFFFF)
            u["tuple"] = t
            out.append(u)
        return np.concatenate(out)

    def _with_cycle(self, ukeys, uops):
        """One CREATE of `D#member@A#member` where D descends from A: A -> ... -> D -> A."""
        from gochugaru_amd.engine import UPDATE_CREATE
        keys = self.keys[(R_MEMBER, T_GROUP, R_MEMBER)]
        rows = (keys >> np.uint64(32)).astype(np.int64)
        a = int(rows[self.rng.integers(0, rows.size)])
        d = a
        for _ in range(6):  # walk down first children
            lo = np.searchsorted(rows, d)
            if lo >= rows.size or rows[lo] != d:
                break
            d = int(keys[lo] & np.uint64(0xFFFFFFFF))
        if d == a:
            return ukeys, uops
        self.cycle = (a, d)
        k = np.uint64((d << 32) | a)
        return np.concatenate([ukeys, [k]]), np.concatenate([uops, [UPDATE_CREATE]])

    def csrs(self):
        """Host CSRs of the current state, in Graph.csrs() order (uint32 offsets / neighbours)."""
        out = []
        for kind in self.KINDS:
            rel = kind[0]
            keys = self.keys[kind]
            n_rows = self.rows[rel]
            off = np.zeros(n_rows + 1, dtype=np.uint32)
            off[1:] = np.cumsum(np.bincount((keys >> np.uint64(32)).astype(np.int64), minlength=n_rows))
            out.append((off, (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), n_rows))
        return out

    def oracle(self):
        """(program, CSR table) of the C oracle over the current state."""
        from oracle import corc
        from oracle import spicedb_ref as ref
        ids = corc.Ids(ref.Schema(SCHEMA))
        idx = {(R_MEMBER, T_USER, ELLIPSIS, False): 0, (R_MEMBER, T_GROUP, R_MEMBER, False): 1,
               (R_VIEWER, T_GROUP, R_MEMBER, False): 2}
        tab = corc.make_csr_table([(off, nbr, None, None, n) for off, nbr, n in self.csrs()])
        return corc.encode_program(ids, idx), tab
