"""Seeded synthetic workloads for BASELINE.json configs 2 and 3 at scale (bench + scale parity).

* config 2, ``gdocs`` — the Google-Docs schema of tests/gen.py (user / group / folder / doc,
  nested groups, parent arrows, a public-doc wildcard): 1M users, 100K groups (nesting DAG of
  6 layers), 200K folders (forest of depth 8), 2M docs, ~10M tuples at scale 1; Pareto(2.1)
  group sizes.
* config 3, ``github`` — the GitHub schema of tests/gen.py (org / team / repo with exclusion
  ``- banned``, intersection ``& org->is_member`` and ``org.all(is_member)``): 10M users, 100K
  orgs, 1M teams (nesting depth 4), 10M repos, 1% banned, ~100M tuples at scale 1.

Everything is built vectorised in torch on the GPU, directly as CSRs in the engine's public id
space (types and relations in schema definition order, oracle/corc.py ``Ids``), so the same
arrays feed the HIP engine (``gck_load_csr``) and the C oracle. Every graph is acyclic (nesting
edges only go to deeper layers). Checks: half sampled from likely-positive pairs (an owner, a
member of a granting group / team), half uniform.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np
import torch

from oracle import corc
from oracle import spicedb_ref as ref
from tests import gen
from tests.synth import _gen, _offsets, _segment_ids

ELLIPSIS = 0xFFFF
WILD = 0xFFFFFFFF


@dataclass
class Workload:
    name: str
    schema: str
    ids: corc.Ids
    counts: Dict[str, int]                       # objects per type
    csrs: List[Tuple[int, int, int, int, torch.Tensor, torch.Tensor]] = field(default_factory=list)
    # (relation id, subject type, subject relation, n_rows, offsets int64, neighbours int32)

    def t(self, name):
        return self.ids.type_id[name]

    def r(self, typ, rel):
        return self.ids.rel_id[(typ, rel)]

    @property
    def n_tuples(self) -> int:
        return int(sum(c[5].numel() for c in self.csrs))

    def find(self, typ, rel, stype, srel=None):
        rid, st = self.r(typ, rel), self.t(stype)
        sr = ELLIPSIS if srel is None else self.r(stype, srel)
        for c in self.csrs:
            if c[0] == rid and c[1] == st and c[2] == sr:
                return c
        raise KeyError((typ, rel, stype, srel))

    def oracle(self):
        """(program, csr table) for oracle/corc.py over host copies of the same arrays."""
        idx, arrays = {}, []
        for rid, st, sr, n_rows, off, nbr in self.csrs:
            idx[(rid, st, sr, False)] = len(arrays)
            arrays.append((off.to(torch.int64).cpu().numpy().astype(np.uint32),
                           nbr.cpu().numpy().view(np.uint32), None, None, n_rows))
        return corc.encode_program(self.ids, idx), corc.make_csr_table(arrays)


def _csr(gen_, n_rows: int, deg: torch.Tensor, subjects) -> Tuple[torch.Tensor, torch.Tensor]:
    """CSR with `deg[r]` draws per row r of subjects(row_ids) (int64), sorted, duplicates dropped;
    the wildcard id 0xFFFFFFFF sorts last."""
    dev = deg.device
    off0 = _offsets(deg)
    total = int(off0[-1])
    if total == 0:
        return torch.zeros(n_rows + 1, dtype=torch.int64, device=dev), torch.zeros(0, dtype=torch.int32, device=dev)
    row = _segment_ids(off0, total)
    s = subjects(row)
    key = torch.unique((row << 32) | s)
    r, s = key >> 32, key & 0xFFFFFFFF
    off = _offsets(torch.bincount(r, minlength=n_rows))
    return off, (s - ((s >= 2 ** 31).to(torch.int64) << 32)).to(torch.int32)  # u32 bits in an int32 tensor


def _uniform(gen_, lo, hi):
    """subjects(row) -> uniform ids in [lo, hi) (lo/hi ints or per-row int64 tensors)."""
    def f(row):
        a = lo[row] if torch.is_tensor(lo) else lo
        b = hi[row] if torch.is_tensor(hi) else hi
        u = torch.rand(row.numel(), generator=gen_, device=row.device, dtype=torch.float64)
        return (a + torch.floor(u * (b - a))).to(torch.int64)
    return f


def _poisson(gen_, n, mean, device):
    return torch.poisson(torch.full((n,), float(mean), device=device), generator=gen_).to(torch.int64)


def _pareto(gen_, n, mean, cap, device, alpha=2.1):
    x_m = mean * (alpha - 1) / alpha
    u = torch.rand(n, generator=gen_, device=device, dtype=torch.float64)
    return torch.floor(x_m * torch.pow(1.0 - u, -1.0 / alpha)).clamp_(1, cap).to(torch.int64)


def _layers(n, k, device):
    """Layer of every id when n ids are split into k equal blocks, and the block starts."""
    start = torch.tensor([n * l // k for l in range(k + 1)], dtype=torch.int64, device=device)
    layer = torch.bucketize(torch.arange(n, device=device), start[1:], right=True)
    return layer, start


def gdocs(scale: float = 1.0, seed: int = 20251003, device="cuda") -> Workload:
    g = _gen(device, seed)
    U, G, F, D = (max(64, int(x * scale)) for x in (1_000_000, 100_000, 200_000, 2_000_000))
    W = Workload("config2-gdocs", gen.GDOCS, corc.Ids(ref.Schema(gen.GDOCS)),
                 {"user": U, "group": G, "folder": F, "doc": D})
    add = W.csrs.append
    t, r = W.t, W.r
    # groups: Pareto sizes of direct users; nesting DAG of 6 layers (children in deeper layers)
    add((r("group", "member"), t("user"), ELLIPSIS, G, *_csr(g, G, _pareto(g, G, 8.0, U, device), _uniform(g, 0, U))))
    gl, gs = _layers(G, 6, device)
    gdeg = torch.where(gl < 5, _poisson(g, G, 0.6, device), torch.zeros_like(gl))
    add((r("group", "member"), t("group"), r("group", "member"), G,
         *_csr(g, G, gdeg, _uniform(g, gs[(gl + 1).clamp(max=5)], G))))
    # folders: forest of depth 8 (parent in the layer above), viewers / editors
    fl, fs = _layers(F, 8, device)
    fdeg = (fl > 0).to(torch.int64)
    add((r("folder", "parent"), t("folder"), ELLIPSIS, F, *_csr(g, F, fdeg, _uniform(g, fs[(fl - 1).clamp(min=0)], fs[fl]))))
    for rel, mu, mg in (("viewer", 1.0, 0.5), ("editor", 0.5, 0.3)):
        add((r("folder", rel), t("user"), ELLIPSIS, F, *_csr(g, F, _poisson(g, F, mu, device), _uniform(g, 0, U))))
        add((r("folder", rel), t("group"), r("group", "member"), F,
             *_csr(g, F, _poisson(g, F, mg, device), _uniform(g, 0, G))))
    # docs: one parent folder, one owner, viewers (0.5 % public: user:*), editors
    one = torch.ones(D, dtype=torch.int64, device=device)
    add((r("doc", "parent"), t("folder"), ELLIPSIS, D, *_csr(g, D, one, _uniform(g, 0, F))))
    add((r("doc", "owner"), t("user"), ELLIPSIS, D, *_csr(g, D, one, _uniform(g, 0, U))))
    vdeg = _poisson(g, D, 1.0, device)
    public = torch.rand(D, generator=g, device=device) < 0.005
    vu = _uniform(g, 0, U)
    add((r("doc", "viewer"), t("user"), ELLIPSIS, D,
         *_csr(g, D, vdeg + public.to(torch.int64),
               lambda row: torch.where(public[row] & (torch.rand(row.numel(), generator=g, device=device) < 0.5),
                                       torch.full_like(row, WILD), vu(row)))))
    add((r("doc", "viewer"), t("group"), r("group", "member"), D,
         *_csr(g, D, _poisson(g, D, 0.5, device), _uniform(g, 0, G))))
    add((r("doc", "editor"), t("user"), ELLIPSIS, D, *_csr(g, D, _poisson(g, D, 0.5, device), _uniform(g, 0, U))))
    add((r("doc", "editor"), t("group"), r("group", "member"), D,
         *_csr(g, D, _poisson(g, D, 0.2, device), _uniform(g, 0, G))))
    return W


def github(scale: float = 1.0, seed: int = 20251003, device="cuda") -> Workload:
    g = _gen(device, seed)
    U, O, T, R = (max(64, int(x * scale)) for x in (10_000_000, 100_000, 1_000_000, 10_000_000))
    W = Workload("config3-github", gen.GITHUB, corc.Ids(ref.Schema(gen.GITHUB)),
                 {"user": U, "team": T, "org": O, "repo": R})
    add = W.csrs.append
    t, r = W.t, W.r
    # teams: maintainers, Pareto direct members, nesting of depth 4 (subteams in deeper layers)
    add((r("team", "maintainer"), t("user"), ELLIPSIS, T, *_csr(g, T, _poisson(g, T, 1.0, device), _uniform(g, 0, U))))
    add((r("team", "direct_member"), t("user"), ELLIPSIS, T,
         *_csr(g, T, _pareto(g, T, 12.0, U, device), _uniform(g, 0, U))))
    tl, ts = _layers(T, 4, device)
    tdeg = torch.where(tl < 3, _poisson(g, T, 0.6, device), torch.zeros_like(tl))
    add((r("team", "direct_member"), t("team"), r("team", "member"), T,
         *_csr(g, T, tdeg, _uniform(g, ts[(tl + 1).clamp(max=3)], T))))
    # orgs: admins, Pareto user members, member teams
    add((r("org", "admin"), t("user"), ELLIPSIS, O, *_csr(g, O, _poisson(g, O, 2.0, device), _uniform(g, 0, U))))
    add((r("org", "member"), t("user"), ELLIPSIS, O, *_csr(g, O, _pareto(g, O, 80.0, U, device), _uniform(g, 0, U))))
    add((r("org", "member"), t("team"), r("team", "member"), O,
         *_csr(g, O, _poisson(g, O, 10.0, device), _uniform(g, 0, T))))
    # repos: one org, readers / writers / admins (users and teams), 1 % banned users
    one = torch.ones(R, dtype=torch.int64, device=device)
    add((r("repo", "org"), t("org"), ELLIPSIS, R, *_csr(g, R, one, _uniform(g, 0, O))))
    for rel, mu, mt in (("reader", 3.0, 1.0), ("writer", 1.5, 0.5), ("admin", 0.5, 0.2)):
        add((r("repo", rel), t("user"), ELLIPSIS, R, *_csr(g, R, _poisson(g, R, mu, device), _uniform(g, 0, U))))
        add((r("repo", rel), t("team"), r("team", "member"), R,
             *_csr(g, R, _poisson(g, R, mt, device), _uniform(g, 0, T))))
    banned = (torch.rand(R, generator=g, device=device) < 0.01).to(torch.int64)
    add((r("repo", "banned"), t("user"), ELLIPSIS, R, *_csr(g, R, banned, _uniform(g, 0, U))))
    return W


def _row_pick(gen_, off, nbr, rows):
    """A random neighbour of each row (rows with no neighbours -> -1)."""
    d = off[rows + 1] - off[rows]
    u = torch.rand(rows.numel(), generator=gen_, device=rows.device)
    p = off[rows] + torch.floor(u * d.to(torch.float32)).to(torch.int64).clamp(min=0)
    p = torch.minimum(p, (off[rows + 1] - 1).clamp(min=0))
    v = nbr[p.clamp(max=max(nbr.numel() - 1, 0))].to(torch.int64) & 0xFFFFFFFF
    return torch.where(d > 0, v, torch.full_like(v, -1))


def checks(W: Workload, n: int = 65536, seed: int = 7) -> torch.Tensor:
    """gck_item records (20 B each) as a uint8 tensor [n, 20]: `doc#view|edit@user` (gdocs) or
    `repo#read|write@user` (github), half from likely-positive pairs, half uniform."""
    dev = W.csrs[0][4].device
    g = _gen(dev, seed)
    res_t = "doc" if "doc" in W.counts else "repo"
    perms = ("view", "edit") if res_t == "doc" else ("read", "write")
    n_res, n_users = W.counts[res_t], W.counts["user"]
    res = torch.floor(torch.rand(n, generator=g, device=dev, dtype=torch.float64) * n_res).to(torch.int64)
    which = torch.randint(0, 2, (n,), generator=g, device=dev)
    grp_t, grp_rel = ("group", "member") if res_t == "doc" else ("team", "member")
    grant = "viewer" if res_t == "doc" else "reader"
    # likely positive: a direct user of the granting relation, or a member of a granting group
    _, _, _, _, uo, un = W.find(res_t, grant, "user")
    direct = _row_pick(g, uo, un, res)
    _, _, _, _, go, gn = W.find(res_t, grant, grp_t, grp_rel)
    grp = _row_pick(g, go, gn, res)
    if grp_t == "group":
        _, _, _, _, mo, mn = W.find("group", "member", "user")
    else:
        _, _, _, _, mo, mn = W.find("team", "direct_member", "user")
    member = _row_pick(g, mo, mn, grp.clamp(min=0))
    member = torch.where(grp >= 0, member, torch.full_like(member, -1))
    pos = torch.where(torch.rand(n, generator=g, device=dev) < 0.5, direct, member)
    pos = torch.where(pos == WILD, torch.full_like(pos, -1), pos)
    rnd = torch.floor(torch.rand(n, generator=g, device=dev, dtype=torch.float64) * n_users).to(torch.int64)
    is_pos = (torch.arange(n, device=dev) < n // 2) & (pos >= 0)
    user = torch.where(is_pos, pos, rnd)
    items = torch.zeros(n, 5, dtype=torch.int64, device=dev)
    p_ids = torch.tensor([W.r(res_t, p) for p in perms], dtype=torch.int64, device=dev)
    items[:, 0] = W.t(res_t) | (p_ids[which] << 16)
    items[:, 1] = res
    items[:, 2] = W.t("user") | (ELLIPSIS << 16)
    items[:, 3] = user
    items = items - ((items >= 2 ** 31).to(torch.int64) << 32)
    return items.to(torch.int32).view(torch.uint8).reshape(n, 20)


CONFIGS = {"gdocs": gdocs, "github": github}
