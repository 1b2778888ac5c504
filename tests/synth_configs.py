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


# ---- config 5: caveats + Watch churn ---------------------------------------------------------

MIXED_SCHEMA = """
caveat only_on_tuesday(day_of_the_week string) {
  day_of_the_week == "tuesday"
}
definition user {}
definition group {
  relation member: user | group#member
}
definition folder {
  relation parent: folder
  relation viewer: user | group#member | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday
  permission edit = editor + parent->edit
  permission view = viewer + edit + parent->view
}
definition doc {
  relation parent: folder
  relation owner: user
  relation viewer: user | user:* | group#member | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday
  permission edit = owner + editor + parent->edit
  permission view = viewer + edit + parent->view
}
"""

CONTEXTS = ['{"day_of_the_week":"tuesday"}', '{"day_of_the_week":"monday"}']  # context slots 1, 2
CHURN_KINDS = [("folder", "viewer"), ("folder", "editor"), ("doc", "viewer"), ("doc", "editor")]


class Mixed:
    """BASELINE.json config 5: the config-2 graph with 10 % of the folder / doc viewer and editor
    user tuples caveated ``with only_on_tuesday``, checks of which half carry a check-time
    context (tuesday: the caveat holds, monday: it fails) and half none (CONDITIONAL), and Watch
    churn on those relations (CREATE / TOUCH / DELETE 45 / 45 / 10, TOUCH toggling the caveat).

    The state of the churned user kinds is kept on the host as sorted (object << 32 | subject)
    keys with a caveat flag, so the expected answers after any number of update batches come
    from the C oracle over a rebuilt snapshot: caveats can only be true, false or missing here,
    so the three context classes are three oracle runs (caveated edges plain / absent /
    CONDITIONAL)."""

    def __init__(self, scale: float = 1.0, seed: int = 20251003, device="cuda", cav_frac: float = 0.1):
        self.W = W = gdocs(scale, seed, device)
        W.name, W.schema = "config5-mixed", MIXED_SCHEMA
        W.ids = corc.Ids(ref.Schema(MIXED_SCHEMA))
        self.device = device
        self.rng = np.random.default_rng(seed)
        self.kinds = [(W.r(t, r), W.t("user"), ELLIPSIS, W.counts[t]) for t, r in CHURN_KINDS]
        self.static = [c for c in W.csrs if (c[0], c[1], c[2]) not in {k[:3] for k in self.kinds}]
        self.state = {}  # kind -> (keys u64 sorted, caveated bool)
        for rid, st, sr, n_rows in self.kinds:
            off, nbr = W.find(*self._names(rid))[4:6]
            row = _segment_ids(off, nbr.numel()).cpu().numpy().astype(np.uint64)
            sid = nbr.cpu().numpy().view(np.uint32).astype(np.uint64)
            keys = (row << np.uint64(32)) | sid
            cav = (self.rng.random(keys.size) < cav_frac) & (sid != WILD)
            self.state[(rid, st, sr)] = (keys, cav)

    def _names(self, rid):
        t, r = self.W.ids.rels[rid]
        return t, r, "user"

    # ---- engine ingest ------------------------------------------------------------------------
    def load(self, eng, plain_csr_loader, cav_instance: int):
        """Static CSRs and the plain part of the churned kinds through `plain_csr_loader`
        (gck_load_csr), the caveated part as interned tuples (gck_add_tuples)."""
        from gochugaru_amd.engine import TUPLE_DTYPE
        for c in self.static:
            plain_csr_loader(*c)
        tups = []
        for (rid, st, sr), (keys, cav) in self.state.items():
            n_rows = self.W.counts[self.W.ids.rels[rid][0]]
            off, nbr = self._csr(keys[~cav], n_rows)
            plain_csr_loader(rid, st, sr, n_rows, torch.from_numpy(off.astype(np.int64)).to(self.device),
                             torch.from_numpy(nbr.view(np.int32)).to(self.device))
            t = np.zeros(int(cav.sum()), dtype=TUPLE_DTYPE)
            t["resource_type"] = self.W.t(self.W.ids.rels[rid][0])
            t["relation"] = rid
            t["resource_id"] = keys[cav] >> np.uint64(32)
            t["subject_type"] = st
            t["subject_relation"] = sr
            t["subject_id"] = keys[cav] & np.uint64(0xFFFFFFFF)
            t["caveat"] = cav_instance
            tups.append(t)
        eng.add_tuples(np.concatenate(tups))

    @staticmethod
    def _csr(keys, n_rows):
        row = (keys >> np.uint64(32)).astype(np.int64)
        off = np.zeros(n_rows + 1, dtype=np.uint32)
        off[1:] = np.cumsum(np.bincount(row, minlength=n_rows))
        return off, (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    # ---- Watch churn ----------------------------------------------------------------------------
    def churn(self, n: int, cav_instance: int):
        """One Watch batch of n updates (unique relationships) as UPDATE_DTYPE records, applied
        to the host state as well."""
        from gochugaru_amd.engine import UPDATE_CREATE, UPDATE_DELETE, UPDATE_DTYPE, UPDATE_TOUCH
        rng = self.rng
        out = []
        per = np.bincount(rng.integers(0, len(self.kinds), n), minlength=len(self.kinds))
        for (rid, st, sr, n_rows), k in zip(self.kinds, per):
            keys, cav = self.state[(rid, st, sr)]
            ops = rng.choice([UPDATE_CREATE, UPDATE_TOUCH, UPDATE_DELETE], size=k, p=[0.45, 0.45, 0.10])
            n_new = int((ops == UPDATE_CREATE).sum())
            new = ((rng.integers(0, n_rows, n_new).astype(np.uint64) << np.uint64(32))
                   | rng.integers(0, self.W.counts["user"], n_new).astype(np.uint64))
            old = keys[rng.integers(0, keys.size, k - n_new)] if keys.size else np.zeros(0, np.uint64)
            ukeys = np.concatenate([new, old])
            uops = np.concatenate([ops[ops == UPDATE_CREATE], ops[ops != UPDATE_CREATE]])
            ukeys, first = np.unique(ukeys, return_index=True)
            uops = uops[first]
            ucav = rng.random(ukeys.size) < 0.1
            # TOUCH of an existing key toggles its caveat half of the time
            pos = np.searchsorted(keys, ukeys)
            exists = (pos < keys.size) & (keys[np.minimum(pos, max(keys.size - 1, 0))] == ukeys)
            toggle = (uops == UPDATE_TOUCH) & exists & (rng.random(ukeys.size) < 0.5)
            ucav = np.where(toggle, ~cav[np.minimum(pos, max(keys.size - 1, 0))], ucav)
            ucav &= (ukeys & np.uint64(0xFFFFFFFF)) != np.uint64(WILD)  # no caveated wildcard kind
            # host state: drop every updated key, re-insert the upserts
            keep = ~np.isin(keys, ukeys)
            up = uops != UPDATE_DELETE
            keys2 = np.concatenate([keys[keep], ukeys[up]])
            cav2 = np.concatenate([cav[keep], ucav[up]])
            order = np.argsort(keys2, kind="stable")
            self.state[(rid, st, sr)] = (keys2[order], cav2[order])
            u = np.zeros(ukeys.size, dtype=UPDATE_DTYPE)
            u["op"] = uops
            t = u["tuple"]
            t["resource_type"] = self.W.t(self.W.ids.rels[rid][0])
            t["relation"] = rid
            t["resource_id"] = ukeys >> np.uint64(32)
            t["subject_type"] = st
            t["subject_relation"] = sr
            t["subject_id"] = ukeys & np.uint64(0xFFFFFFFF)
            t["caveat"] = np.where(ucav & up, cav_instance, 0)
            u["tuple"] = t
            out.append(u)
        # (filled in place: np.concatenate would return the records packed, without the padding
        # UPDATE_DTYPE has, and the engine call would then convert them field by field)
        res = np.empty(sum(u.size for u in out), dtype=UPDATE_DTYPE)
        at = 0
        for u in out:
            res[at:at + u.size] = u
            at += u.size
        return res

    # ---- expected answers ------------------------------------------------------------------------
    def expected(self, items_host: np.ndarray, threads: int = 16, stats: dict = None):
        """(perm, err) for items whose context_slot is 0 (none), 1 (tuesday) or 2 (monday).
        `stats` (a dict) receives the oracle's work on the items of each context class only —
        `seconds` (the C oracle's time answering the batch once), `rows` / `edges` /
        `cav_edges` (its counting, for SURVEY §8d's algorithmic bytes)."""
        res = []
        slot = items_host["context_slot"]
        if stats is not None:
            stats.update(seconds=0.0, rows=0, edges=0, cav_edges=0)
        for m, mode in enumerate(("cond", "true", "false")):
            idx, arrays = {}, []
            for rid, st, sr, n_rows, off, nbr in self.static:
                idx[(rid, st, sr, False)] = len(arrays)
                arrays.append((off.to(torch.int64).cpu().numpy().astype(np.uint32),
                               nbr.cpu().numpy().view(np.uint32), None, None, n_rows))
            for (rid, st, sr), (keys, cav) in self.state.items():
                n_rows = self.W.counts[self.W.ids.rels[rid][0]]
                sel = np.ones(keys.size, bool) if mode == "true" else ~cav
                off, nbr = self._csr(keys[sel], n_rows)
                idx[(rid, st, sr, False)] = len(arrays)
                arrays.append((off, nbr, None, None, n_rows))
                if mode == "cond" and cav.any():
                    off, nbr = self._csr(keys[cav], n_rows)
                    idx[(rid, st, sr, True)] = len(arrays)
                    arrays.append((off, nbr, np.ones(nbr.size, np.uint32), np.zeros(nbr.size, np.int64), n_rows))
            prog = corc.encode_program(self.W.ids, idx)
            tab = corc.make_csr_table(arrays)
            res.append(corc.check(prog, tab, items_host, threads=threads)[:2])
            if stats is not None:
                import time
                sub = items_host[slot == m]
                if sub.size:
                    t0 = time.perf_counter()
                    _, _, cnt = corc.check(prog, tab, sub, threads=threads)
                    stats["seconds"] += time.perf_counter() - t0
                    stats["rows"] += cnt["rows"]
                    stats["edges"] += cnt["edges"]
                    stats["cav_edges"] += cnt.get("ext_edges", 0)
        perm = np.where(slot == 1, res[1][0], np.where(slot == 2, res[2][0], res[0][0]))
        err = np.where(slot == 1, res[1][1], np.where(slot == 2, res[2][1], res[0][1]))
        return perm, err

    def checks(self, n: int, seed: int) -> torch.Tensor:
        """Config-2 checks with context slots: 25 % tuesday, 25 % monday, 50 % none."""
        items = checks(self.W, n, seed)
        g = _gen(items.device, seed + 1)
        slot = torch.floor(torch.rand(n, generator=g, device=items.device) * 4).to(torch.int32).clamp_(max=3)
        slot = torch.where(slot >= 2, torch.zeros_like(slot), slot + 1)
        items.view(torch.int32).reshape(n, 5)[:, 4] = slot
        return items



# ---- config 5 variant: per-relationship and per-request caveat contexts ---------------------

QUOTA_SCHEMA = MIXED_SCHEMA.replace(
    'caveat only_on_tuesday(day_of_the_week string) {\n  day_of_the_week == "tuesday"\n}',
    "caveat quota(limit int, used int) {\n  used < limit\n}").replace("only_on_tuesday", "quota")
BAD_USED = np.iinfo(np.int64).min  # corc.check_quota: the context gives `used` a wrong type


class Quota(Mixed):
    """BASELINE config 5 with realistic caveat contexts: the config-2 graph with 10 % of the
    folder / doc viewer and editor user tuples caveated ``with quota``, each relationship storing
    its own ``{"limit": L}`` (L from `n_limits` distinct values, so that many partial caveat
    instances), and every check carrying its own ``{"used": U}`` (one context per request; 10 %
    carry none and stay CONDITIONAL). The caveat holds when U < L: the outcome depends on the
    (instance, context) pair, which the C oracle's threshold mode (corc.check_quota) restates."""

    def __init__(self, scale: float = 1.0, seed: int = 20251003, device="cuda", cav_frac: float = 0.1,
                 n_limits: int = 32768):
        super().__init__(scale, seed, device, cav_frac)
        W = self.W
        W.name, W.schema = "config5-quota", QUOTA_SCHEMA
        W.ids = corc.Ids(ref.Schema(QUOTA_SCHEMA))
        self.limits = np.sort(self.rng.choice(1 << 20, n_limits, replace=False)).astype(np.int64)
        # per caveated relationship: the index of its limit
        self.lim = {k: self.rng.integers(0, n_limits, int(c.sum())) for k, (_, c) in self.state.items()}

    def load(self, eng, plain_csr_loader, cav_instance=None):
        """Static and plain CSRs through `plain_csr_loader`; one caveat instance per distinct
        limit (gck_add_caveat_instance) and the caveated relationships as interned tuples."""
        from gochugaru_amd.engine import TUPLE_DTYPE
        self.inst = np.array([eng.add_caveat_instance("quota", '{"limit":%d}' % v) for v in self.limits],
                             dtype=np.uint32)
        for c in self.static:
            plain_csr_loader(*c)
        tups = []
        for (rid, st, sr), (keys, cav) in self.state.items():
            n_rows = self.W.counts[self.W.ids.rels[rid][0]]
            off, nbr = self._csr(keys[~cav], n_rows)
            plain_csr_loader(rid, st, sr, n_rows, torch.from_numpy(off.astype(np.int64)).to(self.device),
                             torch.from_numpy(nbr.view(np.int32)).to(self.device))
            t = np.zeros(int(cav.sum()), dtype=TUPLE_DTYPE)
            t["resource_type"] = self.W.t(self.W.ids.rels[rid][0])
            t["relation"] = rid
            t["resource_id"] = keys[cav] >> np.uint64(32)
            t["subject_type"] = st
            t["subject_relation"] = sr
            t["subject_id"] = keys[cav] & np.uint64(0xFFFFFFFF)
            t["caveat"] = self.inst[self.lim[(rid, st, sr)]]
            tups.append(t)
        eng.add_tuples(np.concatenate(tups))

    def checks(self, n: int, seed: int, bad: float = 0.0):
        """(items [n, 20] u8 on the device, used values i64[n_slots], context texts): check i
        has context slot i + 1 with its own `used` (10 % have slot 0: no context); a fraction
        `bad` of the contexts give `used` a string (an evaluation error when a walk meets it)."""
        items = checks(self.W, n, seed)
        rng = np.random.default_rng(seed + 7)
        used = rng.integers(0, 1 << 20, n).astype(np.int64)
        texts = ['{"used":%d}' % u for u in used]
        for i in np.nonzero(rng.random(n) < bad)[0]:
            used[i] = BAD_USED
            texts[i] = '{"used":"many"}'
        slot = np.arange(1, n + 1, dtype=np.int64)
        slot[rng.random(n) < 0.1] = 0
        items.view(torch.int32).reshape(n, 5)[:, 4] = torch.from_numpy(slot.astype(np.int32)).to(items.device)
        return items, used, texts

    def expected(self, items_host: np.ndarray, used: np.ndarray, threads: int = 16):
        """(perm, err) from the C oracle's threshold mode over the same snapshot."""
        prog, tab, limits = self.oracle()
        return corc.check_quota(prog, tab, items_host, limits, used, threads=threads)

    def oracle(self):
        """(program, csr table, limit per caveat id) for corc.check_quota."""
        idx, arrays = {}, []
        for rid, st, sr, n_rows, off, nbr in self.static:
            idx[(rid, st, sr, False)] = len(arrays)
            arrays.append((off.to(torch.int64).cpu().numpy().astype(np.uint32),
                           nbr.cpu().numpy().view(np.uint32), None, None, n_rows))
        for (rid, st, sr), (keys, cav) in self.state.items():
            n_rows = self.W.counts[self.W.ids.rels[rid][0]]
            off, nbr = self._csr(keys[~cav], n_rows)
            idx[(rid, st, sr, False)] = len(arrays)
            arrays.append((off, nbr, None, None, n_rows))
            if cav.any():
                off, nbr = self._csr(keys[cav], n_rows)  # keys are sorted: rows in order
                idx[(rid, st, sr, True)] = len(arrays)
                cid = (self.lim[(rid, st, sr)] + 1).astype(np.uint32)
                arrays.append((off, nbr, cid, np.zeros(nbr.size, np.int64), n_rows))
        prog = corc.encode_program(self.W.ids, idx)
        return prog, corc.make_csr_table(arrays), np.concatenate([[0], self.limits]).astype(np.int64)
