"""BASELINE.json config 5 at reduced scale: caveated tuples (10 % of the folder / doc viewer and
editor user tuples ``with only_on_tuesday``), check-time contexts (tuesday / monday / none) and
Watch churn at a moving revision (CREATE / TOUCH / DELETE, TOUCH toggling the caveat). After
every update batch the engine's answers are compared bit-exactly with the C oracle over the
rebuilt snapshot (tests/synth_configs.py Mixed.expected)."""
import numpy as np
import pytest
import torch

from gochugaru_amd.engine import Engine
from oracle import corc
from tests import synth_configs as S

pytestmark = pytest.mark.gpu


def load(M, **kw):
    e = Engine(device=0, **kw)
    e.load_schema(M.W.schema)
    for t, n in M.W.counts.items():
        e.reserve_objects(M.W.t(t), n)
    e.begin_snapshot(1)
    cav = e.add_caveat_instance("only_on_tuesday", "")
    keep = []

    def loader(rid, st, sr, n_rows, off, nbr):
        off32 = off.to(torch.int32).contiguous()
        nbr32 = nbr.contiguous()
        keep.append((off32, nbr32))
        e.load_csr(rid, st, sr, n_rows, off32.data_ptr(), nbr32.data_ptr(), nbr32.numel(), device=True)

    M.load(e, loader, cav)
    torch.cuda.synchronize()
    e.commit_snapshot()
    return e, cav


def run(e, items):
    n = items.shape[0]
    perm = torch.zeros(n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(n, dtype=torch.int32, device="cuda")
    e.check_bulk_device(items.data_ptr(), n, perm.data_ptr(), err.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream, contexts=S.CONTEXTS)
    return perm.cpu().numpy(), err.cpu().numpy()


@pytest.mark.parametrize("path", ["bundle", "wide"])
def test_mixed_caveats_and_churn(path):
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M, **({"wide_only": True} if path == "wide" else {}))
    items = M.checks(16384, seed=9)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    n_tuples = M.W.n_tuples
    seen = {1: 0, 2: 0, 3: 0}
    for step in range(4):
        if step:
            ups = M.churn(n_tuples // 100, cav)
            e.apply_updates(1 + step, ups)
            assert e.revision == 1 + step
        gp, ge = run(e, items)
        cp, ce = M.expected(hi)
        bad = np.nonzero((gp != cp) | (ge != ce))[0]
        assert len(bad) == 0, (step, [(int(i), int(hi[i]["context_slot"]), int(gp[i]), int(cp[i])) for i in bad[:6]])
        for k in seen:
            seen[k] += int((gp == k).sum())
    assert all(v > 0 for v in seen.values()), seen  # NO, HAS and CONDITIONAL all occur
    e.close()


def test_label_tables_hold_under_a_long_watch_stream():
    """BASELINE config 5's Watch stream (client/client.go:370-413 is unbounded) at reduced scale:
    200 batches of 0.1 % of the tuples each (CREATE / TOUCH / DELETE of folder and document
    viewers and editors, TOUCH toggling the caveat). The label tables are kept throughout: a
    subject whose grants changed is still answered by the join unless a changed object is the
    resource or one of its folders (labels.inc round 2, the arrow forest). Bit-exact against the
    C oracle after 1, 50 and 200 batches, with at least 95 % of the checks through the join at
    the end."""
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M)
    n = 16384
    items = M.checks(n, seed=12)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    frac = {}
    for step in range(1, 201):
        e.apply_updates(1 + step, M.churn(max(1, M.W.n_tuples // 1000), cav))
        if step in (1, 50, 200):
            e.reset_stats()
            gp, ge = run(e, items)
            st = e.stats()
            cp, ce = M.expected(hi)
            bad = np.nonzero((gp != cp) | (ge != ce))[0]
            assert len(bad) == 0, (step, [(int(i), int(gp[i]), int(cp[i])) for i in bad[:6]])
            frac[step] = st["label_checks"] / n
    print("label-join share after 1 / 50 / 200 batches:", frac)
    assert frac[200] >= 0.95, frac
    e.close()


def _parents(M):
    """doc -> its folder, folder -> its parent folder (-1: none), and folder -> its documents."""
    W = M.W
    out = {}
    for t in ("doc", "folder"):
        _, _, _, n, off, nbr = W.find(t, "parent", "folder")
        off, nbr = off.cpu().numpy(), nbr.cpu().numpy().astype(np.int64)
        par = np.full(n, -1, np.int64)
        has = off[1:] > off[:-1]
        par[has] = nbr[off[:-1][has]]
        out[t] = par
    order = np.argsort(out["doc"], kind="stable")
    docs_of = {}
    for d in order:
        f = int(out["doc"][d])
        if f >= 0:
            docs_of.setdefault(f, []).append(int(d))
    return out, docs_of


def _aimed_checks(M, ups, parents, docs_of, rng):
    """Checks at the grants a Watch batch changed: every one is an overlay hit of a dirty subject
    (the changed object is the resource or one of its ancestors)."""
    W = M.W
    t = ups["tuple"]
    doc_t, folder_t = W.t("doc"), W.t("folder")
    rows = []
    for rt, rid, sid in zip(t["resource_type"], t["resource_id"], t["subject_id"]):
        if int(sid) == S.WILD:
            continue
        if rt == doc_t:
            rows.append(("doc", int(rid), int(sid)))
        else:
            rows.append(("folder", int(rid), int(sid)))
            # a document under the folder or under one of its descendants' chain: the folder's own
            ds = docs_of.get(int(rid))
            if ds:
                rows.append(("doc", ds[int(rng.integers(0, len(ds)))], int(sid)))
    n = len(rows)
    items = np.zeros((n, 5), np.int64)
    for k, (typ, rid, sid) in enumerate(rows):
        perm = ("view", "edit")[int(rng.integers(0, 2))]
        items[k] = [W.t(typ) | (W.r(typ, perm) << 16), rid, W.t("user") | (S.ELLIPSIS << 16), sid,
                    int(rng.integers(0, 3))]
    items = items - ((items >= 2 ** 31).astype(np.int64) << 32)
    return torch.from_numpy(items.astype(np.int32)).view(torch.uint8).reshape(n, 20).cuda()


def test_overlay_hits_decided_by_the_chain_walk():
    """A dirty subject's check whose changed grant lies on the resource's own chain (the document,
    its folder, the folder's ancestors: an overlay hit) is decided in the label join from the
    current revision's rows (labels.inc lj_chain_walk, round 3) instead of the wave bundles. Every
    check here is aimed at a grant the last Watch batch changed (CREATE / TOUCH / DELETE, caveat
    toggles, with tuesday / monday / no context): bit-exact against the C oracle after each of 12
    batches, and every check through the join (no deferral)."""
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M)
    rng = np.random.default_rng(5)
    parents, docs_of = _parents(M)
    total = 0
    for step in range(1, 13):
        ups = M.churn(max(1, M.W.n_tuples // 1000), cav)
        e.apply_updates(1 + step, ups)
        items = _aimed_checks(M, ups, parents, docs_of, rng)
        n = items.shape[0]
        plain = step % 3 == 0  # (every third batch without check contexts: the kernels without the caveat plane)
        if plain:
            items.view(torch.int32).reshape(n, 5)[:, 4] = 0
        hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
        e.reset_stats()
        if plain:
            gp = torch.zeros(n, dtype=torch.uint8, device="cuda")
            ge = torch.zeros(n, dtype=torch.int32, device="cuda")
            e.check_bulk_device(items.data_ptr(), n, gp.data_ptr(), ge.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream)
            gp, ge = gp.cpu().numpy(), ge.cpu().numpy()
        else:
            gp, ge = run(e, items)
        st = e.stats()
        cp, ce = M.expected(hi)
        bad = np.nonzero((gp != cp) | (ge != ce))[0]
        assert len(bad) == 0, (step, [(int(i), hi[i], int(gp[i]), int(cp[i]), int(ge[i]), int(ce[i])) for i in bad[:6]])
        assert st["label_checks"] == n, (step, st["label_checks"], n)
        total += n
    assert total > 1000, total
    e.close()


def _wild_checks(M, ups, rng, per=8):
    """Checks of the documents whose wildcard grant (doc#viewer@user:*) a Watch batch touched or
    deleted, each against `per` random users, view and edit, with a random context slot."""
    W = M.W
    t = ups["tuple"]
    docs = np.unique(t["resource_id"][(t["subject_id"] == S.WILD) & (t["resource_type"] == W.t("doc"))])
    n = len(docs) * per
    items = np.zeros((n, 5), np.int64)
    for k in range(n):
        perm = ("view", "edit")[int(rng.integers(0, 2))]
        items[k] = [W.t("doc") | (W.r("doc", perm) << 16), int(docs[k // per]), W.t("user") | (S.ELLIPSIS << 16),
                    int(rng.integers(0, W.counts["user"])), int(rng.integers(0, 3))]
    items = items - ((items >= 2 ** 31).astype(np.int64) << 32)
    return len(docs), torch.from_numpy(items.astype(np.int32)).view(torch.uint8).reshape(n, 20).cuda()


def test_wildcard_grant_changes_decided_by_the_walk():
    """A Watch batch that touches or deletes a document's wildcard grant keeps the label tables: the
    document's slot is marked (kLjHdrWildDirty) rather than deferred, and its checks are decided in
    the join from the slot without its wildcard entries, joined with a walk of the current rows for
    the subject and for the wildcard (labels.inc lj_chain_wave, round 3). Bit-exact against the C
    oracle after each of 16 batches, every check through the join, also for a subject that is dirty
    itself."""
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M)
    rng = np.random.default_rng(8)
    n_docs = 0
    for step in range(1, 17):
        ups = M.churn(max(1, M.W.n_tuples // 100), cav)
        e.apply_updates(1 + step, ups)
        nd, items = _wild_checks(M, ups, rng)
        if nd == 0:
            continue
        n_docs += nd
        n = items.shape[0]
        hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
        e.reset_stats()
        gp, ge = run(e, items)
        st = e.stats()
        cp, ce = M.expected(hi)
        bad = np.nonzero((gp != cp) | (ge != ce))[0]
        assert len(bad) == 0, (step, [(int(i), hi[i], int(gp[i]), int(cp[i])) for i in bad[:6]])
        assert st["label_checks"] == n, (step, st["label_checks"], n)
    assert n_docs >= 10, n_docs
    e.close()


def test_label_tables_hold_over_2000_batches():
    """The Watch stream of config 5 over 2,000 batches (0.1 % of the tuples each: at this scale
    every user's grants have changed several times, so nearly every subject is dirty and most
    overlays have overflowed): the tables are never rebuilt, and the chain walk keeps the checks in
    the join — bit-exact against the C oracle after 2,000 batches with at least 99 % of the checks
    through the join."""
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M)
    n = 16384
    items = M.checks(n, seed=21)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    frac = {}
    for step in range(1, 2001):
        e.apply_updates(1 + step, M.churn(max(1, M.W.n_tuples // 1000), cav))
        if step in (1, 2000):
            e.reset_stats()
            gp, ge = run(e, items)
            st = e.stats()
            cp, ce = M.expected(hi)
            bad = np.nonzero((gp != cp) | (ge != ce))[0]
            assert len(bad) == 0, (step, [(int(i), int(gp[i]), int(cp[i])) for i in bad[:6]])
            frac[step] = st["label_checks"] / n
    print("label-join share after 1 / 2000 batches:", frac)
    assert frac[2000] >= 0.99, frac
    e.close()
