"""Uniform requests and the evaluated revision on the GPU (include/gck.h ABI 13).

gck_check_bulk_uniform / gck_check_submit_uniform carry what Client.Check sends for relationships of
one shape (client/client.go:241-259) as one header and 8-B (resource id, subject id) pairs, and
answer with packed 2-bit Permissionships plus a sparse error list. Bar: for every shape of every
family, the packed results equal the oracle's Permissionship (0 for an errored check) and the error
list equals the oracle's errored checks, in order — on the zero-copy join path (pinned and pageable
buffers), on the expanded fallback (check contexts, profiling), across chunks above max_batch and
through the compiled submit/wait loop. gck_check_bulk_at / gck_check_wait_at report the revision a
batch ran on (CheckBulkPermissionsResponse.CheckedAt), also when a Watch batch publishes between
the submit and the wait."""
import json

import numpy as np
import pytest

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu
NOW_US = gen.NOW_US


def _engine(schema, tuples, revision=1, **kw):
    e = E.Engine(device=0, **kw)
    e.load_schema(schema)
    e.load_snapshot_text(revision, "\n".join(tuples))
    return e


def _shapes(items):
    """Groups of request positions with one (resource type, permission, subject type, subject
    relation): one uniform request each."""
    key = np.stack([items["resource_type"], items["permission"], items["subject_type"],
                    items["subject_relation"]], axis=1)
    groups = {}
    for i, k in enumerate(map(tuple, key)):
        groups.setdefault(k, []).append(i)
    return groups


def _expected(want, idx):
    perm = [w[0] if w[1] == 0 else 0 for w in (want[i] for i in idx)]
    errs = [(k, want[i][1]) for k, i in enumerate(idx) if want[i][1] != 0]
    return perm, errs


def _run_family(e, schema, tuples, checks, depth, pinned, contexts=None, ctx_slot=0):
    ck = oracle_for(schema, tuples, max_depth=depth, now=NOW_US / 1e6)
    ctx = contexts[ctx_slot - 1] if ctx_slot else None
    want = [ck.check(to_oracle_item(parse_check(c), ctx)) for c in checks]
    items = e.make_items([parse_check(c) for c in checks])
    n_shapes = 0
    for shape, idx in _shapes(items).items():
        pairs = np.stack([items["resource_id"][idx], items["subject_id"][idx]], axis=1).astype(np.uint32)
        n = len(idx)
        if pinned:
            p = e.host_array(2 * n, np.uint32)
            p[:] = pairs.reshape(-1)
            words = e.host_array((n + 31) // 32, np.uint64)
            words[:] = 0xFFFFFFFFFFFFFFFF  # poisoned: every word must be written
            pairs_arg = p.reshape(-1, 2)
        else:
            words = None
            pairs_arg = pairs
        out, errs, rev = e.check_uniform(tuple(int(x) for x in shape) + (ctx_slot,), pairs_arg, now_us=NOW_US,
                                         contexts=contexts, out_packed=words)
        assert rev == e.revision
        got = E.unpack_results(out, n).tolist()
        wp, we = _expected(want, idx)
        bad = [(checks[idx[k]], wp[k], got[k]) for k in range(n) if wp[k] != got[k]]
        assert not bad, bad[:5]
        assert [(int(r["index"]), int(r["code"])) for r in errs] == we
        n_shapes += 1
    return n_shapes


FAMS = ["gdocs", "github", "nested", "gdocs_deep", "cyclic", "near_budget", "caveated", "hub_arrow"]


@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
@pytest.mark.parametrize("family", FAMS)
def test_uniform_matches_oracle(family, pinned):
    """Every shape of a family's checks as one uniform request: bit-exact, errors (depth budget)
    listed in request order, deferred checks (bundles) patched into the words."""
    schema, tuples, checks = gen.FAMILIES[family](2)
    depth = gen.FAMILY_DEPTH.get(family, 50)
    e = _engine(schema, tuples, max_depth=depth)
    e.reset_stats()
    assert _run_family(e, schema, tuples, checks, depth, pinned) >= 2
    st = e.stats()
    if family in ("nested", "gdocs", "github"):  # the zero-copy join path ran (label or closure join)
        assert st["closure_checks"] > 0 and st["aql_batches"] > 0
    e.close()


@pytest.mark.parametrize("family", ["caveated", "cyclic"])
def test_uniform_with_a_check_context(family):
    """A header context slot (every pair's context): the expanded path, bit-exact against the
    oracle under that context (CONDITIONAL without it, HAS / NO with it)."""
    schema, tuples, checks = gen.FAMILIES[family](3)
    depth = gen.FAMILY_DEPTH.get(family, 50)
    e = _engine(schema, tuples, max_depth=depth)
    ctxs = [json.dumps({"day_of_the_week": "tuesday"}), json.dumps({"day_of_the_week": "monday"})]
    for slot in (0, 1, 2):
        _run_family(e, schema, tuples, checks, depth, pinned=False,
                    contexts=[json.loads(c) for c in ctxs], ctx_slot=slot)
    e.close()


def test_uniform_on_every_engine_path():
    """The uniform request on the engine's other paths: no AQL queues, no label join, no closure
    join, profiling (the expanded fallback), the level-synchronous path alone."""
    schema, tuples, checks = gen.gdocs(4)
    for kw in ({"labels": False}, {"closure": False, "labels": False}, {"wide_only": True}, {}):
        e = _engine(schema, tuples, **kw)
        _run_family(e, schema, tuples, checks, 50, pinned=True)
        e.set_profile(True)
        _run_family(e, schema, tuples, checks, 50, pinned=False)
        e.close()


def test_uniform_chunks_above_max_batch():
    """A request above max_batch runs in chunks of max_batch (rounded to 32 checks) over two
    workspaces; the words and the error indices are the request's."""
    schema, tuples, _ = gen.nested(5, n_users=400, n_groups=160, n_docs=200)
    rng = np.random.default_rng(3)
    checks = [f"doc:d{rng.integers(0, 205)}#view@user:u{rng.integers(0, 405)}" for _ in range(5000)]
    e = _engine(schema, tuples, max_batch=1000)
    assert _run_family(e, schema, tuples, checks, 50, pinned=True) == 1
    assert _run_family(e, schema, tuples, checks, 50, pinned=False) == 1
    e.close()


def test_uniform_compiled_loop():
    """gckd_run_uniform (the cgo caller's loop): 24 requests, 8 in flight, pinned buffers; every
    request's words equal the oracle's. (8 in flight from one thread needs 8 workspaces: a submit
    waits for a free one, include/gck.h gck_config.workspaces.)"""
    schema, tuples, _ = gen.gdocs(6)
    rng = np.random.default_rng(9)
    e = _engine(schema, tuples, workspaces=8)
    t_doc = e.type_id("doc")
    t_user = e.type_id("user")
    view = e.relation_id(t_doc, "view")
    n_docs, n_users = e.object_count(t_doc), e.object_count(t_user)
    ck = oracle_for(schema, tuples, now=NOW_US / 1e6)
    n, k = 1000, 24
    pairs = [e.host_array(2 * n, np.uint32) for _ in range(k)]
    packed = [e.host_array((n + 31) // 32, np.uint64) for _ in range(k)]
    errs = [e.host_array(n, E.ITEM_ERROR_DTYPE) for _ in range(k)]
    for p in pairs:
        p[0::2] = rng.integers(0, n_docs, n)
        p[1::2] = rng.integers(0, n_users, n)
    e.run_uniform_batches((t_doc, view, t_user, E.ELLIPSIS), [p.ctypes.data for p in pairs],
                          [w.ctypes.data for w in packed], [x.ctypes.data for x in errs], n, n, 8, now_us=NOW_US)
    for b in range(k):
        got = E.unpack_results(packed[b], n)
        for j in range(0, n, 37):
            r = e.object_name(t_doc, int(pairs[b][2 * j]))
            u = e.object_name(t_user, int(pairs[b][2 * j + 1]))
            want = ck.check(to_oracle_item(parse_check(f"doc:{r}#view@user:{u}")))
            assert (int(got[j]), 0) == tuple(want), (b, j, r, u)
    e.close()


def test_evaluated_revision_across_a_watch_publication():
    """A batch submitted at revision 1 reports 1 at its wait although a Watch batch moved the
    engine to 2 in between (the publication first finishes the batches in flight); the next check
    reports 2 and sees the update."""
    schema = gen.GDOCS
    _, tuples, _ = gen.gdocs(7)
    e = _engine(schema, tuples, revision=1)
    cands = [f"doc:d{d}#view@user:u{u}" for d in range(5) for u in range(40)]
    perm, _ = e.check_bulk(e.make_items([parse_check(c) for c in cands]), now_us=NOW_US)
    c = cands[int(np.flatnonzero(perm == E.PERM_NO)[0])]  # a pair without the permission at revision 1
    d, u = c.split("#")[0], c.split("@")[1]
    items = e.make_items([parse_check(c)])
    b = e.submit(items)
    e.apply_updates_text(2, f"CREATE {d}#viewer@{u}")
    perm, _ = b.wait()
    assert b.revision == 1 and int(perm[0]) == E.PERM_NO
    # (interned again: the subject may be a name revision 1 did not hold — ABSENT in the request
    # made then — which the update created; a caller interns each request's names)
    items = e.make_items([parse_check(c)])
    perm, err, rev = e.check_bulk_at(items)
    assert rev == 2 and int(perm[0]) == E.PERM_HAS
    t_doc, t_user = e.type_id("doc"), e.type_id("user")
    hdr = (t_doc, e.relation_id(t_doc, "view"), t_user, E.ELLIPSIS)
    pairs = np.array([[items["resource_id"][0], items["subject_id"][0]]], dtype=np.uint32)
    ub = e.submit_uniform(hdr, pairs, np.zeros(1, dtype=np.uint64), np.zeros(1, dtype=E.ITEM_ERROR_DTYPE))
    e.apply_updates_text(3, f"DELETE {d}#viewer@{u}")
    words, errs, rev = ub.wait()
    assert rev == 2 and E.unpack_results(words, 1).tolist() == [E.PERM_HAS] and len(errs) == 0
    words, errs, rev = e.check_uniform(hdr, pairs)
    assert rev == 3 and E.unpack_results(words, 1).tolist() == [E.PERM_NO]
    e.close()
