"""GPU parity: the HIP engine (through the C ABI) against the reference's known answers, the
hand-derived SpiceDB-semantics fixtures and the Python oracle on seeded random graphs.
Bar: bit-exact tri-state (HAS / NO / CONDITIONAL) and per-item error codes."""
import json

import numpy as np
import pytest

from gochugaru_amd import consistency, rel
from gochugaru_amd import engine as E
from gochugaru_amd.client import Client, CheckItemError, OverlapKeyPanic, WithOverlapRequired
from oracle import spicedb_ref as ref
from tests import gen
from tests.helpers import (expected_code, iso_to_unix, load_golden, oracle_for, parse_check,
                           to_oracle_item)

pytestmark = pytest.mark.gpu

CLIENT = load_golden("client_check.json")
FOUNDERS = load_golden("readme_founders.json")
SEM = load_golden("semantics.json")
NOW_US = int(iso_to_unix(SEM["now"]) * 1e6)


def make_engine(schema, tuples, revision=1, **kw):
    e = E.Engine(**kw)
    e.load_schema(schema)
    e.load_snapshot_text(revision, "\n".join(tuples))
    return e


def device_results(e, checks, now_us=NOW_US, contexts=None):
    """Check strings through gck_check_bulk_ctx; contexts[i] is check i's caveat context."""
    items = e.make_items([parse_check(s) for s in checks])
    texts, slots = [], {}
    for i, ctx in enumerate(contexts or []):
        if ctx is None:
            continue
        js = json.dumps(ctx, sort_keys=True)
        if js not in slots:
            texts.append(js)
            slots[js] = len(texts)
        items[i]["context_slot"] = slots[js]
    perm, err = e.check_bulk(items, now_us=now_us, contexts=texts)
    return [(int(p), int(x)) for p, x in zip(perm, err)]


# ---- reference known answers (client/client_test.go:141-216, README.md:71-88) --------------

@pytest.fixture(scope="module")
def doc_client():
    e = make_engine(CLIENT["schema"], CLIENT["tuples"])
    yield Client(e)
    e.close()


@pytest.mark.parametrize("case", CLIENT["cases"], ids=lambda c: c["name"])
def test_client_check_known_answers(doc_client, case):
    cs = consistency.Full() if case["consistency"] == "full" else consistency.MinLatency()
    results, err = doc_client.Check(None, cs, *[parse_check(s) for s in case["checks"]])
    assert err is None
    assert results == case["expected"]


def test_check_one_any_all(doc_client):
    ok, err = doc_client.CheckOne(None, consistency.MinLatency(),
                                  rel.MustFromTriple("document:check_test1", "edit", "user:alice"))
    assert (ok, err) == (True, None)
    rs = [rel.MustFromTriple("document:check_test1", "edit", "user:bob"),
          rel.MustFromTriple("document:check_test1", "view", "user:bob")]
    assert doc_client.CheckAny(None, consistency.MinLatency(), *rs) == (True, None)
    assert doc_client.CheckAll(None, consistency.MinLatency(), *rs) == (False, None)
    assert doc_client.CheckAll(None, consistency.MinLatency()) == (True, None)  # vacuous
    assert doc_client.CheckAny(None, consistency.MinLatency()) == (False, None)


def test_check_iter_and_item_error(doc_client):
    rs = [rel.MustFromTriple("document:check_test1", "view", "user:bob")] * 2500
    out = list(doc_client.CheckIter(None, consistency.MinLatency(), iter(rs)))
    assert len(out) == 2500 and all(v == (True, None) for v in out)
    # the first per-item error stops the iteration (client/client.go:168-171)
    bad = rs[:3] + [rel.MustFromTriple("document:README", "owner", "user:bot")] + rs[:3]
    out = list(doc_client.CheckIter(None, consistency.MinLatency(), iter(bad), chunk=2))
    assert out[:2] == [(True, None), (True, None)]
    assert out[2][0] is False and isinstance(out[2][1], CheckItemError) and len(out) == 3
    # Check returns the prefix before the error (client/client.go:279-280)
    results, err = doc_client.Check(None, consistency.MinLatency(), *bad)
    assert results == [True, True, True] and isinstance(err, CheckItemError)


def test_overlap_required_panics():
    # client/client_test.go:218-277
    e = make_engine(CLIENT["schema"], CLIENT["tuples"])
    c, _ = Client.NewWithOpts(e, WithOverlapRequired())
    r = rel.MustFromTriple("document:README", "owner", "user:bot")
    with pytest.raises(OverlapKeyPanic):
        c.CheckOne(None, consistency.Full(), r)
    c.CheckOne(consistency.WithOverlapKey(None, "test"), consistency.Full(), r)  # no panic
    e.close()


def test_consistency_revisions():
    e = make_engine(CLIENT["schema"], CLIENT["tuples"], revision=7)
    c = Client(e)
    r = rel.MustFromTriple("document:check_test1", "edit", "user:alice")
    assert c.CheckOne(None, consistency.AtLeast("7"), r) == (True, None)
    assert c.CheckOne(None, consistency.Snapshot("7"), r) == (True, None)
    ctx = consistency.Context(metadata={})
    object.__setattr__(ctx, "deadline", 0)  # no retries
    ok, err = c.CheckOne(ctx, consistency.AtLeast("8"), r)
    assert ok is False and isinstance(err, E.GckError) and err.code == E.GCK_E_REVISION
    ok, err = c.CheckOne(ctx, consistency.Snapshot("6"), r)
    assert err is not None
    e.close()


def test_readme_founders():
    e = make_engine(FOUNDERS["schema"], FOUNDERS["tuples"])
    c = Client(e)
    founders = [rel.FromTriple("company:authzed", "founder", "user:" + f) for f in ("jake", "joey", "jimmy")]
    assert c.CheckAll(None, consistency.MinLatency(), *founders) == (True, None)
    e.close()
    e = make_engine(FOUNDERS["schema"], [t for t in FOUNDERS["tuples"] if t != FOUNDERS["negative_remove"]])
    assert Client(e).CheckAll(None, consistency.MinLatency(), *founders) == (False, None)
    e.close()


# ---- hand-derived SpiceDB semantics (tests/golden/semantics.json) ---------------------------

def _suite(name):
    return next(s for s in SEM["suites"] if s["name"] == name)


def test_semantics_rewrites():
    s = _suite("gdocs-arrows-exclusion-intersection-wildcard")
    e = make_engine(s["schema"], s["tuples"])
    got = device_results(e, [c[0] for c in s["checks"]])
    for (chk, label, note), g in zip(s["checks"], got):
        assert g == expected_code(label), (chk, note)
    e.close()


def test_semantics_depth():
    s = _suite("depth-budget")
    for chk, depth, label, note in s["depth_checks"]:
        e = make_engine(s["schema"], s["tuples"], max_depth=depth)
        assert device_results(e, [chk]) == [expected_code(label)], (chk, depth, note)
        e.close()


def test_semantics_caveats():
    """Hand-derived caveat cases with their check contexts: the host evaluates each caveat
    instance under each context (cel.cpp) and the device walk uses the outcomes."""
    s = _suite("caveats-and-expiration")
    e = make_engine(s["schema"], s["tuples"])
    rows = s["caveat_checks"]
    got = device_results(e, [c[0] for c in rows], contexts=[c[1] for c in rows])
    for c, g in zip(rows, got):
        assert g == expected_code(c[3]), c
    # one at a time (each call its own context table) gives the same answers
    for c in rows:
        assert device_results(e, [c[0]], contexts=[c[1]]) == [expected_code(c[3])], c
    e.close()


# ---- random graphs vs the oracle -------------------------------------------------------------

PATHS = {
    # closure-join stage, then the persistent wave-bundle kernel (default)
    "bundle": {},
    # grid-wide level-synchronous kernels only
    "wide": {"wide_only": True},
    # the bundle machinery on its own (no closure-join stage) ...
    "noclosure": {"closure": False, "labels": False},
    # tiny per-wave scratch: most bundles overflow and are re-run by the later stages
    "bundle-deferred": {"bundle_checks": 3, "bundle_frontier": 8, "bundle_visited": 8, "closure": False, "labels": False},
    # tiny work budget: almost every check is handed to a 16-wave workgroup bundle
    "giant": {"bundle_budget": 2, "closure": False, "labels": False},
    # ... and those overflow their workgroup scratch into the grid-wide path
    "giant-deferred": {"bundle_budget": 2, "giant_frontier": 8, "giant_visited": 16, "giant_slots": 3,
                       "closure": False, "labels": False},
    # deferred checks straight to the grid-wide path
    "giant-skip": {"bundle_budget": 2, "giant_stage": False, "closure": False, "labels": False},
    # what the closure-join stage leaves goes through the bundles' deferral chain
    "closure-giant": {"bundle_budget": 2},
    # the closure join's task rounds alone (no user / resource slots)
    "noslots": {"slots": False},
    # one check per wavefront, few resident waves
    "bundle-1": {"bundle_checks": 1, "bundle_waves_per_cu": 4, "closure": False, "labels": False},
    # binary-search membership instead of the hashed index, both paths
    "nohash": {"membership_hash": False, "labels": False},
    "nohash-wide": {"membership_hash": False, "wide_only": True},
    # forward-only wave bundles (no bidirectional checks, hence no closure join)
    "nobidir": {"bidir": False, "labels": False},
    # bidirectional checks always expanding only the smaller side (most carrying) ...
    "bidir-one": {"bidir_both": 1, "closure": False, "labels": False},
    # ... or always both sides; and bidirectional checks deferred to the later stages
    "bidir-all": {"bidir_both": 1 << 30, "closure": False, "labels": False},
    "bidir-deferred": {"bundle_budget": 6, "bundle_frontier": 16, "bundle_visited": 64, "closure": False, "labels": False},
    # the label join (labels.inc) for every root it takes, the nested-group ones included ...
    "labels": {"closure": False},
    # ... with its leftovers through the bundles' deferral chain
    "labels-deferred": {"closure": False, "bundle_budget": 2},
    # no label join: the default stage A of round 2 (closure join, then bundles)
    "nolabels": {"labels": False},
}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("family", sorted(gen.FAMILIES))
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_parity(family, seed, path):
    schema, tuples, checks = gen.FAMILIES[family](seed)
    contexts = gen.check_contexts(seed, len(checks))
    depth = gen.FAMILY_DEPTH.get(family, 50)
    ck = oracle_for(schema, tuples, max_depth=depth, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, contexts)]
    e = make_engine(schema, tuples, max_depth=depth, **PATHS[path])
    got = device_results(e, checks, now_us=gen.NOW_US, contexts=contexts)
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
    assert not bad, bad[:10]
    deep = family in ("cyclic", "near_budget")  # roots that may hit the budget take the exact path
    if path == "bundle-deferred" and family not in ("caveated", "hub_arrow"):  # (too small to overflow)
        assert e.stats()["deferred"] > 0
    if path == "bundle" and not deep:
        assert e.stats()["deferred"] == 0
    if path == "bundle" and family in ("nested", "gdocs_deep"):
        assert e.stats()["closure_checks"] > 0  # nested doc#view / group#member checks
    if path == "bundle" and family == "nested":
        assert e.stats()["slot_checks"] > 0  # doc#view@user decided from the slots
    if path == "noslots":
        assert e.stats()["slot_checks"] == 0
    if path == "labels" and family in ("nested", "gdocs", "github", "gdocs_deep"):
        assert e.stats()["slot_checks"] > 0  # decided by the label join's slots
        assert e.stats()["label_checks"] > 0
    if path == "noclosure" and family in ("nested", "gdocs_deep"):
        assert e.stats()["bidir_checks"] > 0 and e.stats()["closure_checks"] == 0
    if path in ("nobidir", "wide") or family == "caveated":
        assert e.stats()["bidir_checks"] == 0
    e.close()


@pytest.mark.parametrize("path", ["bundle", "wide"])
def test_semantics_all_paths(path):
    for s in SEM["suites"]:
        rows = s.get("checks") or s.get("caveat_checks")
        if not rows:
            continue
        e = make_engine(s["schema"], s["tuples"], **PATHS[path])
        ctxs = None if "checks" in s else [c[1] for c in rows]
        got = device_results(e, [c[0] for c in rows], contexts=ctxs)
        col = 1 if "checks" in s else 3
        assert got == [expected_code(c[col]) for c in rows], s["name"]
        e.close()


def test_small_batches_and_overflow_retry():
    schema, tuples, checks = gen.gdocs(11)
    ck = oracle_for(schema, tuples)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    # tiny workspace: forces batch splits and overflow retries, results must not change
    e = make_engine(schema, tuples, max_batch=37, frontier_capacity=64, segment_capacity=64,
                    visited_capacity=256, query_capacity=64, wide_only=True)
    got = device_results(e, checks, now_us=gen.NOW_US)
    assert got == want
    st = e.stats()
    assert st["batches"] >= len(checks) // 37
    e.close()
    # the same through bundles whose deferrals land in the tiny wide workspace
    e = make_engine(schema, tuples, max_batch=37, frontier_capacity=64, segment_capacity=64,
                    visited_capacity=256, query_capacity=64, bundle_checks=2, bundle_frontier=4,
                    bundle_visited=8)
    assert device_results(e, checks, now_us=gen.NOW_US) == want
    e.close()


def test_determinism_and_empty():
    schema, tuples, checks = gen.github(5)
    e = make_engine(schema, tuples)
    a = device_results(e, checks)
    b = device_results(e, checks)
    assert a == b
    perm, err = e.check_bulk(np.zeros(0, dtype=E.ITEM_DTYPE))
    assert len(perm) == 0 and len(err) == 0
    e.close()


def test_device_buffers_api():
    import torch
    schema, tuples, checks = gen.nested(4)
    e = make_engine(schema, tuples)
    items = e.make_items([parse_check(c) for c in checks])
    want_p, want_e = e.check_bulk(items, now_us=gen.NOW_US)
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    d_perm = torch.zeros(len(items), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(len(items), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e.check_bulk_device(d_items.data_ptr(), len(items), d_perm.data_ptr(), d_err.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream, now_us=gen.NOW_US)
    assert np.array_equal(d_perm.cpu().numpy(), want_p)
    assert np.array_equal(d_err.cpu().numpy(), want_e)
    e.close()


def test_device_buffers_api_with_contexts():
    """gck_check_bulk_device_ctx: device-resident items, host-side check contexts."""
    import torch
    schema, tuples, checks = gen.caveated(2)
    contexts = gen.check_contexts(2, len(checks))
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, contexts)]
    e = make_engine(schema, tuples)
    items = e.make_items([parse_check(c) for c in checks])
    texts = []
    for i, x in enumerate(contexts):
        if x is not None:
            texts.append(json.dumps(x))
            items[i]["context_slot"] = len(texts)
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    d_perm = torch.zeros(len(items), dtype=torch.uint8, device="cuda")
    d_err = torch.zeros(len(items), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e.check_bulk_device(d_items.data_ptr(), len(items), d_perm.data_ptr(), d_err.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream, now_us=gen.NOW_US, contexts=texts)
    got = [(int(p), int(x)) for p, x in zip(d_perm.cpu().numpy(), d_err.cpu().numpy())]
    assert got == want
    e.close()


def test_client_check_sends_caveat_context():
    """Client.Check passes rel.Relationship's caveat context as the check context
    (client/client.go:257); CONDITIONAL maps to false (client/client.go:274-277)."""
    s = _suite("caveats-and-expiration")
    e = make_engine(s["schema"], s["tuples"])
    c = Client(e)
    r = rel.MustFromTriple("doc:a", "viewer", "user:u1")
    ok, err = c.CheckOne(None, consistency.MinLatency(), r)
    assert err is None and ok is False  # CONDITIONAL
    ok, err = c.CheckOne(None, consistency.MinLatency(), r.WithCaveat("only_on_tuesday", {"day_of_the_week": "tuesday"}))
    assert err is None and ok is True
    res, err = c.Check(None, consistency.MinLatency(),
                       r.WithCaveat("only_on_tuesday", {"day_of_the_week": "monday"}),
                       r.WithCaveat("only_on_tuesday", {"day_of_the_week": "tuesday"}),
                       rel.MustFromTriple("doc:a", "view", "user:u2"))
    assert err is None and res == [False, True, True]
    e.close()


def test_device_api_is_ordered_after_callers_stream():
    """Regression: with stream=NULL (PyTorch's default stream) the check must run after work
    the caller queued there — here a long kernel followed by writes of the items and outputs."""
    import torch
    schema, tuples, checks = gen.nested(4)
    e = make_engine(schema, tuples)
    items = e.make_items([parse_check(c) for c in checks])
    want_p, want_e = e.check_bulk(items, now_us=gen.NOW_US)
    host_items = torch.from_numpy(items.view(np.uint8).copy())
    for _ in range(4):
        d_items = torch.zeros(host_items.numel(), dtype=torch.uint8, device="cuda")
        d_perm = torch.zeros(len(items), dtype=torch.uint8, device="cuda")
        d_err = torch.zeros(len(items), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)  # keep the default stream busy
        d_items.copy_(host_items.cuda(non_blocking=True))
        d_perm.fill_(7)
        d_err.fill_(-1)
        e.check_bulk_device(d_items.data_ptr(), len(items), d_perm.data_ptr(), d_err.data_ptr(),
                            stream=torch.cuda.current_stream().cuda_stream, now_us=gen.NOW_US)
        assert np.array_equal(d_perm.cpu().numpy(), want_p)
        assert np.array_equal(d_err.cpu().numpy(), want_e)
    e.close()
