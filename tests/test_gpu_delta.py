"""GPU parity of Watch-driven incremental updates: a snapshot kept
current with ``gck_apply_updates`` — the device-side CSR merge of delta.inc — answers exactly
what a snapshot built from scratch out of the same relationships answers (the Python oracle
over the updated tuple set), on every engine path.

Update semantics follow rel.Update (rel/relationship.go:267-301) as a Watch stream carries
them (client/client.go:370-413): CREATE and TOUCH upsert (a relationship is identified by
resource, relation and subject; its caveat and expiration are replaced), DELETE removes, and
within one batch the last write of a relationship wins."""
import random

import numpy as np
import pytest

from gochugaru_amd import consistency, rel
from gochugaru_amd import engine as E
from gochugaru_amd.client import Client
from oracle import spicedb_ref as ref
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu

PATHS = {
    "bundle": {},
    "wide": {"wide_only": True},
    "nobidir": {"bidir": False},
    "nohash": {"membership_hash": False},
}
FUTURE, PAST = "2999-01-01T00:00:00Z", "2020-01-01T00:00:00Z"


def rel_key(line):
    t = ref.parse_tuple(line)
    return (t.resource_type, t.resource_id, t.relation, t.subject_type, t.subject_id, t.subject_relation)


def strip_trailers(line):
    return line.split("[", 1)[0]


def apply_to_store(store, ups):
    for op, line in ups:
        k = rel_key(line)
        if op == "DELETE":
            store.pop(k, None)
        else:
            store[k] = line


def random_batch(rng, family, store, round_no, size=40):
    """A mixed batch: deletes of live relationships, creates from a differently seeded graph of
    the same family, relationships on objects the snapshot has never seen, re-writes of the same
    relationship inside the batch, and (caveated family) caveat / expiration toggles."""
    live = sorted(store.values())
    _, pool, _ = gen.FAMILIES[family](1000 + 17 * round_no + rng.randrange(1000))
    ups = []
    for _ in range(size):
        x = rng.random()
        if x < 0.3 and live:
            ups.append(("DELETE", rng.choice(live)))
        elif x < 0.6:
            ups.append((rng.choice(["CREATE", "TOUCH"]), rng.choice(pool)))
        elif x < 0.7:
            line = rng.choice(pool)  # a brand-new resource object
            res, rest = line.split("#", 1)
            ups.append(("CREATE", f"{res}_n{round_no}#{rest}"))
        elif x < 0.8 and live:
            line = rng.choice(live)  # written twice: the last write wins
            ups.append(("DELETE", line))
            if rng.random() < 0.5:
                ups.append(("TOUCH", line))
        elif family == "caveated" and live:
            cands = [l for l in live if l.startswith("doc:") and "#viewer@user:" in l]
            if cands:
                base = strip_trailers(rng.choice(cands))
                trailer = rng.choice(["", "[only_on_tuesday]", f"[expiration:{FUTURE}]", f"[expiration:{PAST}]",
                                      '[only_on_tuesday:{"day_of_the_week":"tuesday"}]'])
                ups.append(("TOUCH", base + trailer))
        elif live:
            ups.append(("TOUCH", rng.choice(live)))
    return ups


def checks_for(family, seed, store, ups):
    _, _, checks = gen.FAMILIES[family](seed)
    extra = []
    for op, line in ups:  # every written relationship, checked as its relation
        extra.append(strip_trailers(line))
    return checks + extra


def engine_results(e, checks):
    items = e.make_items([parse_check(c) for c in checks])
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    return [(int(p), int(x)) for p, x in zip(perm, err)]


def oracle_results(schema, store, checks):
    ck = oracle_for(schema, list(store.values()), now=gen.NOW_US / 1e6)
    return [ck.check(to_oracle_item(parse_check(c))) for c in checks]


@pytest.mark.parametrize("path", sorted(PATHS))
# gdocs_deep is left out: unions of its long chains from several seeds give re-converging paths
# that straddle the depth budget, where SpiceDB's own answer depends on traversal order
# 
@pytest.mark.parametrize("family", ["caveated", "gdocs", "github", "nested"])
@pytest.mark.parametrize("seed", [1, 2])
def test_updates_match_rebuilt_snapshot(family, seed, path):
    schema, tuples, _ = gen.FAMILIES[family](seed)
    rng = random.Random(seed * 7919 + len(path))
    e = E.Engine(**PATHS[path])
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    for rnd in range(4):
        ups = random_batch(rng, family, store, rnd)
        e.apply_updates_text(2 + rnd, "\n".join(f"{op} {line}" for op, line in ups))
        apply_to_store(store, ups)
        assert e.revision == 2 + rnd
        assert e.tuple_count == len(store), rnd
        checks = checks_for(family, seed, store, ups)
        want = oracle_results(schema, store, checks)
        got = engine_results(e, checks)
        bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
        assert not bad, (rnd, bad[:10])
    e.close()


def test_client_apply_updates_and_consistency():
    schema = "definition user {}\ndefinition company { relation founder: user }"
    e = E.Engine()
    c = Client(e)
    c.LoadSnapshot(schema, 3, [rel.MustFromTriple("company:authzed", "founder", "user:" + u)
                               for u in ("jake", "joey")])
    founders = [rel.MustFromTriple("company:authzed", "founder", "user:" + u) for u in ("jake", "joey", "jimmy")]
    assert c.CheckAll(None, consistency.MinLatency(), *founders) == (False, None)
    c.ApplyUpdates(4, [rel.Update(rel.UpdateCreate, founders[2])])
    assert c.CheckAll(None, consistency.AtLeast("4"), *founders) == (True, None)
    assert c.CheckOne(None, consistency.Snapshot("4"), founders[2]) == (True, None)
    ctx = consistency.Context(metadata={})
    object.__setattr__(ctx, "deadline", 0)  # no retries
    ok, err = c.CheckOne(ctx, consistency.Snapshot("3"), founders[2])  # the old revision is gone
    assert isinstance(err, E.GckError) and err.code == E.GCK_E_REVISION_GONE
    c.ApplyUpdates(5, [rel.Update(rel.UpdateDelete, founders[0])])
    assert c.Check(None, consistency.Full(), *founders) == ([False, True, True], None)
    # stale revision, unknown update type, rejected relationship: nothing is applied
    with pytest.raises(E.GckError) as ei:
        c.ApplyUpdates(5, [rel.Update(rel.UpdateCreate, founders[0])])
    assert ei.value.code == E.GCK_E_REVISION
    with pytest.raises(Exception):
        c.ApplyUpdates(6, [rel.Update(rel.UpdateUnknown, founders[0])])
    with pytest.raises(E.GckError) as ei:
        e.apply_updates_text(6, "CREATE company:authzed#founder@user:jake\nCREATE company:authzed#nosuch@user:x")
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    with pytest.raises(E.GckError):
        e.apply_updates_text(6, "UPSERT company:authzed#founder@user:jake")
    # a rejected batch leaves no interned ids behind (a new user and company in its valid lines)
    user, company = e.type_id("user"), e.type_id("company")
    n_users, n_companies = e.object_count(user), e.object_count(company)
    with pytest.raises(E.GckError):
        e.apply_updates_text(6, "CREATE company:newco#founder@user:newbie\nCREATE company:newco#nosuch@user:x")
    with pytest.raises(E.GckError) as ei:  # stale: refused before the text is read
        e.apply_updates_text(5, "CREATE company:other#founder@user:someone")
    assert ei.value.code == E.GCK_E_REVISION
    assert (e.object_count(user), e.object_count(company)) == (n_users, n_companies)
    assert e.intern(user, ["newbie", "someone"]).tolist() == [E.ID_ABSENT, E.ID_ABSENT]
    assert e.revision == 5
    assert c.Check(None, consistency.Full(), *founders) == ([False, True, True], None)
    # an empty batch may advance the revision (a Watch checkpoint)
    c.ApplyUpdates(9, [])
    assert e.revision == 9
    e.close()


def test_binary_updates_and_index_rebuild():
    """Interned updates (gck_update records); repeated delete / re-insert rounds fill the
    membership index with tombstones until it is rebuilt — results stay exact throughout."""
    schema, tuples, checks = gen.nested(3)
    e = E.Engine()
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    user, group = e.type_id("user"), e.type_id("group")
    member = e.relation_id(group, "member")
    direct = [l for l in tuples if "@user:" in l]
    bytes0 = e.device_bytes
    rng = random.Random(5)
    for rnd in range(12):
        picked = rng.sample(direct, 120)
        ops = [("DELETE", l) for l in picked] + [("CREATE", l) for l in picked[: 60]]
        ups = np.zeros(len(ops), dtype=E.UPDATE_DTYPE)
        for i, (op, line) in enumerate(ops):
            t = ref.parse_tuple(line)
            ups[i]["op"] = E.UPDATE_DELETE if op == "DELETE" else E.UPDATE_CREATE
            tt = ups[i]["tuple"]
            tt["resource_type"], tt["relation"] = group, member
            tt["resource_id"] = e.intern(group, [t.resource_id])[0]
            tt["subject_type"], tt["subject_relation"] = user, E.ELLIPSIS
            tt["subject_id"] = e.intern(user, [t.subject_id])[0]
            ups[i]["tuple"] = tt
        e.apply_updates(2 + rnd, ups)
        apply_to_store(store, ops)
        direct = [l for l in store.values() if "@user:" in l] + picked[60:]
        got = engine_results(e, checks)
        assert got == oracle_results(schema, store, checks), rnd
    assert e.tuple_count == len(store)
    assert e.device_bytes < 3 * bytes0  # merged arrays replace the old ones (no leak)
    e.close()


def test_skewed_batch_on_one_object():
    """A batch whose updates crowd onto a few objects (hundreds of subjects of one group, writes of
    the same relationship repeated inside the batch): the grouping's bucketed sort keeps every key
    in order and the last write of each relationship (snapshot.cpp group_updates)."""
    schema, tuples, checks = gen.nested(3)
    e = E.Engine()
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    rng = random.Random(11)
    for rnd in range(3):
        ups = []
        for k in rng.sample(range(200), 150):  # one object, many subjects (users u0..u199)
            ups.append(("CREATE", f"group:g{rnd}#member@user:u{k}"))
        tail = [("DELETE", f"group:g{rnd}#member@user:u{k}") for k in rng.sample(range(200), 100)]
        tail += [("TOUCH", f"group:g{rnd}#member@user:u{k}") for k in rng.sample(range(200), 60)]  # third writes
        tail += [(rng.choice(["CREATE", "DELETE"]), f"group:g{rnd + 10}#member@user:u{rng.randrange(200)}")
                 for _ in range(40)]  # a second object interleaved
        rng.shuffle(tail)
        ups += tail
        e.apply_updates_text(2 + rnd, "\n".join(f"{op} {line}" for op, line in ups))
        apply_to_store(store, ups)
        probe = checks + [f"group:g{rnd}#member@user:u{k}" for k in range(200)] + \
            [f"group:g{rnd + 10}#member@user:u{k}" for k in range(200)]
        assert engine_results(e, probe) == oracle_results(schema, store, probe), rnd
    # a batch large enough for the grouping's resident workers (>= 4096 updates, several groups)
    ups = [(rng.choice(["CREATE", "DELETE", "TOUCH"]), f"group:g{rng.randrange(120)}#member@user:u{rng.randrange(200)}")
           for _ in range(5000)]
    ups += [(rng.choice(["CREATE", "DELETE"]), f"doc:d{rng.randrange(80)}#viewer@group:g{rng.randrange(30)}#member")
            for _ in range(600)]
    e.apply_updates_text(9, "\n".join(f"{op} {line}" for op, line in ups))
    apply_to_store(store, ups)
    got, want = engine_results(e, checks), oracle_results(schema, store, checks)
    bad = [i for i in range(len(checks)) if got[i] != want[i]]
    if bad:  # (what a fresh engine over the same relationships answers, for the report)
        f = E.Engine()
        f.load_schema(schema)
        f.load_snapshot_text(9, "\n".join(store.values()))
        fresh = engine_results(f, [checks[i] for i in bad])
        f.close()
        again = engine_results(e, checks)
        pytest.fail("after the large batch: " + "; ".join(
            f"{checks[i]} got {got[i]} want {want[i]} fresh {fresh[k]} again {again[i]}" for k, i in enumerate(bad[:8]))
            + f" ({len(bad)} of {len(checks)}; stats {e.stats()})")
    assert e.tuple_count == len(store)
    e.close()


def _records(e, ops):
    """(op, tuple line) -> gck_update records (new object names interned first)."""
    ups = np.zeros(len(ops), dtype=E.UPDATE_DTYPE)
    for i, (op, line) in enumerate(ops):
        t = ref.parse_tuple(line)
        rt, st = e.type_id(t.resource_type), e.type_id(t.subject_type)
        ups[i]["op"] = {"CREATE": E.UPDATE_CREATE, "TOUCH": E.UPDATE_TOUCH, "DELETE": E.UPDATE_DELETE}[op]
        tt = ups[i]["tuple"]
        tt["resource_type"], tt["relation"] = rt, e.relation_id(rt, t.relation)
        tt["resource_id"] = e.intern(rt, [t.resource_id], create=True)[0]
        tt["subject_type"] = st
        srel = t.subject_relation
        tt["subject_relation"] = e.relation_id(st, srel) if srel and srel != "..." else E.ELLIPSIS
        tt["subject_id"] = e.intern(st, [t.subject_id], create=True)[0]
        ups[i]["tuple"] = tt
    return ups


@pytest.mark.parametrize("family", ["nested", "gdocs"])
def test_staged_watch_batches(family):
    """Pipelined Watch (gck_watch_stage / gck_watch_apply_staged): each batch is staged while the
    previous one applies, two ahead at times; results after every batch equal the oracle's on the
    same store. A staged batch the staging rejects fails at its apply (nothing applied, the
    revision stays); a discarded ticket is gone."""
    schema, tuples, _ = gen.FAMILIES[family](4)
    rng = random.Random(23)
    e = E.Engine()
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    # batches over names the snapshot already holds (interned before staging)
    plan = []
    for rnd in range(6):
        ups = [(op, l) for op, l in random_batch(rng, family, dict(store), rnd) if "_n" not in l.split("#")[0]]
        plan.append(ups)
    recs = [None] * len(plan)
    recs[0] = _records(e, plan[0])
    tickets = [e.stage_updates(recs[0])]
    rev = 1
    for k, ups in enumerate(plan):
        if k + 1 < len(plan):
            recs[k + 1] = _records(e, plan[k + 1])
            tickets.append(e.stage_updates(recs[k + 1]))
        rev += 1
        e.apply_staged(rev, tickets[k])
        apply_to_store(store, ups)
        assert e.revision == rev and e.tuple_count == len(store), k
        checks = checks_for(family, 4, store, ups)
        assert engine_results(e, checks) == oracle_results(schema, store, checks), k
    # a rejected staged batch: an unknown operation
    bad = _records(e, plan[0][:3])
    bad[1]["op"] = 77
    t = e.stage_updates(bad)
    with pytest.raises(E.GckError) as ei:
        e.apply_staged(rev + 1, t)
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT and e.revision == rev
    # staged, then discarded: never applied
    t = e.stage_updates(_records(e, plan[1]))
    e.discard_staged(t)
    with pytest.raises(E.GckError):
        e.apply_staged(rev + 1, t)
    assert e.revision == rev
    e.close()


def test_staging_slots_and_tickets():
    """Up to four batches staged at once; a ticket is applied once; the staging thread ends with
    the engine."""
    schema, tuples, _ = gen.nested(2)
    e = E.Engine()
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    line = [l for l in tuples if "@user:" in l][0]
    recs = _records(e, [("TOUCH", line)])
    ts = [e.stage_updates(recs) for _ in range(4)]
    with pytest.raises(E.GckError) as ei:
        e.stage_updates(recs)
    assert ei.value.code == E.GCK_E_CAPACITY
    for i, t in enumerate(ts):
        e.apply_staged(2 + i, t)
    with pytest.raises(E.GckError) as ei:
        e.apply_staged(9, ts[0])
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    assert e.revision == 5
    e.close()
