"""LookupResources / LookupSubjects (client/client.go:501-599) on the GPU: the reference's known
answers (client/client_test.go:107-139, tests/golden/lookup_resources.json) through the client
mirror, and every candidate of seeded random graphs against the oracle's checks."""
import numpy as np
import pytest

from gochugaru_amd import consistency
from gochugaru_amd import engine as E
from gochugaru_amd.client import Client
from tests import gen
from tests.helpers import load_golden, oracle_for
from tests.lookup_cases import WILD_CASES, WILD_SCHEMA
from oracle import spicedb_ref as ref

pytestmark = pytest.mark.gpu

LOOKUP = load_golden("lookup_resources.json")


def make_engine(schema, tuples, **kw):
    e = E.Engine(device=0, **kw)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    return e


@pytest.mark.parametrize("case", LOOKUP["cases"], ids=lambda c: c["name"])
def test_reference_lookup_resources(case):
    e = make_engine(LOOKUP["schema"], LOOKUP["tuples"])
    c = Client(e)
    ids = []
    for oid, err in c.LookupResources(None, consistency.Full(), case["permission"], case["subject"]):
        assert err is None
        ids.append(oid)
    assert sorted(ids) == case["expected"]
    e.close()


def test_lookup_errors_and_subjects():
    e = make_engine(LOOKUP["schema"], LOOKUP["tuples"])
    c = Client(e)
    out = list(c.LookupResources(None, consistency.MinLatency(), "document#nosuch", "user:alice"))
    assert len(out) == 1 and out[0][0] == "" and out[0][1] is not None
    out = list(c.LookupResources(None, consistency.MinLatency(), "documentwriter", "user:alice"))
    assert out[0][1] is not None  # ErrInvalidTypedRelationString
    subs = sorted(s for s, err in c.LookupSubjects(None, consistency.MinLatency(), "document:check_test1", "view", "user"))
    assert subs == ["alice", "bob", "charlie"]
    subs = sorted(s for s, err in c.LookupSubjects(None, consistency.MinLatency(), "document:check_test2", "edit", "user"))
    assert subs == ["charlie"]
    assert list(c.LookupResources(None, consistency.MinLatency(), "document#view", "user:nobody")) == []
    e.close()


def _oracle_lookup(ck, e, typ, fixed, vary_resource):
    tid = e.type_id(typ)
    out = []
    for i in range(e.object_count(tid)):
        name = e.object_name(tid, i)
        it = fixed(name)
        p, err = ck.check(it)
        assert err == 0, (it, err)
        if p in (ref.HAS, ref.COND):
            out.append((i, p))
    return out


@pytest.mark.parametrize("family,seed", [("gdocs", 1), ("github", 2), ("nested", 3), ("caveated", 4)])
@pytest.mark.parametrize("path", ["bundle", "wide"])
def test_lookup_parity(family, seed, path):
    schema, tuples, checks = gen.FAMILIES[family](seed)
    e = make_engine(schema, tuples, **({"wide_only": True} if path == "wide" else {}))
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    rng = np.random.default_rng(seed)
    for c in rng.choice(checks, size=4, replace=False):
        res, subj = c.split("@")
        rtype, rest = res.split(":", 1)
        _, perm = rest.split("#", 1)
        stype, sid = subj.split(":", 1)
        want = _oracle_lookup(ck, e, rtype, lambda n: ref.Item(rtype, n, perm, stype, sid), True)
        ids, perms = e.lookup_resources(e.type_id(rtype), e.relation_id(e.type_id(rtype), perm), e.type_id(stype),
                                        E.ELLIPSIS, int(e.intern(e.type_id(stype), [sid])[0]), now_us=gen.NOW_US)
        assert list(zip(ids.tolist(), perms.tolist())) == want, c
        rid = rest.split("#", 1)[0]
        want = ck.lookup_subjects(rtype, rid, perm, stype)
        ids, perms = e.lookup_subjects(e.type_id(rtype), int(e.intern(e.type_id(rtype), [rid])[0]),
                                       e.relation_id(e.type_id(rtype), perm), e.type_id(stype), now_us=gen.NOW_US)
        got = [("*" if i == E.ID_WILDCARD else e.object_name(e.type_id(stype), i), p)
               for i, p in zip(ids.tolist(), perms.tolist())]
        assert sorted(got) == sorted(want), c
        # every subject the candidate sweep finds is reported, or folded into "*"
        sweep = _oracle_lookup(ck, e, stype, lambda n: ref.Item(rtype, rid, perm, stype, n), False)
        named = {n for n, _ in got}
        assert all(e.object_name(e.type_id(stype), i) in named or "*" in named for i, _ in sweep), c
    e.close()


@pytest.mark.parametrize("case", range(len(WILD_CASES)))
@pytest.mark.parametrize("path", ["bundle", "wide"])
def test_lookup_subjects_wildcard(case, path):
    """LookupSubjects reports a wildcard grant as the subject "*" (client/client.go:560-599 yields
    SubjectObjectId), beside the concrete subjects the walk meets; hand-derived answers, also the
    oracle's (tests/test_oracle.py)."""
    tuples, perm, kind, want = WILD_CASES[case]
    e = make_engine(WILD_SCHEMA, tuples + ["doc:other#viewer@user:zed", "group:h#member@user:yan"],
                    **({"wide_only": True} if path == "wide" else {}))
    c = Client(e)
    got = sorted(s for s, err in c.LookupSubjects(None, consistency.MinLatency(), "doc:d", perm, kind))
    assert got == sorted(n for n, _ in want)
    st, _, srel = kind.partition("#")
    tid = e.type_id(st)
    ids, perms = e.lookup_subjects(e.type_id("doc"), int(e.intern(e.type_id("doc"), ["d"])[0]),
                                   e.relation_id(e.type_id("doc"), perm), tid,
                                   e.relation_id(tid, srel) if srel else E.ELLIPSIS)
    named = sorted(("*" if i == E.ID_WILDCARD else e.object_name(tid, i), p) for i, p in zip(ids.tolist(), perms.tolist()))
    assert named == sorted(want)
    e.close()
