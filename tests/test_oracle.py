"""Pins the Python oracle (oracle/spicedb_ref.py) against the reference's known answers and
the hand-derived SpiceDB-semantics fixtures. CPU only."""
import pytest

from oracle import spicedb_ref as ref
from tests.lookup_cases import WILD_CASES, WILD_SCHEMA
from tests.helpers import (expected_code, iso_to_unix, load_golden, oracle_for, parse_check,
                           to_oracle_item)

CLIENT = load_golden("client_check.json")
FOUNDERS = load_golden("readme_founders.json")
SEM = load_golden("semantics.json")


@pytest.mark.parametrize("case", CLIENT["cases"], ids=lambda c: c["name"])
def test_client_check_known_answers(case):
    # client/client_test.go:141-216 — HAS -> true, everything else false
    ck = oracle_for(CLIENT["schema"], CLIENT["tuples"])
    got = [ck.check(to_oracle_item(parse_check(s)))[0] == ref.HAS for s in case["checks"]]
    assert got == case["expected"]


def test_readme_founders():
    ck = oracle_for(FOUNDERS["schema"], FOUNDERS["tuples"])
    res = [ck.check(to_oracle_item(parse_check(s))) for s in FOUNDERS["checks"]]
    assert all(p == ref.HAS and e == 0 for p, e in res) == FOUNDERS["expected_all"]
    tuples = [t for t in FOUNDERS["tuples"] if t != FOUNDERS["negative_remove"]]
    ck = oracle_for(FOUNDERS["schema"], tuples)
    res = [ck.check(to_oracle_item(parse_check(s))) for s in FOUNDERS["checks"]]
    assert all(p == ref.HAS for p, _ in res) == FOUNDERS["expected_all_negative"]


def _suite(name):
    return next(s for s in SEM["suites"] if s["name"] == name)


S1 = _suite("gdocs-arrows-exclusion-intersection-wildcard")


@pytest.mark.parametrize("chk", S1["checks"], ids=lambda c: c[0])
def test_semantics_rewrites(chk):
    ck = oracle_for(S1["schema"], S1["tuples"], now=iso_to_unix(SEM["now"]))
    assert ck.check(to_oracle_item(parse_check(chk[0]))) == expected_code(chk[1])


S2 = _suite("depth-budget")


@pytest.mark.parametrize("chk", S2["depth_checks"], ids=lambda c: f"{c[0]}-d{c[1]}")
def test_semantics_depth(chk):
    ck = oracle_for(S2["schema"], S2["tuples"], max_depth=chk[1])
    assert ck.check(to_oracle_item(parse_check(chk[0]))) == expected_code(chk[2])


S3 = _suite("caveats-and-expiration")


@pytest.mark.parametrize("chk", S3["caveat_checks"], ids=lambda c: f"{c[0]}-{c[1]}")
def test_semantics_caveats(chk):
    now = iso_to_unix(SEM["now"])
    item = to_oracle_item(parse_check(chk[0]), chk[1])
    dev = oracle_for(S3["schema"], S3["tuples"], now=now, evaluate_caveats=False)
    assert dev.check(item) == expected_code(chk[2])
    full = oracle_for(S3["schema"], S3["tuples"], now=now, evaluate_caveats=True)
    assert full.check(item) == expected_code(chk[3])


def test_schema_errors():
    bad = [
        "definition a { relation r: nosuch }",
        "definition a { permission p = nosuch }",
        "definition a { relation r: a }\ndefinition a {}",
        "definition a { relation r: a  permission p = r->missing }",
        "definition a { relation r: a:*  permission p = r->p }",
        "definition a { relation r: a with nocaveat }",
    ]
    for s in bad:
        with pytest.raises(ref.SchemaError):
            ref.Schema(s)


def test_precedence_and_flattening():
    sc = ref.Schema("definition u {}\ndefinition d { relation a: u\nrelation b: u\nrelation c: u\n"
                    "permission p = a + b - c\npermission q = a - b + c\npermission r = a & b + c }")
    p = sc.relation("d", "p").expr
    assert p.op == "exclude" and p.children[0].op == "union"
    q = sc.relation("d", "q").expr
    assert q.op == "exclude" and q.children[1].op == "union"
    r = sc.relation("d", "r").expr
    assert r.op == "intersect" and r.children[1].op == "union"


def test_cel_partial_evaluation():
    sc = ref.Schema('caveat c(a int, b string) { a > 3 || b == "x" }\ndefinition u {}')
    e = sc.caveats["c"].expr
    assert ref.cel_eval(e, {"a": 5}) is True
    assert ref.cel_eval(e, {"a": 1}) is ref.UNKNOWN
    assert ref.cel_eval(e, {"a": 1, "b": "y"}) is False
    assert ref.cel_eval(e, {"b": "x"}) is True


def test_cycle_is_max_depth_error():
    # SpiceDB recursion on cyclic data that never reaches the subject ends in max depth
    ck = oracle_for("definition user {}\ndefinition group { relation member: user | group#member }",
                    ["group:a#member@group:b#member", "group:b#member@group:a#member",
                     "group:b#member@user:x"], max_depth=50)
    assert ck.check(to_oracle_item(parse_check("group:a#member@user:x"))) == (ref.HAS, 0)
    assert ck.check(to_oracle_item(parse_check("group:a#member@user:y"))) == (0, ref.ITEM_ERR_MAX_DEPTH)


def test_lookup_resources_known_answers():
    """client/client_test.go:107-139: LookupResources as the oracle's checks over every document."""
    g = load_golden("lookup_resources.json")
    ck = oracle_for(g["schema"], g["tuples"])
    docs = sorted({t.split("#")[0].split(":")[1] for t in g["tuples"]})
    for case in g["cases"]:
        typ, perm = case["permission"].split("#")
        stype, sid = case["subject"].split(":")
        got = [d for d in docs if ck.check(ref.Item(typ, d, perm, stype, sid))[0] == ref.HAS]
        assert got == case["expected"], case["name"]


@pytest.mark.parametrize("case", range(len(WILD_CASES)))
def test_lookup_subjects_wildcard(case):
    """The oracle's LookupSubjects on the hand-derived wildcard cases (parity unpinned by the
    reference: its only LookupSubjects-shaped vectors are client_test.go's LookupResources ones)."""
    tuples, perm, kind, want = WILD_CASES[case]
    ck = oracle_for(WILD_SCHEMA, tuples + ["doc:other#viewer@user:zed", "group:h#member@user:yan"])
    st, _, srel = kind.partition("#")
    got = ck.lookup_subjects("doc", "d", perm, st, srel or ref.ELLIPSIS)
    assert sorted(got) == sorted(want)


@pytest.mark.parametrize("family,seed", [("gdocs", 1), ("github", 2), ("nested", 3), ("caveated", 4)])
def test_lookup_subjects_walk_matches_the_candidate_sweep(family, seed):
    """The oracle's LookupSubjects walk against a brute-force sweep of every subject: the same
    concrete subjects, except that the ones only a wildcard grants fold into "*" (and "*" is
    reported exactly when an absent subject has the permission)."""
    from tests import gen
    schema, tuples, checks = gen.FAMILIES[family](seed)
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    users = sorted({t.split("@", 1)[1].split("[", 1)[0].split(":", 1)[1]
                    for t in tuples if t.split("@", 1)[1].startswith("user:")} - {"*"})
    for c in checks[:6]:
        res = c.split("@", 1)[0]
        rtype, rest = res.split(":", 1)
        rid, perm = rest.split("#", 1)
        got = dict(ck.lookup_subjects(rtype, rid, perm, "user"))
        sweep = {u: p for u in users
                 for p, err in [ck.check(ref.Item(rtype, rid, perm, "user", u))] if p in (ref.HAS, ref.COND)}
        absent = ck.check(ref.Item(rtype, rid, perm, "user", "\x00absent"))[0]
        assert ("*" in got) == (absent in (ref.HAS, ref.COND)), c
        for u, p in sweep.items():
            assert got.get(u) == p or ("*" in got and u not in got), (c, u)
        assert all(u == "*" or u in sweep for u in got), c
