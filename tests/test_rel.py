"""rel/consistency mirrors against the reference's own goldens (rel/relationship_test.go)."""
from datetime import datetime, timezone

import pytest

from gochugaru_amd import consistency, rel
from tests.helpers import load_golden

G = load_golden("rel_strings.json")


@pytest.mark.parametrize("case", G["parse_errors"], ids=lambda c: c["name"])
def test_relationship_parsing_triples(case):
    # rel/relationship_test.go:11-29
    if case["error"] is None:
        rel.FromTriple(case["resource"], case["relation"], case["subject"])
    else:
        with pytest.raises(rel.RelError) as ei:
            rel.FromTriple(case["resource"], case["relation"], case["subject"])
        assert str(ei.value) == case["error"]


@pytest.mark.parametrize("case", G["strings"], ids=lambda c: c["source"])
def test_relationship_string_goldens(case):
    r = rel.MustFromTriple(*case["triple"])
    if "caveat" in case:
        r = r.WithCaveat(case["caveat"][0], case["caveat"][1])
    if "expiration" in case:
        if case["expiration"] == "zero":
            r = r.WithExpiration(rel.ZERO_TIME)
            assert not r.HasExpiration()
        else:
            t = datetime.fromisoformat(case["expiration"].replace("Z", "+00:00"))
            r = r.WithExpiration(t)
            assert r.HasExpiration()
    assert r.String() == case["expected"]
    assert str(r) == case["expected"]


def test_readme_read_example():
    c = G["readme_read_example"]
    assert str(rel.MustFromTriple(*c["triple"])) == c["expected"]


def test_parse_roundtrip():
    for s in ["document:example#viewer@user:jzelinskie",
              "team:a#member@team:b#member",
              'document:example#viewer@user:jzelinskie[only_on_tuesday:{"day_of_the_week":"wednesday"}]',
              "document:example#viewer@user:jzelinskie[expiration:2024-12-25T15:30:00Z]",
              "document:example#viewer@user:x[cav][expiration:2024-12-25T15:30:00.5Z]"]:
        assert rel.Parse(s).String() == s


def test_rfc3339nano_and_numbers():
    t = datetime(2024, 12, 25, 15, 30, 0, 120000, tzinfo=timezone.utc)
    r = rel.MustFromTriple("d:x", "v", "u:y").WithExpiration(t).WithCaveat("c", {"n": 5, "f": 1.5, "b": True})
    assert r.String() == 'd:x#v@u:y[c:{"b":true,"f":1.5,"n":5}][expiration:2024-12-25T15:30:00.12Z]'


def test_parse_object_set_and_typed_relation():
    # rel/strings.go:19-38
    assert rel.ParseObjectSet("document:README") == ("document", "README", "")
    assert rel.ParseObjectSet("document:README#reader") == ("document", "README", "reader")
    with pytest.raises(rel.RelError):
        rel.ParseObjectSet("documentREADME")
    assert rel.ParseTypedRelation("document#reader") == ("document", "reader")
    with pytest.raises(rel.RelError):
        rel.ParseTypedRelation("document")


def test_consistency_constructors():
    # consistency/consistency.go:29-77
    assert consistency.Full().V1Consistency.requirement == consistency.FULLY_CONSISTENT
    assert consistency.MinLatency().V1Consistency.requirement == consistency.MINIMIZE_LATENCY
    a = consistency.AtLeast("42").V1Consistency
    assert (a.requirement, a.token) == (consistency.AT_LEAST_AS_FRESH, "42")
    s = consistency.Snapshot("7").V1Consistency
    assert (s.requirement, s.token) == (consistency.AT_EXACT_SNAPSHOT, "7")
    ctx = consistency.WithOverlapKey(None, "k")
    assert ctx.metadata[consistency.REQUEST_OVERLAP_KEY] == "k"


def test_from_objects():
    r = rel.FromObjects(rel.Object("doc", "1", "view"), rel.Object("user", "a"))
    assert r.String() == "doc:1#view@user:a"
