"""Cross-checks the two independent oracle restatements: the C oracle (check_oracle.c, used at
scale and as the CPU baseline) against the Python oracle (pinned by the reference's known
answers). CPU only."""
import numpy as np
import pytest

from oracle import corc
from oracle import spicedb_ref as ref
from tests import gen
from tests.helpers import expected_code, iso_to_unix, load_golden, parse_check, to_oracle_item

SEM = load_golden("semantics.json")


def run_both(schema, tuples, checks, now=0.0, max_depth=50, threads=1):
    sc = ref.Schema(schema)
    tps = [ref.parse_tuple(t) for t in tuples]
    py = ref.Checker(sc, ref.TupleStore(tps), max_depth=max_depth, now=now, evaluate_caveats=False)
    items = [to_oracle_item(parse_check(c)) for c in checks]
    want = [py.check(it) for it in items]
    st = corc.Store(sc, tps)
    perm, err, _ = corc.check(st.program, st.csr_table(), st.items(items), now_us=int(now * 1e6),
                              max_depth=max_depth, threads=threads)
    got = [(int(p), int(e)) for p, e in zip(perm, err)]
    return want, got


@pytest.mark.parametrize("family", sorted(gen.FAMILIES))
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_c_oracle_matches_python_oracle(family, seed):
    schema, tuples, checks = gen.FAMILIES[family](seed)
    want, got = run_both(schema, tuples, checks, now=gen.NOW_US / 1e6, threads=2,
                         max_depth=gen.FAMILY_DEPTH.get(family, 50))
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
    assert not bad, bad[:10]


def test_c_oracle_semantics_fixtures():
    now = iso_to_unix(SEM["now"])
    s1 = SEM["suites"][0]
    want, got = run_both(s1["schema"], s1["tuples"], [c[0] for c in s1["checks"]], now=now)
    assert got == [expected_code(c[1]) for c in s1["checks"]]
    s2 = SEM["suites"][1]
    for chk, depth, label, _ in s2["depth_checks"]:
        _, got = run_both(s2["schema"], s2["tuples"], [chk], max_depth=depth)
        assert got == [expected_code(label)], (chk, depth)
    s3 = SEM["suites"][2]
    _, got = run_both(s3["schema"], s3["tuples"], [c[0] for c in s3["caveat_checks"]], now=now)
    assert got == [expected_code(c[2]) for c in s3["caveat_checks"]]


def test_count_bfs_rule():
    schema, tuples, checks = gen.nested(7)
    sc = ref.Schema(schema)
    tps = [ref.parse_tuple(t) for t in tuples]
    st = corc.Store(sc, tps)
    items = st.items([to_oracle_item(parse_check(c)) for c in checks])
    a = corc.count_bfs(st.program, st.csr_table(), items, threads=1)
    b = corc.count_bfs(st.program, st.csr_table(), items, threads=4)
    assert a == b and a["expanded"] >= len(checks)
    schema, tuples, checks = gen.github(1)
    st = corc.Store(ref.Schema(schema), [ref.parse_tuple(t) for t in tuples])
    with pytest.raises(ValueError):
        corc.count_bfs(st.program, st.csr_table(), st.items([to_oracle_item(parse_check(checks[0]))]))


QUOTA = """
caveat quota(limit int, used int) {
  used < limit
}
definition user {}
definition group {
  relation member: user | user with quota | group#member
}
definition doc {
  relation viewer: user | user with quota | group#member | group#member with quota
  relation banned: user with quota
  permission view = viewer - banned
}
"""


def quota_case(seed, n_checks=300):
    import random
    rng = random.Random(seed)
    users = [f"u{i}" for i in range(25)]
    tuples = []
    for g in range(6):
        for u in rng.sample(users, 4):
            tuples.append(f"group:g{g}#member@user:{u}" + (f'[quota:{{"limit":{rng.randrange(100)}}}]'
                                                            if rng.random() < 0.5 else ""))
        if g < 5 and rng.random() < 0.6:
            tuples.append(f"group:g{g}#member@group:g{rng.randrange(g + 1, 6)}#member")
    for d in range(15):
        for u in rng.sample(users, 3):
            tuples.append(f"doc:d{d}#viewer@user:{u}" + (f'[quota:{{"limit":{rng.randrange(100)}}}]'
                                                          if rng.random() < 0.6 else ""))
        g = rng.randrange(6)
        tuples.append(f"doc:d{d}#viewer@group:g{g}#member" + (f'[quota:{{"limit":{rng.randrange(100)}}}]'
                                                              if rng.random() < 0.5 else ""))
        if rng.random() < 0.4:
            tuples.append(f'doc:d{d}#banned@user:{rng.choice(users)}[quota:{{"limit":{rng.randrange(100)}}}]')
    checks = [f"doc:d{rng.randrange(15)}#view@user:{rng.choice(users)}" for _ in range(n_checks)]
    used = [None if rng.random() < 0.15 else rng.randrange(100) for _ in checks]
    return tuples, checks, used


def run_quota(tuples, checks, used, threads=1):
    """(Python oracle, C oracle threshold mode) answers of the checks; used[i] None = no context,
    a string = a wrongly typed `used`."""
    sc = ref.Schema(QUOTA)
    tps = [ref.parse_tuple(t) for t in tuples]
    py = ref.Checker(sc, ref.TupleStore(tps))
    items = [to_oracle_item(parse_check(c), None if u is None else {"used": u}) for c, u in zip(checks, used)]
    want = [py.check(it) for it in items]
    st = corc.Store(sc, tps)
    limits = [0] + [dict(ctx)["limit"] for _, ctx in st.caveats[1:]]
    ci = st.items(items)
    vals = []
    for i, u in enumerate(used):
        if u is not None:
            vals.append(corc_used(u))
            ci[i]["context_slot"] = len(vals)
    perm, err = corc.check_quota(st.program, st.csr_table(), ci, np.array(limits), np.array(vals, dtype=np.int64),
                                 threads=threads)
    return want, [(int(p), int(e)) for p, e in zip(perm, err)]


def corc_used(u):
    return np.iinfo(np.int64).min if isinstance(u, str) else u


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_c_oracle_quota_mode_matches_python_oracle(seed):
    tuples, checks, used = quota_case(seed)
    want, got = run_quota(tuples, checks, used, threads=2)
    bad = [(c, u, w, g) for c, u, w, g in zip(checks, used, want, got) if w != g]
    assert not bad, bad[:10]
    assert {w[0] for w in want} >= {1, 2, 3}


def test_caveat_eval_error_fails_only_its_checks():
    """A wrongly typed `used` is an error for the checks whose walk meets the caveat, and for no
    other (single-path data: the walk order cannot matter)."""
    tuples = ['doc:a#viewer@user:x[quota:{"limit":10}]', "doc:b#viewer@user:x", "doc:c#viewer@user:y"]
    checks = ["doc:a#view@user:x", "doc:b#view@user:x", "doc:c#view@user:x", "doc:a#view@user:x"]
    used = ["many", "many", "many", 3]
    want, got = run_quota(tuples, checks, used)
    assert want == got == [(0, ref.ITEM_ERR_CAVEAT_EVAL), (ref.HAS, 0), (ref.NO, 0), (ref.HAS, 0)]
