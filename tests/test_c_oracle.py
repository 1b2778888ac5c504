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
