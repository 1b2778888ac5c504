"""The closure join's slot fast path (closure.inc, tree labels + covers from bidir.inc
build_ancestors) on group hierarchies that are far from trees: every group below the top layer
has one to three parents, so most groups' ancestors are not their tree ancestors and their
covers carry several entries. Every (doc, user) pair is checked against the oracle, with the
slots and without them; the slots must decide the checks themselves (slot_checks), exactly."""
import random

import pytest

from tests.helpers import oracle_for, parse_check, to_oracle_item
from tests.test_gpu_parity import device_results, make_engine

pytestmark = pytest.mark.gpu

SCHEMA = """
definition user {}
definition group { relation member: user | group#member }
definition doc { relation viewer: group#member  permission view = viewer }
"""


def dag(seed, layers=6, width=8, max_parents=3, users=30, docs=20):
    rng = random.Random(seed)
    groups = [[f"g{l}_{k}" for k in range(width)] for l in range(layers)]
    tuples = []
    for l in range(1, layers):
        for g in groups[l]:
            for p in rng.sample([x for ll in range(l) for x in groups[ll]], rng.randint(1, max_parents)):
                tuples.append(f"group:{p}#member@group:{g}#member")
    flat = [g for layer in groups for g in layer]
    us = [f"u{i}" for i in range(users)]
    for u in us:
        for g in rng.sample(flat, rng.randint(1, 4)):
            tuples.append(f"group:{g}#member@user:{u}")
    for d in range(docs):
        for g in rng.sample(flat, rng.randint(1, 3)):
            tuples.append(f"doc:d{d}#viewer@group:{g}#member")
    checks = [f"doc:d{d}#view@user:{u}" for d in range(docs) for u in us]
    return tuples, checks


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
@pytest.mark.parametrize("max_parents", [1, 2, 3])
def test_slots_exact_on_dags(seed, max_parents):
    tuples, checks = dag(seed, max_parents=max_parents)
    ck = oracle_for(SCHEMA, tuples)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    assert {w[0] for w in want} == {1, 2}
    for slots in (True, False):
        e = make_engine(SCHEMA, tuples, slots=slots)
        e.reset_stats()
        got = device_results(e, checks)
        bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
        assert not bad, (slots, bad[:10])
        st = e.stats()
        if slots and max_parents == 1:  # a forest: every cover is one entry, every check fits
            assert st["slot_checks"] == len(checks), st["slot_checks"]
        elif slots:  # three parents per group: large covers overflow some users' slots
            assert st["slot_checks"] > 0.5 * len(checks), st["slot_checks"]
        else:
            assert st["slot_checks"] == 0
        e.close()
