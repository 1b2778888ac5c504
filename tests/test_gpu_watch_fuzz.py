"""A Watch x join fuzz: hypothesis-driven CREATE / TOUCH / DELETE batches on
the nested-group family (BASELINE config 4's shape) — memberships, nesting changes across any
layers (the group DAG stays acyclic, as config 4's; tests/test_gpu_watch_nested.py covers cycles), brand-new groups granted to documents, and skewed batches that pile many updates
on one object — applied through gck_apply_updates (delta.inc), and after every batch the engine's
answers compared with the oracle over the updated relationships and with a snapshot rebuilt from
them. Two engines run the same stream: one whose stage A is the closure join (closure.inc), one
whose stage A is the label join (labels.inc); each must still answer through its join after every
batch (closure_checks > 0 / label_checks > 0). Stream semantics: rel.Update
(rel/relationship.go:267-301) as Client.UpdatesSinceRevision delivers it (client/client.go:370-413)."""
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu

N_USERS, N_GROUPS, N_DOCS = 120, 48, 40


def _key(line):
    res, sub = line.split("@", 1)
    return res, sub


@st.composite
def batches(draw, n_batches):
    """n_batches Watch batches over the nested family's names (gen.nested's u / g / d ids), as
    lists of (op, relationship line)."""
    out = []
    for b in range(n_batches):
        kind = draw(st.sampled_from(["mixed", "mixed", "nesting", "skew", "new_groups"]))
        ups = []
        if kind == "skew":  # many updates on one object: members and nesting of one group
            g = draw(st.integers(0, N_GROUPS - 1))
            for _ in range(draw(st.integers(10, 40))):
                if draw(st.booleans()):
                    ups.append((draw(st.sampled_from(["CREATE", "TOUCH", "DELETE"])),
                                f"group:g{g}#member@user:u{draw(st.integers(0, N_USERS - 1))}"))
                elif g > 0:  # nesting into it from a lower group (the hierarchy stays acyclic)
                    h = draw(st.integers(0, g - 1))
                    ups.append((draw(st.sampled_from(["CREATE", "DELETE"])), f"group:g{h}#member@group:g{g}#member"))
        elif kind == "new_groups":  # groups the snapshot has never seen, nested and granted
            for k in range(draw(st.integers(1, 4))):
                name = f"gn{b}_{k}"
                for _ in range(draw(st.integers(1, 5))):
                    ups.append(("CREATE", f"group:{name}#member@user:u{draw(st.integers(0, N_USERS - 1))}"))
                x = draw(st.integers(0, N_GROUPS - 2))
                ups.append(("CREATE", f"group:g{x}#member@group:{name}#member"))
                if draw(st.booleans()):  # (below x: no cycle through the new group)
                    ups.append(("CREATE", f"group:{name}#member@group:g{draw(st.integers(x + 1, N_GROUPS - 1))}#member"))
                ups.append(("CREATE", f"doc:d{draw(st.integers(0, N_DOCS - 1))}#viewer@group:{name}#member"))
        else:
            n = draw(st.integers(1, 30))
            for _ in range(n):
                op = draw(st.sampled_from(["CREATE", "TOUCH", "DELETE", "DELETE"]))
                x = draw(st.integers(0, 9))
                if x < 5 and kind == "mixed":
                    line = f"group:g{draw(st.integers(0, N_GROUPS - 1))}#member@user:u{draw(st.integers(0, N_USERS - 1))}"
                elif x < 7 and kind == "mixed":
                    line = f"doc:d{draw(st.integers(0, N_DOCS - 1))}#viewer@group:g{draw(st.integers(0, N_GROUPS - 1))}#member"
                else:  # nesting across any layers, lower group to higher (acyclic, as config 4's DAG)
                    a = draw(st.integers(0, N_GROUPS - 2))
                    c = draw(st.integers(a + 1, N_GROUPS - 1))
                    line = f"group:g{a}#member@group:g{c}#member"
                ups.append((op, line))
        out.append(ups)
    return out


def _checks(seed, store, ups):
    import random
    rng = random.Random(seed)
    cs = [f"doc:d{rng.randrange(N_DOCS)}#view@user:u{rng.randrange(N_USERS)}" for _ in range(300)]
    cs += [f"group:g{rng.randrange(N_GROUPS)}#member@user:u{rng.randrange(N_USERS)}" for _ in range(60)]
    for op, line in ups:  # the batch's own objects
        res, sub = _key(line)
        obj = res.split("#")[0]
        if obj.startswith("group:"):
            cs.append(f"{obj}#member@user:u{rng.randrange(N_USERS)}")
            cs += [f"doc:d{rng.randrange(N_DOCS)}#view@{sub}" for _ in range(2) if sub.startswith("user:")]
        else:
            cs.append(f"{obj}#view@user:u{rng.randrange(N_USERS)}")
    return cs


def _results(e, checks):
    items = e.make_items([parse_check(c) for c in checks])
    e.reset_stats()
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    return [(int(p), int(x)) for p, x in zip(perm, err)], e.stats()


@settings(max_examples=5, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
@given(stream=batches(12))
def test_watch_stream_keeps_both_joins_exact(stream):
    """5 streams x 12 batches (60 batches per engine): after every batch both engines equal the
    oracle and a rebuilt snapshot bit-exactly, and each still answers through its join."""
    schema, tuples, _ = gen.nested(11, n_users=N_USERS, n_groups=N_GROUPS, layers=6, n_docs=N_DOCS)
    store = {_key(t): t for t in tuples}
    engines = {"closure": E.Engine(labels=False), "labels": E.Engine(closure=False)}
    for e in engines.values():
        e.load_schema(schema)
        e.load_snapshot_text(1, "\n".join(tuples))
    try:
        for b, ups in enumerate(stream):
            text = "\n".join(f"{op} {line}" for op, line in ups)
            for e in engines.values():
                e.apply_updates_text(2 + b, text)
            for op, line in ups:
                if op == "DELETE":
                    store.pop(_key(line), None)
                else:
                    store[_key(line)] = line
            checks = _checks(b, store, ups)
            ck = oracle_for(schema, list(store.values()), now=gen.NOW_US / 1e6)
            want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
            rebuilt = E.Engine()
            rebuilt.load_schema(schema)
            rebuilt.load_snapshot_text(2 + b, "\n".join(store.values()))
            got_r, _ = _results(rebuilt, checks)
            rebuilt.close()
            assert got_r == want, ("rebuilt", b, [(c, w, g) for c, w, g in zip(checks, want, got_r) if w != g][:5])
            for name, e in engines.items():
                assert e.tuple_count == len(store), (name, b)
                got, stt = _results(e, checks)
                bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
                assert not bad, (name, b, ups[:8], bad[:5])
                if name == "closure":
                    assert stt["closure_checks"] > 0, (b, stt)
                else:
                    assert stt["label_checks"] > 0, (b, stt)
    finally:
        for e in engines.values():
            e.close()
