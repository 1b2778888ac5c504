"""The label join (gochugaru_amd/csrc/labels.inc) against the oracle: hub hierarchies (nested
groups, teams inside organisations), resource-side flattening through arrow chains (folder
forests), exclusion and intersection terms, wildcards, the extension records of resources whose
grants do not fit a slot, cover lists of users in many groups, and what it must leave to the wave
bundles (resources at the depth budget, userset subjects, other subject types, cyclic
hierarchies). Every answer is compared with oracle/spicedb_ref.py, and the label
path's use is asserted from the engine's counters."""
import json
import random

import pytest

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu


def _run(schema, tuples, checks, max_depth=50, **kw):
    ck = oracle_for(schema, tuples, max_depth=max_depth, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    e = E.Engine(max_depth=max_depth, **kw)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    got = [(int(p), int(x)) for p, x in zip(perm, err)]
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
    st = e.stats()
    e.close()
    assert not bad, bad[:10]
    return st, want


GDOCS_WIDE = gen.GDOCS


def _folder_chain_graph(rng, n_users=40, n_groups=30, depth=12, n_docs=60, fat=False):
    """A folder chain `depth` long with grants on every folder (so deep documents flatten to many
    users and groups: extension records when `fat`), nested groups, a public document."""
    t = []
    for g in range(1, n_groups):
        t.append(f"group:g{g}#member@group:g{rng.randrange(0, g)}#member")
    for g in range(n_groups):
        for _ in range(rng.randrange(1, 4)):
            t.append(f"group:g{g}#member@user:u{rng.randrange(n_users)}")
    for f in range(1, depth):
        t.append(f"folder:f{f}#parent@folder:f{f - 1}")
    for f in range(depth):
        for _ in range(rng.randrange(1, 6 if fat else 2)):
            t.append(f"folder:f{f}#viewer@user:u{rng.randrange(n_users)}")
        t.append(f"folder:f{f}#editor@group:g{rng.randrange(n_groups)}#member")
    for d in range(n_docs):
        t.append(f"doc:d{d}#parent@folder:f{rng.randrange(depth)}")
        t.append(f"doc:d{d}#owner@user:u{rng.randrange(n_users)}")
        if d % 17 == 0:
            t.append(f"doc:d{d}#viewer@user:*")
        if rng.random() < 0.5:
            t.append(f"doc:d{d}#editor@group:g{rng.randrange(n_groups)}#member")
    checks = [f"doc:d{rng.randrange(n_docs)}#{p}@user:u{rng.randrange(n_users + 3)}"
              for p in ("view", "edit") for _ in range(300)]
    return sorted(set(t)), checks


@pytest.mark.parametrize("fat", [False, True])
def test_folder_chains_flatten(fat):
    schema = GDOCS_WIDE
    tuples, checks = _folder_chain_graph(random.Random(3 + fat), fat=fat)
    st, want = _run(schema, tuples, checks)
    assert st["slot_checks"] > 0
    assert any(w[0] == 2 for w in want) and any(w[0] == 1 for w in want)


def test_github_terms_exclusion_intersection():
    """read = (reader + writer + admin + org->is_member) - banned; write = (writer + admin) &
    org->is_member: organisations are hubs over their teams; banned users and users outside the
    organisation flip the answers."""
    for seed in range(1, 5):
        schema, tuples, checks = gen.github(seed)
        st, _ = _run(schema, tuples, checks)
        assert st["slot_checks"] > 0, seed
        # the same with the closure join and labels off: identical answers (the oracle says so)
        _run(schema, tuples, checks, labels=False)


def test_user_in_many_groups_uses_cover_lists():
    """A user listed by 40 unrelated groups: its covers exceed a slot, so its checks read the
    cover list (the second round) and still match the oracle."""
    rng = random.Random(11)
    t = [f"group:g{g}#member@user:hub" for g in range(40)]
    t += [f"group:g{g}#member@user:u{g}" for g in range(40)]
    t += [f"doc:d{d}#viewer@group:g{rng.randrange(40)}#member" for d in range(50)]
    t += [f"doc:d{d}#owner@user:u{d % 7}" for d in range(50)]
    schema = """
definition user {}
definition group { relation member: user | group#member }
definition doc {
  relation owner: user
  relation viewer: user | group#member
  permission view = viewer + owner
}"""
    checks = [f"doc:d{d}#view@user:{u}" for d in range(50) for u in ("hub", "u3", "u9", "nobody")]
    st, want = _run(schema, tuples=sorted(set(t)), checks=checks)
    assert st["slot_checks"] > 0
    assert all(w[0] == 2 for c, w in zip(checks, want) if c.endswith("@user:hub"))


def test_deferred_shapes_match_the_oracle():
    """What the label join leaves to the bundles — userset subjects, a subject type that is not
    the slots' type, unknown ids, relations (not permissions) — is still answered exactly."""
    schema, tuples, _ = gen.gdocs(2)
    checks = ["doc:d1#view@group:g1#member", "doc:d2#edit@group:g3#member", "group:g1#member@user:u1",
              "doc:d3#view@user:no_such_user", "doc:no_such#view@user:u1", "doc:d4#viewer@user:u2",
              "folder:f1#view@user:u5", "folder:f2#edit@group:g2#member"]
    _run(schema, tuples, checks)


def test_resources_at_the_budget_are_deferred():
    """near_budget: resources whose dispatch height reaches max_depth carry the overflow mark;
    the exact-depth path answers them (MAX_DEPTH errors included)."""
    for seed in (1, 2):
        schema, tuples, checks = gen.near_budget(seed)
        _run(schema, tuples, checks, max_depth=gen.FAMILY_DEPTH.get("near_budget", 50))


def test_cyclic_hierarchy_condensed():
    """Cycles in the group hierarchy are condensed (labels.inc hier_scc); resources that reach a
    cycle sit at the depth budget and are deferred to the exact-depth path."""
    for seed in (1, 2):
        schema, tuples, checks = gen.cyclic(seed)
        _run(schema, tuples, checks, max_depth=gen.FAMILY_DEPTH.get("cyclic", 50))


def test_labels_follow_watch_batches():
    """A Watch batch rebuilds the slots: grants added and removed through the folder chain and the
    group hierarchy are seen by the next check."""
    schema = GDOCS_WIDE
    tuples, checks = _folder_chain_graph(random.Random(5))
    e = E.Engine()
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    cur = set(tuples)
    rng = random.Random(9)
    for rev in range(2, 5):
        ups = []
        for t in rng.sample(sorted(cur), 6):
            ups.append("DELETE " + t)
            cur.discard(t)
        for _ in range(6):
            t = f"folder:f{rng.randrange(12)}#viewer@user:u{rng.randrange(40)}"
            ups.append("TOUCH " + t)
            cur.add(t)
        e.apply_updates_text(rev, "\n".join(ups))
        ck = oracle_for(schema, sorted(cur), now=gen.NOW_US / 1e6)
        want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
        items = e.make_items([parse_check(c) for c in checks])
        perm, err = e.check_bulk(items, now_us=gen.NOW_US)
        got = [(int(p), int(x)) for p, x in zip(perm, err)]
        assert got == want, rev
    e.close()


# ---- the caveat plane (BASELINE config 5 shape: caveated grants through folder chains) -------

CAV_PLANE = """
caveat only_on_tuesday(day_of_the_week string) {
  day_of_the_week == "tuesday"
}
caveat before_2030(now timestamp) {
  now < timestamp("2030-01-01T00:00:00Z")
}
definition user {}
definition group {
  relation member: user | group#member
}
definition folder {
  relation parent: folder
  relation viewer: user | group#member | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday | user with before_2030
  permission edit = editor + parent->edit
  permission view = viewer + edit + parent->view
}
definition doc {
  relation parent: folder
  relation owner: user
  relation viewer: user | user:* | group#member | user with only_on_tuesday | user:* with only_on_tuesday | user with expiration
  relation banned: user | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday
  permission edit = owner + editor + parent->edit
  permission view = viewer + edit + parent->view
  permission strict = view - banned
  permission both = view & edit
}
use expiration
"""

CAV_CONTEXTS = [None, {"day_of_the_week": "tuesday"}, {"day_of_the_week": "monday"},
                {"now": "2025-01-01T00:00:00Z"}, {"now": "2031-01-01T00:00:00Z", "day_of_the_week": "tuesday"},
                {"now": "not a timestamp"}]


def _caveat_plane_graph(rng, n_users=60, n_groups=20, n_folders=24, n_docs=120):
    """Config 5 in small: a folder forest with caveated user grants on every level — a partial
    caveat, one decided by its stored context alone (true or false), another caveat — nested
    groups, caveated wildcards and bans, and a few expiring grants (left to the bundles)."""
    def user_grant():
        u = f"user:u{rng.randrange(n_users)}"
        x = rng.random()
        if x < 0.45:
            return u
        if x < 0.75:
            return u + "[only_on_tuesday]"
        if x < 0.85:
            return u + '[only_on_tuesday:{"day_of_the_week":"tuesday"}]'
        return u + '[only_on_tuesday:{"day_of_the_week":"monday"}]'
    t = []
    for g in range(1, n_groups):
        t.append(f"group:g{g}#member@group:g{rng.randrange(0, g)}#member")
    for g in range(n_groups):
        for _ in range(rng.randrange(1, 4)):
            t.append(f"group:g{g}#member@user:u{rng.randrange(n_users)}")
    for f in range(1, n_folders):
        t.append(f"folder:f{f}#parent@folder:f{rng.randrange(max(0, f - 4), f)}")
    for f in range(n_folders):
        for _ in range(rng.randrange(0, 4)):
            t.append(f"folder:f{f}#viewer@{user_grant()}")
        if rng.random() < 0.3:
            t.append(f"folder:f{f}#editor@user:u{rng.randrange(n_users)}[before_2030]")
        if rng.random() < 0.4:
            t.append(f"folder:f{f}#editor@group:g{rng.randrange(n_groups)}#member")
    for d in range(n_docs):
        t.append(f"doc:d{d}#parent@folder:f{rng.randrange(n_folders)}")
        t.append(f"doc:d{d}#owner@user:u{rng.randrange(n_users)}")
        for _ in range(rng.randrange(0, 3)):
            t.append(f"doc:d{d}#viewer@{user_grant()}")
        if rng.random() < 0.5:
            t.append(f"doc:d{d}#editor@{user_grant()}")
        if d % 13 == 0:
            t.append(f"doc:d{d}#viewer@user:*[only_on_tuesday]")
        if d % 29 == 0:
            t.append(f"doc:d{d}#viewer@user:*")
        if d % 31 == 0:
            t.append(f"doc:d{d}#viewer@user:u{rng.randrange(n_users)}[expiration:2999-01-01T00:00:00Z]")
        if rng.random() < 0.3:
            t.append(f"doc:d{d}#banned@{user_grant()}")
    checks = [f"doc:d{rng.randrange(n_docs)}#{p}@user:u{rng.randrange(n_users)}"
              for p in ("view", "edit", "strict", "both") for _ in range(500)]
    checks += [f"folder:f{rng.randrange(n_folders)}#{p}@user:u{rng.randrange(n_users)}"
               for p in ("view", "edit") for _ in range(200)]
    return sorted(set(t)), checks


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_caveat_plane(seed, lazy):
    """Caveated grants in the label join's slots (labels.inc kLjCav): a term that reaches the
    subject only through partial caveats is decided by the caveat under the check's context —
    the dense outcome table, or the lazy (instance, context) map when every check brings its own
    context — in SpiceDB's tri-state algebra through exclusion and intersection, CONDITIONAL
    without a context, the item error when the caveat fails to evaluate. Bit-exact against the
    oracle; nearly every check answered by the label join (resources with an expiring grant are
    the bundles')."""
    rng = random.Random(seed)
    tuples, checks = _caveat_plane_graph(rng)
    ctxs = [rng.choice(CAV_CONTEXTS) for _ in checks]
    if lazy:  # distinct contexts: more (instance, context) pairs than the dense table takes
        ctxs = [dict(c or {}, k=i) for i, c in enumerate(ctxs)]
    ck = oracle_for(CAV_PLANE, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, ctxs)]
    e = E.Engine()
    e.load_schema(CAV_PLANE)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    texts, slots = [], {}
    for i, x in enumerate(ctxs):
        if x is None:
            continue
        js = json.dumps(x, sort_keys=True)
        if js not in slots:
            texts.append(js)
            slots[js] = len(texts)
        items[i]["context_slot"] = slots[js]
    e.reset_stats()
    perm, err = e.check_bulk(items, now_us=gen.NOW_US, contexts=texts)
    st = e.stats()
    e.close()
    got = [(int(p), int(x)) for p, x in zip(perm, err)]
    bad = [(c, x, w, g) for c, x, w, g in zip(checks, ctxs, want, got) if w != g]
    assert not bad, bad[:10]
    kinds = {w for w in want}
    assert (3, 0) in kinds and (2, 0) in kinds and (1, 0) in kinds and (0, 6) in kinds, kinds
    assert st["label_checks"] >= 0.8 * len(checks), (st["label_checks"], len(checks))
    if lazy:
        assert st["caveat_passes"] >= 1, st


@pytest.mark.parametrize("lazy", [False, True])
def test_caveat_plane_on_the_engine_queue(lazy):
    """Device batches with check contexts on the engine's stream: the label join with the caveat
    plane is dispatched into the engine's HSA queue (aql.inc) — its Ctx written with the kernel
    arguments, the checks' caveat flags cleared by the join itself — and later batches (chained
    behind bundles) launch through HIP; a lazy batch's rerun passes follow it. Every batch
    bit-exact against the oracle."""
    import os

    import numpy as np
    import torch
    rng = random.Random(5)
    tuples, checks = _caveat_plane_graph(rng)
    ctxs = [rng.choice(CAV_CONTEXTS) for _ in checks]
    if lazy:
        ctxs = [dict(c or {}, k=i) for i, c in enumerate(ctxs)]
    ck = oracle_for(CAV_PLANE, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, ctxs)]
    e = E.Engine()
    e.load_schema(CAV_PLANE)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    texts, slots = [], {}
    for i, x in enumerate(ctxs):
        if x is None:
            continue
        js = json.dumps(x, sort_keys=True)
        if js not in slots:
            texts.append(js)
            slots[js] = len(texts)
        items[i]["context_slot"] = slots[js]
    n = len(items)
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    e.reset_stats()
    for rnd in range(4):
        perm = torch.full((n,), 0xFF, dtype=torch.uint8, device="cuda")
        err = torch.full((n,), -7, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        e.submit(d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(), now_us=gen.NOW_US, contexts=texts,
                 device=True, engine_stream=True).wait()
        got = [(int(p), int(x)) for p, x in zip(perm.cpu().numpy(), err.cpu().numpy())]
        bad = [(c, x, w, g) for c, x, w, g in zip(checks, ctxs, want, got) if w != g]
        assert not bad, (rnd, bad[:10])
    st = e.stats()
    e.close()
    assert st["label_checks"] >= 0.8 * 4 * n, st["label_checks"]
    if os.path.exists(os.path.join(os.path.dirname(E.__file__), "libgck_kernels.co")):
        assert st["aql_batches"] >= 1, st


def test_caveat_plane_without_contexts():
    """No check contexts: a subject reached only through partial caveats is CONDITIONAL; one
    decided by its stored context alone is a plain grant or none."""
    rng = random.Random(3)
    tuples, checks = _caveat_plane_graph(rng)
    st, want = _run(CAV_PLANE, tuples, checks)
    assert any(w == (3, 0) for w in want)
    assert st["label_checks"] >= 0.8 * len(checks), st["label_checks"]


def test_direct_grant_churn_keeps_the_tables():
    """Watch batches that change only direct grants (config 5's churn: viewers and editors created,
    touched with and without a caveat, deleted — wildcard grants of documents included) keep the
    label tables: the subjects they touch are marked dirty and their checks go to the bundles, a
    document whose wildcard grant changed is deferred, everything else the tables answer as
    before. Bit-exact against the oracle after every batch, with most checks still through the
    join."""
    rng = random.Random(11)
    tuples, checks = _caveat_plane_graph(rng, n_users=200, n_docs=300)
    ctxs = [rng.choice(CAV_CONTEXTS[:4]) for _ in checks]
    cur = {t.split("[")[0]: t for t in tuples}  # (one relationship per key, as SpiceDB keeps it)
    e = E.Engine()
    e.load_schema(CAV_PLANE)
    e.load_snapshot_text(1, "\n".join(sorted(cur.values())))
    items = e.make_items([parse_check(c) for c in checks])
    texts, slots = [], {}
    for i, x in enumerate(ctxs):
        if x is None:
            continue
        js = json.dumps(x, sort_keys=True)
        if js not in slots:
            texts.append(js)
            slots[js] = len(texts)
        items[i]["context_slot"] = slots[js]
    grants = [k for k in cur if ("#viewer@user:" in k or "#editor@user:" in k)]
    for rev in range(2, 6):
        ups = []
        for k in rng.sample(sorted(grants), 12):  # deletes and caveat toggles of existing grants
            if rng.random() < 0.4:
                ups.append("DELETE " + cur.pop(k))
                grants.remove(k)
            else:
                t = k + ("[only_on_tuesday]" if "[" not in cur[k] else "")
                ups.append("TOUCH " + t)
                cur[k] = t
        for _ in range(12):  # new grants, caveated or not, and a public document now and then
            d = rng.randrange(300)
            k = (f"doc:d{d}#viewer@user:*" if rng.random() < 0.15 else
                 f"{rng.choice(['doc:d%d' % d, 'folder:f%d' % rng.randrange(24)])}#{rng.choice(['viewer', 'editor'])}"
                 f"@user:u{rng.randrange(200)}")
            t = k + ("[only_on_tuesday]" if rng.random() < 0.3 and "*" not in k else "")
            ups.append("TOUCH " + t)
            cur[k] = t
            if k not in grants:
                grants.append(k)
        e.apply_updates_text(rev, "\n".join(ups))
        ck = oracle_for(CAV_PLANE, sorted(cur.values()), now=gen.NOW_US / 1e6)
        want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, ctxs)]
        e.reset_stats()
        perm, err = e.check_bulk(items, now_us=gen.NOW_US, contexts=texts)
        st = e.stats()
        got = [(int(p), int(x)) for p, x in zip(perm, err)]
        bad = [(c, x, w, g) for c, x, w, g in zip(checks, ctxs, want, got) if w != g]
        assert not bad, (rev, bad[:10])
        assert st["label_checks"] >= 0.4 * len(checks), (rev, st["label_checks"])
    e.close()
