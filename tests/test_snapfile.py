"""On-disk snapshot cache (``gck_save_snapshot`` / ``gck_load_snapshot_file``):
a snapshot saved by one engine and loaded by another answers every check exactly as the saving
engine does and as the oracle over the same relationships does — after text ingest, after Watch
batches (rel.Update, rel/relationship.go:267-301) and with caveats, check contexts and
expirations — and keeps the revision, the tuple count and the interned ids. The load replaces
re-reading the snapshot through ExportRelationships (client/client.go:472-499).

The error paths that are decided before anything reaches the device run on CPU too."""
import os
import random

import numpy as np
import pytest

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item
from tests.test_gpu_delta import apply_to_store, random_batch


def results(e, checks):
    items = e.make_items([parse_check(c) for c in checks])
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    return [(int(p), int(x)) for p, x in zip(perm, err)]


def oracle_results(schema, tuples, checks):
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    return [ck.check(to_oracle_item(parse_check(c))) for c in checks]


@pytest.mark.gpu
@pytest.mark.parametrize("family", ["caveated", "gdocs", "github", "nested"])
def test_round_trip_after_watch_batches(family, tmp_path):
    schema, tuples, checks = gen.FAMILIES[family](4)
    a = E.Engine()
    a.load_schema(schema)
    a.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    rng = random.Random(11)
    for rnd in range(2):
        ups = random_batch(rng, family, store, rnd)
        a.apply_updates_text(2 + rnd, "\n".join(f"{op} {line}" for op, line in ups))
        apply_to_store(store, ups)
    path = str(tmp_path / "snap.gck")
    a.save_snapshot(path)
    assert os.path.getsize(path) > 0 and not os.path.exists(path + ".tmp")

    b = E.Engine()
    b.load_schema(schema)
    b.load_snapshot_file(path)
    assert b.revision == a.revision == 3
    assert b.tuple_count == a.tuple_count == len(store)
    want = oracle_results(schema, list(store.values()), checks)
    assert results(a, checks) == want
    assert results(b, checks) == want
    # interned ids survive: every object the saving engine knows has the same id in the loader
    for tname in ("user", "doc", "group", "repo", "team", "folder", "org"):
        try:
            t = a.type_id(tname)
        except E.GckError:
            continue
        names = sorted({c.split("#")[0].split(":", 1)[1] for c in tuples if c.startswith(tname + ":")})[:50]
        assert list(a.intern(t, names, create=False)) == list(b.intern(t, names, create=False))
    # the loaded snapshot keeps moving with Watch batches
    ups = random_batch(rng, family, store, 7)
    for eng in (a, b):
        eng.apply_updates_text(9, "\n".join(f"{op} {line}" for op, line in ups))
    apply_to_store(store, ups)
    want = oracle_results(schema, list(store.values()), checks)
    assert results(b, checks) == want == results(a, checks)
    a.close()
    b.close()


@pytest.mark.gpu
def test_round_trip_with_check_contexts(tmp_path):
    """Caveat instances keep their ids, so per-call check contexts evaluate identically (and as
    the oracle evaluates them)."""
    from tests.test_gpu_parity import device_results

    schema, tuples, checks = gen.caveated(6)
    ctxs = gen.check_contexts(6, len(checks))
    a = E.Engine()
    a.load_schema(schema)
    a.load_snapshot_text(5, "\n".join(tuples))
    path = str(tmp_path / "c.gck")
    a.save_snapshot(path)
    b = E.Engine()
    b.load_schema(schema)
    b.load_snapshot_file(path)
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, ctxs)]
    assert device_results(b, checks, now_us=gen.NOW_US, contexts=ctxs) == want
    assert device_results(a, checks, now_us=gen.NOW_US, contexts=ctxs) == want
    assert any(p == E.PERM_CONDITIONAL for p, _ in want)
    a.close()
    b.close()


@pytest.mark.gpu
def test_round_trip_prebuilt_device_csrs(tmp_path):
    """Config-4-shaped graph (tests/synth.py) loaded from device-resident CSRs with anonymous
    reserved ids — the bench's ingest — at 2e6 tuples: the reloaded snapshot answers a 64K batch
    bit-exactly as the saving engine and the C oracle do."""
    from tests import synth
    from tests.test_gpu_scale import load_engine, run
    from tests.test_synth import _oracle

    G = synth.build(2e6, device="cuda")
    a = load_engine(G)
    items = synth.checks(G, 65536, seed=21)
    pa, ea = run(a, items)
    path = str(tmp_path / "n.gck")
    a.save_snapshot(path)
    b = E.Engine(device=0)
    b.load_schema(synth.SCHEMA)
    b.load_snapshot_file(path)
    assert b.tuple_count == a.tuple_count and b.revision == a.revision
    pb, eb = run(b, items)
    assert (pa == pb).all() and (ea == eb).all()
    from oracle import corc

    _, prog, tab = _oracle(G)
    cp, ce, _ = corc.check(prog, tab, items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1), threads=16)
    assert (cp == pb).all() and (ce == eb).all()
    a.close()
    b.close()


# ---- error paths (no device needed: refused before any upload) -------------------------------

def test_rejects_foreign_and_corrupt_files(tmp_path):
    e = E.Engine()
    e.load_schema("definition user {}\ndefinition company { relation founder: user }")
    with pytest.raises(E.GckError) as ei:
        e.save_snapshot(str(tmp_path / "x.gck"))  # nothing committed
    assert ei.value.code == E.GCK_E_STATE
    with pytest.raises(E.GckError) as ei:
        e.load_snapshot_file(str(tmp_path / "missing.gck"))
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    bad = tmp_path / "bad.gck"
    bad.write_bytes(b"not a snapshot file at all")
    with pytest.raises(E.GckError) as ei:
        e.load_snapshot_file(str(bad))
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    # a header saved under another schema text
    other = "definition user {}"
    hdr = b"GCKSNAP\x01" + len(other).to_bytes(8, "little") + other.encode()
    (tmp_path / "other.gck").write_bytes(hdr)
    with pytest.raises(E.GckError) as ei:
        e.load_snapshot_file(str(tmp_path / "other.gck"))
    assert ei.value.code == E.GCK_E_SCHEMA
    e.close()


def _snapfile(schema, counts, rows, off, nbr, n_tuples=None):
    """A hand-written snapshot file (snapfile.cpp layout) with one plain CSR of relation 0."""
    le = lambda v, n: int(v).to_bytes(n, "little")
    b = b"GCKSNAP\x01" + le(len(schema), 8) + schema.encode() + le(7, 8) + le(len(nbr) if n_tuples is None else n_tuples, 8)
    b += le(len(counts), 4) + b"".join(le(c, 4) + le(0, 4) for c in counts)
    b += le(0, 4) + le(1, 4)
    b += le(0, 2) + le(0, 2) + le(0xFFFF, 2) + le(0, 1) + le(0, 1) + le(rows, 4) + le(len(nbr), 8)
    b += np.asarray(off, np.uint32).tobytes() + np.asarray(nbr, np.uint32).tobytes()
    return b + le(0x444E455041534B43, 8)


@pytest.mark.parametrize("case", ["rows", "offsets", "neighbour", "unsorted", "wildcard"])
def test_rejects_inconsistent_csrs(tmp_path, case):
    """A file whose CSR disagrees with its own interner (row count, neighbour ids), or whose
    offsets / rows are not what build_csrs writes, is refused before any device upload, and the
    engine keeps its state."""
    schema = "definition user {}\ndefinition company { relation founder: user }"
    counts = [4, 3]  # users, companies
    off, nbr, rows = [0, 1, 3, 4], [2, 0, 3, 1], 3
    if case == "rows":  # more rows than objects of the type
        rows, off = 4, [0, 1, 3, 4, 4]
    elif case == "offsets":
        off = [0, 3, 1, 4]
    elif case == "neighbour":
        nbr = [2, 0, 4, 1]
    elif case == "unsorted":
        nbr = [2, 3, 0, 1]
    elif case == "wildcard":
        nbr = [2, 0, 0xFFFFFFFF, 1]
    path = tmp_path / f"{case}.gck"
    path.write_bytes(_snapfile(schema, counts, rows, off, nbr))
    e = E.Engine()
    e.load_schema(schema)
    with pytest.raises(E.GckError) as ei:
        e.load_snapshot_file(str(path))
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT, ei.value
    assert e.revision == 0
    e.close()


@pytest.mark.gpu
def test_interned_pages_match_text_ingest():
    """gck_add_tuples pages (threaded validation + radix-sorted CSR build) give the snapshot the
    text ingest gives; a page holding one invalid tuple is refused whole (nothing staged)."""
    from oracle import spicedb_ref as ref

    schema, tuples, checks = gen.gdocs(3)
    tuples = tuples + tuples[:40]  # duplicates: the last write wins
    a = E.Engine()
    a.load_schema(schema)
    a.load_snapshot_text(1, "\n".join(tuples))
    b = E.Engine()
    b.load_schema(schema)
    recs = np.zeros(len(tuples), dtype=E.TUPLE_DTYPE)
    for i, line in enumerate(tuples):
        t = ref.parse_tuple(line)
        rt, st = b.type_id(t.resource_type), b.type_id(t.subject_type)
        recs[i]["resource_type"], recs[i]["subject_type"] = rt, st
        recs[i]["relation"] = b.relation_id(rt, t.relation)
        recs[i]["resource_id"] = b.intern(rt, [t.resource_id], create=True)[0]
        recs[i]["subject_id"] = b.intern(st, [t.subject_id], create=True)[0]
        recs[i]["subject_relation"] = (E.ELLIPSIS if t.subject_relation == ref.ELLIPSIS
                                       else b.relation_id(st, t.subject_relation))
    b.begin_snapshot(1)
    bad = recs[:300].copy()
    bad[250]["relation"] = 0xFFF0
    with pytest.raises(E.GckError):
        b.add_tuples(bad)
    for k in range(0, len(recs), 97):
        b.add_tuples(recs[k:k + 97])
    b.commit_snapshot()
    assert b.tuple_count == a.tuple_count
    assert results(b, checks) == results(a, checks) == oracle_results(schema, tuples, checks)
    a.close()
    b.close()
