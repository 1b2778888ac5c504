"""Concurrent and asynchronous checks on one engine (include/gck.h threading contract): pooled
workspaces, gck_check_submit / gck_check_wait, checks racing Watch batches, consistency waits
(consistency.Full after gck_set_head_revision, AtLeast) that the client's retry
(client/client.go:193-211) carries over, and the permanent error for a Snapshot revision the
engine has moved past. Every result is compared with the oracle."""
import os
import threading
import time

import numpy as np
import pytest

from gochugaru_amd import consistency, rel
from gochugaru_amd import engine as E
from gochugaru_amd.client import Client
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu


def _engine(schema, tuples, revision=1, **kw):
    e = E.Engine(**kw)
    e.load_schema(schema)
    e.load_snapshot_text(revision, "\n".join(tuples))
    return e


def _want(schema, tuples, checks):
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    return [ck.check(to_oracle_item(parse_check(c))) for c in checks]


def _got(perm, err):
    return [(int(p), int(x)) for p, x in zip(perm, err)]


@pytest.mark.parametrize("workspaces", [1, 2, 4])
def test_concurrent_callers(workspaces):
    """Four threads, each its own batches of a different family's checks (one engine, one graph
    per family): every result equals the oracle whatever the interleaving."""
    schema, tuples, checks = gen.gdocs(5)
    e = _engine(schema, tuples, workspaces=workspaces)
    want = _want(schema, tuples, checks)
    items = e.make_items([parse_check(c) for c in checks])
    rng = np.random.default_rng(7)
    orders = [rng.permutation(len(checks)) for _ in range(4)]
    errors, results = [], [None] * 4

    def worker(k):
        try:
            out = []
            for rep in range(6):
                idx = orders[k] if rep % 2 else orders[k][::-1]
                perm, err = e.check_bulk(items[idx], now_us=gen.NOW_US)
                got = _got(perm, err)
                out.append(all(got[i] == want[j] for i, j in enumerate(idx)))
            results[k] = out
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert all(r is not None and all(r) for r in results), results
    e.close()


def test_submit_wait_host_and_device():
    import torch
    schema, tuples, checks = gen.github(3)
    e = _engine(schema, tuples, workspaces=3)
    want = _want(schema, tuples, checks)
    items = e.make_items([parse_check(c) for c in checks])
    # three host batches in flight, waited for out of order
    bs = [e.submit(items[k::3], now_us=gen.NOW_US) for k in range(3)]
    for k in (2, 0, 1):
        perm, err = bs[k].wait()
        assert _got(perm, err) == want[k::3]
    # device batches on two streams
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    n = len(items)
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        perm = torch.zeros(n, dtype=torch.uint8, device="cuda")
        err = torch.zeros(n, dtype=torch.int32, device="cuda")
        b = e.submit(d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(), now_us=gen.NOW_US, device=True,
                     stream=s.cuda_stream)
        outs.append((b, perm, err, s))
    for b, perm, err, s in outs:
        b.wait()
        s.synchronize()
        assert _got(perm.cpu().numpy(), err.cpu().numpy()) == want
    # more batches than workspaces: submit blocks until one is released by a wait... so wait in
    # turn (a 4th submit before any wait would block this thread forever by design)
    for _ in range(3):
        b = e.submit(items, now_us=gen.NOW_US)
        assert _got(*b.wait()) == want
    e.close()


def test_submitted_batch_keeps_its_snapshot_across_a_watch_batch():
    """A batch submitted at revision 1 and waited for after a Watch batch moved the snapshot
    to revision 2 answers for revision 1 (the writer finishes it before the swap)."""
    schema, tuples, checks = gen.nested(4)
    e = _engine(schema, tuples, workspaces=2)
    items = e.make_items([parse_check(c) for c in checks])
    want1 = _want(schema, tuples, checks)
    # delete every direct user membership of one group layer: many answers change
    gone = [t for t in tuples if t.startswith("group:g1") and "@user:" in t]
    later = [t for t in tuples if t not in gone]
    want2 = _want(schema, later, checks)
    assert want1 != want2
    b = e.submit(items, now_us=gen.NOW_US)
    e.apply_updates_text(2, "\n".join("DELETE " + t for t in gone))
    assert _got(*b.wait()) == want1
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    assert _got(perm, err) == want2
    e.close()


def test_checks_racing_watch_batches():
    """One thread applies Watch batches (add / remove a chain link) while another checks: every
    check batch equals the oracle of one of the two states (a batch never sees half a Watch
    batch)."""
    schema, tuples, checks = gen.nested(9)
    e = _engine(schema, tuples, workspaces=2)
    items = e.make_items([parse_check(c) for c in checks])
    link = [t for t in tuples if "#member@group:" in t][:20]
    base = [t for t in tuples if t not in link]
    want_a, want_b = _want(schema, tuples, checks), _want(schema, base, checks)
    stop = threading.Event()
    errors = []

    def writer():
        try:
            rev = 1
            while not stop.is_set():
                rev += 1
                e.apply_updates_text(rev, "\n".join("DELETE " + t for t in link))
                rev += 1
                e.apply_updates_text(rev, "\n".join("CREATE " + t for t in link))
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    t = threading.Thread(target=writer)
    t.start()
    seen = set()
    try:
        for _ in range(40):
            got = _got(*e.check_bulk(items, now_us=gen.NOW_US))
            assert got in (want_a, want_b)
            seen.add(got == want_a)
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errors, errors
    e.close()


def test_full_consistency_waits_for_the_head_revision():
    """consistency.Full after SetHeadRevision(3): Unavailable (retried by the client's backoff)
    until a Watch batch moves the snapshot to revision 3, then the answer of revision 3."""
    schema = "definition user {}\ndefinition document { relation reader: user\n permission view = reader }"
    e = _engine(schema, ["document:d#reader@user:a"], revision=1)
    c = Client(e)
    c.SetHeadRevision(3)
    r = rel.MustFromTriple("document:d", "view", "user:b")
    ctx = consistency.Context(metadata={})
    object.__setattr__(ctx, "deadline", 0)
    ok, err = c.CheckOne(ctx, consistency.Full(), r)  # no retry: the error itself
    assert ok is False and isinstance(err, E.GckError) and err.code == E.GCK_E_REVISION
    assert c.CheckOne(None, consistency.MinLatency(), r) == (False, None)

    def watch():
        time.sleep(0.3)
        e.apply_updates_text(2, "")
        time.sleep(0.2)
        e.apply_updates_text(3, "CREATE document:d#reader@user:b")

    t = threading.Thread(target=watch)
    t0 = time.monotonic()
    t.start()
    assert c.CheckOne(None, consistency.Full(), r) == (True, None)  # retried until revision 3
    assert time.monotonic() - t0 >= 0.45
    t.join()
    # AtLeast behaves the same way
    t = threading.Thread(target=lambda: (time.sleep(0.2), e.apply_updates_text(4, "DELETE document:d#reader@user:b")))
    t.start()
    assert c.CheckOne(None, consistency.AtLeast("4"), r) == (False, None)
    t.join()
    e.close()


def test_snapshot_revision_passed_is_permanent():
    schema = "definition user {}\ndefinition document { relation reader: user }"
    e = _engine(schema, ["document:d#reader@user:a"], revision=5)
    c = Client(e)
    r = rel.MustFromTriple("document:d", "reader", "user:a")
    t0 = time.monotonic()
    ok, err = c.CheckOne(None, consistency.Snapshot("4"), r)  # no retry, no 15-minute backoff
    assert time.monotonic() - t0 < 1.0
    assert ok is False and isinstance(err, E.GckError) and err.code == E.GCK_E_REVISION_GONE
    assert c.CheckOne(None, consistency.Snapshot("5"), r) == (True, None)
    e.close()


def test_lookup_sees_expiration_between_calls():
    """two lookups on one snapshot at wall-clock time; a relationship that expires
    between them must disappear from the second."""
    schema = ("definition user {}\ndefinition document {\n relation reader: user with expiration\n"
              " permission view = reader\n}\nuse expiration")
    soon = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(time.time() + 2))
    e = _engine(schema, [f"document:a#reader@user:u[expiration:{soon}]", "document:b#reader@user:u"])
    rt, st = e.type_id("document"), e.type_id("user")
    view = e.relation_id(rt, "view")
    uid = int(e.intern(st, ["u"])[0])
    ids1, _ = e.lookup_resources(rt, view, st, E.ELLIPSIS, uid)
    time.sleep(3.2)  # past the expiration (whole seconds in the text form)
    ids2, _ = e.lookup_resources(rt, view, st, E.ELLIPSIS, uid)
    names1 = sorted(e.object_name(rt, int(i)) for i in ids1)
    names2 = sorted(e.object_name(rt, int(i)) for i in ids2)
    assert names1 == ["a", "b"] and names2 == ["b"], (names1, names2)
    e.close()


def test_pinned_host_buffers():
    """gck_host_alloc buffers: the batch is copied by DMA straight from / into them (no staging
    copy); results equal the pageable path and the oracle, also when stage B/C run."""
    schema, tuples, checks = gen.gdocs_deep(2)
    want = _want(schema, tuples, checks)
    for kw in ({}, {"bundle_budget": 2}):
        e = _engine(schema, tuples, workspaces=2, **kw)
        items = e.make_items([parse_check(c) for c in checks])
        p_items = e.host_array(len(items), E.ITEM_DTYPE)
        p_items[:] = items
        perm, err = e.host_array(len(items), np.uint8), e.host_array(len(items), np.int32)
        b = e.submit_into(p_items, perm, err, now_us=gen.NOW_US)
        b.wait()
        assert _got(perm, err) == want
        # pinned items, pageable results (and the other way round)
        perm2, err2 = np.zeros(len(items), np.uint8), np.zeros(len(items), np.int32)
        e.submit_into(p_items, perm2, err2, now_us=gen.NOW_US).wait()
        assert _got(perm2, err2) == want
        perm[:] = 0
        e.submit_into(items.copy(), perm, err, now_us=gen.NOW_US).wait()
        assert _got(perm, err) == want
        e.close()


@pytest.mark.parametrize("engine_streams", [False, True])
def test_compiled_submit_loop(engine_streams):
    """libgck_driver.so's loop (bench.py's timed region): 6 device batches, 3 in flight, on the
    caller's streams or the engine's (GCK_SUBMIT_ENGINE_STREAM); every result equals the oracle."""
    import torch
    schema, tuples, checks = gen.github(4)
    e = _engine(schema, tuples, workspaces=3)
    want = _want(schema, tuples, checks)
    items = e.make_items([parse_check(c) for c in checks])
    n = len(items)
    d_items = [torch.from_numpy(np.roll(items, k).view(np.uint8).copy()).cuda() for k in range(6)]
    outs = [(torch.zeros(n, dtype=torch.uint8, device="cuda"), torch.zeros(n, dtype=torch.int32, device="cuda"))
            for _ in range(6)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    torch.cuda.synchronize()
    secs = e.run_device_batches([d.data_ptr() for d in d_items], [p.data_ptr() for p, _ in outs],
                                [x.data_ptr() for _, x in outs], n, 3, [streams[k % 3].cuda_stream for k in range(6)],
                                engine_streams=engine_streams, now_us=gen.NOW_US)
    torch.cuda.synchronize()
    assert secs > 0
    for k, (perm, err) in enumerate(outs):
        rolled = (want[-k:] + want[:-k]) if k else want  # np.roll(items, k)[i] = items[i - k]
        assert _got(perm.cpu().numpy(), err.cpu().numpy()) == rolled, k
    e.close()


@pytest.mark.parametrize("family", ["nested", "gdocs"])
def test_engine_stream_results_read_right_after_wait(family):
    """A device batch on the engine's stream has no caller stream to order reads after: the
    results a caller reads on another stream the moment gck_check_wait returns — no
    synchronisation with the engine's stream — are the final ones (the AQL packet's release fence
    and completion signal, or k_publish after a HIP-launched join). 48 batches over poisoned
    buffers, 3 in flight."""
    import torch
    schema, tuples, checks = getattr(gen, family)(3)
    e = _engine(schema, tuples, workspaces=3)
    want = _want(schema, tuples, checks)
    items = e.make_items([parse_check(c) for c in checks])
    n = len(items)
    d_items = [torch.from_numpy(np.roll(items, k).view(np.uint8).copy()).cuda() for k in range(8)]
    reader = torch.cuda.Stream()
    for rnd in range(6):
        outs = [(torch.full((n,), 0xFF, dtype=torch.uint8, device="cuda"),
                 torch.full((n,), -7, dtype=torch.int32, device="cuda")) for _ in range(8)]
        torch.cuda.synchronize()
        pending, copies = [], {}
        for k in range(8):
            if len(pending) >= 3:
                j, b = pending.pop(0)
                b.wait()
                with torch.cuda.stream(reader):  # read at once, on a stream the engine never saw
                    copies[j] = (outs[j][0].clone(), outs[j][1].clone())
            pending.append((k, e.submit(d_items[k].data_ptr(), n, outs[k][0].data_ptr(), outs[k][1].data_ptr(),
                                        now_us=gen.NOW_US, device=True, engine_stream=True)))
        for j, b in pending:
            b.wait()
            with torch.cuda.stream(reader):
                copies[j] = (outs[j][0].clone(), outs[j][1].clone())
        reader.synchronize()
        for k in range(8):
            rolled = (want[-k:] + want[:-k]) if k else want
            assert _got(copies[k][0].cpu().numpy(), copies[k][1].cpu().numpy()) == rolled, (rnd, k)
    torch.cuda.synchronize()
    if family == "nested" and os.path.exists(os.path.join(os.path.dirname(E.__file__), "libgck_kernels.co")):
        # the closure join of these batches went into the engine's HSA queue (aql.inc)
        assert e.stats()["aql_batches"] > 0, e.stats()
    e.close()


def test_no_allocation_after_commit():
    """Every workspace exists once the snapshot is committed (engine.hip ensure_pool): the first
    batches after the commit — as many concurrent ones as the pool holds — allocate nothing, so
    no caller's latency includes creating a workspace. gck_device_bytes counts the snapshot plus
    every workspace's scratch."""
    schema, tuples, checks = gen.nested(2)
    e = _engine(schema, tuples, workspaces=4)
    want = _want(schema, tuples, checks)
    items = e.make_items([parse_check(c) for c in checks])
    before = e.device_bytes
    assert before > 4 * 64 << 20, before  # four workspaces' bundle scratch is in the count
    bs = [e.submit(items, now_us=gen.NOW_US) for _ in range(4)]  # the whole pool at once
    for b in bs:
        perm, err = b.wait()
        assert _got(perm, err) == want
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    assert _got(perm, err) == want
    assert e.device_bytes == before
    e.close()


def test_two_workspace_requests_never_deadlock():
    """A request above max_batch alternates over two workspaces, taken together
    (gck_api.cpp gck_check_bulk_ctx / acquire_ws_n): with one workspace it runs on that one, and
    four threads sending such requests to a pool of two all finish."""
    schema, tuples, checks = gen.gdocs(6)
    want = _want(schema, tuples, checks)
    reps = 12
    for ws, n_threads in ((1, 1), (1, 3), (2, 4)):
        e = _engine(schema, tuples, workspaces=ws, max_batch=256)
        items = e.make_items([parse_check(c) for c in checks] * reps)
        assert len(items) > 2 * 256
        errors, done = [], []

        def worker():
            try:
                for _ in range(3):
                    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
                    assert _got(perm, err) == want * reps
                done.append(1)
            except Exception as ex:  # noqa: BLE001
                errors.append(ex)

        threads = [threading.Thread(target=worker) for _ in range(n_threads)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=90)
        assert not errors, errors
        assert len(done) == n_threads, f"workspaces={ws}: {n_threads - len(done)} callers stuck"
        e.close()


def test_pinned_array_outlives_close():
    """host_array() memory stays valid after Engine.close() while an array views it (the engine is
    destroyed with its last pinned buffer)."""
    schema, tuples, checks = gen.nested(1)
    e = _engine(schema, tuples)
    a = e.host_array(1000, np.int32)
    a[:] = np.arange(1000)
    e.close()
    assert e._h is not None  # kept for `a`
    assert int(a.sum()) == 499500
    del a
    import gc
    gc.collect()
    assert e._h is None


_KNOB_PROBE = r"""
import json, sys
sys.path.insert(0, {root!r})
import numpy as np
from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item
schema, tuples, checks = gen.nested(4)
e = E.Engine(device=0, profile=True, workspaces=3)
e.load_schema(schema)
e.load_snapshot_text(1, "\n".join(tuples))
items = e.make_items([parse_check(c) for c in checks])
ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
import torch
n = len(items)
d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
ok = True
for _ in range(8):  # device batches on the engine's streams: the AQL path when it is on
    perm = torch.zeros(n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    e.submit(d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(), now_us=gen.NOW_US, device=True,
             engine_stream=True).wait()
    ok &= [(int(p), int(x)) for p, x in zip(perm.cpu().numpy(), err.cpu().numpy())] == want
st = e.stats()
print(json.dumps({{"ok": ok, "aql_batches": int(st["aql_batches"]), "bundle_ms": float(st["bundle_ms"]),
                  "launches": int(st["bundle_launches"])}}))
"""


def test_launch_path_knobs():
    """The engine's two launch-path knobs, each in a process of its own (read once):
    GCK_AQL=0 sends every join through HIP, GCK_AQL_TIMED=0 only the profiled (timed) ones;
    results equal the oracle's either way, and the profiled batches are timed. (The probe's batches
    leave checks to the bundles, so after the first one every join is chained and launched through
    HIP: the first batch, profiled, is the one the knobs move.)"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for knob in ["GCK_AQL=0", "GCK_AQL_TIMED=0", ""]:
        env = dict(os.environ)
        if knob:
            k, v = knob.split("=")
            env[k] = v
        r = subprocess.run([sys.executable, "-c", _KNOB_PROBE.format(root=root)], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, (knob, r.stderr[-3000:])
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["ok"], (knob, out)
        assert out["launches"] > 0 and out["bundle_ms"] > 0, (knob, out)
        outs[knob] = out["aql_batches"]
    assert outs["GCK_AQL=0"] == 0, outs
    if os.path.exists(os.path.join(os.path.dirname(E.__file__), "libgck_kernels.co")):
        assert outs[""] > outs["GCK_AQL_TIMED=0"], outs
