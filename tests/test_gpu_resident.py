"""The resident closure join (gochugaru_amd/csrc/resident.inc, GCK_FLAG_RESIDENT) on the GPU.

One long-running launch per engine takes 128-check chunks of the requests the host posts, so a
small request (a 64K request sharded over 8 GPUs leaves 8,192 checks per GPU) costs no dispatch of
its own. Bar: every request's results equal the oracle's bit-exactly whatever its size (chunk
edges, partial waves), with many requests in flight, over host (zero-copy) and device buffers and
the uniform format, across Watch publications (the launch is sealed and a new one started) and idle
gaps (the keeper seals an idle launch; the next request starts another); and the batches really
went through the resident launch (resident_batches)."""
import time

import numpy as np
import pytest
import torch

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu
NOW_US = gen.NOW_US


def _setup(seed=3, **kw):
    schema, tuples, _ = gen.nested(seed, n_users=600, n_groups=240, layers=8, n_docs=300)
    e = E.Engine(device=0, resident=True, workspaces=8, **kw)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    return e, schema, tuples


def _random_checks(rng, n, n_docs=300, n_users=600):
    # (names the snapshot holds: a request with unknown names leaves its checks to the bundles —
    # 2-3 % of 8,192 here — and a batch leaving 32 or more has the next 16 chained behind their joins
    # on a HIP stream, engine.hip kChainLeftovers, which is not the resident launch)
    return [f"doc:d{rng.integers(0, n_docs)}#view@user:u{rng.integers(0, n_users)}" for _ in range(n)]


def _want(schema, tuples, checks):
    ck = oracle_for(schema, tuples, now=NOW_US / 1e6)
    return [ck.check(to_oracle_item(parse_check(c))) for c in checks]


@pytest.mark.parametrize("sizes", [[1, 31, 32, 33, 127, 129, 255, 257], [4096, 8192, 1000, 8191, 64]])
def test_resident_sizes_in_flight(sizes):
    """Requests of every size at chunk edges, all in flight at once (device buffers on the
    engine's streams, then host buffers zero-copy), each bit-exact."""
    e, schema, tuples = _setup()
    rng = np.random.default_rng(len(sizes))
    reqs = [_random_checks(rng, n) for n in sizes]
    wants = [_want(schema, tuples, r) for r in reqs]
    e.reset_stats()
    items = [torch.from_numpy(e.make_items([parse_check(c) for c in r]).view(np.uint8).copy()).cuda() for r in reqs]
    outs = [(torch.zeros(len(r), dtype=torch.uint8, device="cuda"), torch.zeros(len(r), dtype=torch.int32, device="cuda"))
            for r in reqs]
    torch.cuda.synchronize()
    bs = [e.submit(it.data_ptr(), len(r), o[0].data_ptr(), o[1].data_ptr(), device=True, engine_stream=True, now_us=NOW_US)
          for it, r, o in zip(items, reqs, outs)]
    for b in bs:
        b.wait()
    for r, o, w in zip(reqs, outs, wants):
        got = list(zip(o[0].cpu().tolist(), o[1].cpu().tolist()))
        assert got == [tuple(x) for x in w]
    st = e.stats()
    assert st["resident_batches"] == len(sizes), st
    # host buffers (zero-copy joins): the same requests
    bs = [e.submit(e.make_items([parse_check(c) for c in r]), now_us=NOW_US) for r in reqs]
    for b, w in zip(bs, wants):
        perm, err = b.wait()
        assert list(zip(perm.tolist(), err.tolist())) == [tuple(x) for x in w]
    e.close()


def test_resident_many_small_requests_and_uniform():
    """400 requests of 8,192 checks (rotated over 16 item arrays), 8 in flight through the compiled
    loop on the engine's streams, then uniform requests: every result equal to the same requests
    checked one at a time without the resident join."""
    e, schema, tuples = _setup(seed=5)
    ref = E.Engine(device=0)
    ref.load_schema(schema)
    ref.load_snapshot_text(1, "\n".join(tuples))
    rng = np.random.default_rng(7)
    n = 8192
    arrays = [e.make_items([parse_check(c) for c in _random_checks(rng, n)]) for _ in range(16)]
    want = [ref.check_bulk(a, now_us=NOW_US) for a in arrays]
    d_items = [torch.from_numpy(a.view(np.uint8).copy()).cuda() for a in arrays]
    k = 400
    perms = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    errs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(k)]
    torch.cuda.synchronize()
    e.reset_stats()
    e.run_device_batches([d_items[j % 16].data_ptr() for j in range(k)], [p.data_ptr() for p in perms],
                         [x.data_ptr() for x in errs], n, 8, [0] * 8, engine_streams=True, now_us=NOW_US)
    torch.cuda.synchronize()
    for j in range(k):
        assert (perms[j].cpu().numpy() == want[j % 16][0]).all(), j
        assert (errs[j].cpu().numpy() == want[j % 16][1]).all(), j
    assert e.stats()["resident_batches"] == k
    t_doc, t_user = e.type_id("doc"), e.type_id("user")
    hdr = (t_doc, e.relation_id(t_doc, "view"), t_user, E.ELLIPSIS)
    for a, (wp, we) in zip(arrays[:4], want[:4]):
        pairs = np.stack([a["resource_id"], a["subject_id"]], axis=1).astype(np.uint32)
        words, ue, _ = e.check_uniform(hdr, pairs, now_us=NOW_US)
        assert (E.unpack_results(words, n) == np.where(we != 0, 0, wp)).all()
        assert len(ue) == int((we != 0).sum())
    e.close()
    ref.close()


def test_resident_across_watch_and_idle():
    """A Watch publication seals the launch (its table and slots change) and the next request
    starts a new one; an idle gap longer than the keeper's seal does the same; results follow the
    updates bit-exactly; closing the engine with a launch running returns."""
    e, schema, tuples = _setup(seed=8)
    rng = np.random.default_rng(11)
    store = {t.split("@")[0] + "@" + t.split("@")[1]: t for t in tuples}
    checks = _random_checks(rng, 3000)
    for rnd in range(4):
        got = [(int(p), int(x)) for p, x in zip(*e.check_bulk(e.make_items([parse_check(c) for c in checks]), now_us=NOW_US))]
        assert got == [tuple(x) for x in _want(schema, list(store.values()), checks)], rnd
        ups = []
        for _ in range(30):
            g, u = rng.integers(0, 240), rng.integers(0, 600)
            line = f"group:g{g}#member@user:u{u}"
            op = "DELETE" if rng.random() < 0.3 else "CREATE"
            ups.append((op, line))
        for _ in range(5):
            d, g = rng.integers(0, 300), rng.integers(0, 60)
            ups.append(("CREATE", f"doc:d{d}#viewer@group:g{g}#member"))
        e.apply_updates_text(2 + rnd, "\n".join(f"{op} {l}" for op, l in ups))
        for op, l in ups:
            if op == "DELETE":
                store.pop(l, None)
            else:
                store[l] = l
        if rnd == 1:
            time.sleep(0.1)  # idle: the keeper seals the launch
    e.reset_stats()
    got = [(int(p), int(x)) for p, x in zip(*e.check_bulk(e.make_items([parse_check(c) for c in checks]), now_us=NOW_US))]
    assert got == [tuple(x) for x in _want(schema, list(store.values()), checks)]
    assert e.stats()["resident_batches"] > 0
    e.close()
