"""Check-time caveat contexts at scale: the device walk meets (partial
caveat instance, context) pairs, the host evaluates only those (engine.hip caveat_passes) and
the batch runs again with their outcomes. Bit-exact against the oracles: the Python oracle on
small seeded graphs (dense and lazy evaluation, every path), the C oracle's threshold mode
(corc.check_quota, pinned to the Python oracle by tests/test_c_oracle.py) on a config-5 variant
with 32K per-relationship stored contexts x one context per request in a 64K batch."""
import numpy as np
import pytest
import torch

from tests.helpers import parse_check
from tests.test_c_oracle import QUOTA, quota_case, run_quota
from tests.test_gpu_parity import device_results, make_engine

pytestmark = pytest.mark.gpu

PATHS = [{}, {"wide_only": True}, {"bidir": False}, {"giant_stage": False, "bundle_budget": 4}]


@pytest.mark.parametrize("lazy", [False, True], ids=["dense", "lazy"])
@pytest.mark.parametrize("path", PATHS, ids=["default", "wide", "nobidir", "budget4"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_quota_caveats_match_oracle(seed, path, lazy):
    tuples, checks, used = quota_case(seed)
    want, _ = run_quota(tuples, checks, used)
    e = make_engine(QUOTA, tuples, lazy_caveats=lazy, **path)
    e.reset_stats()
    got = device_results(e, checks, contexts=[None if u is None else {"used": u} for u in used])
    bad = [(c, u, w, g) for c, u, w, g in zip(checks, used, want, got) if w != g]
    assert not bad, bad[:10]
    st = e.stats()
    if lazy:
        assert st["caveat_passes"] >= 1 and st["caveat_evals"] > 0
    else:
        assert st["caveat_passes"] == 0
    e.close()


@pytest.mark.parametrize("lazy", [False, True], ids=["dense", "lazy"])
@pytest.mark.parametrize("path", PATHS[:2], ids=["default", "wide"])
def test_caveat_eval_error_is_per_item(path, lazy):
    """A context that gives `used` a string fails the checks whose walk meets the caveat
    (GCK_ITEM_ERR_CAVEAT_EVAL) and no other check of the call."""
    tuples = ['doc:a#viewer@user:x[quota:{"limit":10}]', "doc:b#viewer@user:x", "doc:c#viewer@user:y",
              'doc:d#viewer@group:g#member[quota:{"limit":5}]', "group:g#member@user:x"]
    checks = ["doc:a#view@user:x", "doc:b#view@user:x", "doc:c#view@user:x", "doc:a#view@user:x",
              "doc:d#view@user:x", "doc:d#view@user:x", "doc:a#view@user:x"]
    used = ["many", "many", "many", 3, "lots", 4, None]
    want, _ = run_quota(tuples, checks, used)
    assert [w[1] for w in want] == [6, 0, 0, 0, 6, 0, 0]
    e = make_engine(QUOTA, tuples, lazy_caveats=lazy, **path)
    got = device_results(e, checks, contexts=[None if u is None else {"used": u} for u in used])
    assert got == want
    e.close()


@pytest.fixture(scope="module")
def quota_workload():
    from tests.synth_configs import Quota
    Q = Quota(scale=0.1, device="cuda")
    return Q


@pytest.mark.parametrize("path", [{}, {"wide_only": True}], ids=["default", "wide"])
def test_quota_variant_64k_contexts_vs_c_oracle(quota_workload, path):
    """Config-5 variant: 32K partial caveat instances (per-relationship limits) x 64K per-request
    contexts in one 64K batch (a dense table would be 2^31 pairs)."""
    from gochugaru_amd.engine import Engine
    Q = quota_workload
    eng = Engine(device=0, **path)
    eng.load_schema(Q.W.schema)
    for t, n in Q.W.counts.items():
        eng.reserve_objects(Q.W.t(t), n)
    eng.begin_snapshot(1)
    keep = []

    def loader(rel, st, sr, n_rows, off, nbr):
        off32 = off.to(torch.int32).contiguous()
        nbr32 = nbr.contiguous()
        keep.append((off32, nbr32))
        eng.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr32.data_ptr(), nbr32.numel(), device=True)
    Q.load(eng, loader)
    torch.cuda.synchronize()
    eng.commit_snapshot()
    assert len(set(Q.inst.tolist())) >= 16384
    items, used, texts = Q.checks(65536, seed=11)
    perm = torch.zeros(65536, dtype=torch.uint8, device="cuda")
    err = torch.zeros(65536, dtype=torch.int32, device="cuda")
    eng.reset_stats()
    eng.check_bulk_device(items.data_ptr(), 65536, perm.data_ptr(), err.data_ptr(), contexts=texts)
    torch.cuda.synchronize()
    st = eng.stats()
    hi = items.cpu().numpy().view(np.uint8).reshape(-1).view(
        np.dtype([("resource_type", "<u2"), ("permission", "<u2"), ("resource_id", "<u4"), ("subject_type", "<u2"),
                  ("subject_relation", "<u2"), ("subject_id", "<u4"), ("context_slot", "<u4")]))
    cp, ce = Q.expected(hi, used)
    gp, ge = perm.cpu().numpy(), err.cpu().numpy()
    bad = np.nonzero((cp != gp) | (ce != ge))[0]
    assert bad.size == 0, [(int(i), int(gp[i]), int(ge[i]), int(cp[i]), int(ce[i])) for i in bad[:10]]
    mix = {k: int((cp == v).sum()) for k, v in (("NO", 1), ("HAS", 2), ("COND", 3))}
    assert min(mix.values()) > 20, mix  # CONDITIONAL: a caveated path and no context (10 % of checks)
    print("quota variant:", mix, {k: st[k] for k in ("caveat_evals", "caveat_passes", "batches")})
    # lazily evaluated: a small fraction of the 32K x 64K pairs, in a few passes
    assert 0 < st["caveat_evals"] < 2_000_000 and 1 <= st["caveat_passes"] <= 8, st
    eng.close()


@pytest.mark.parametrize("lazy", [False, True], ids=["dense", "lazy"])
def test_malformed_context_fails_the_call(lazy):
    from gochugaru_amd import engine as E
    tuples = ['doc:a#viewer@user:x[quota:{"limit":10}]']
    e = make_engine(QUOTA, tuples, lazy_caveats=lazy)
    items = e.make_items([parse_check("doc:a#view@user:x")])
    items[0]["context_slot"] = 1
    with pytest.raises(E.GckError) as ei:
        e.check_bulk(items, contexts=['{"used": 3'])
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    perm, err = e.check_bulk(items, contexts=['{"used": 3}'])  # the engine is still usable
    assert (int(perm[0]), int(err[0])) == (2, 0)
    e.close()
