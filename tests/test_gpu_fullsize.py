"""Full-size parity for every BASELINE.json configuration (VERDICT r1 "next" item 2): the exact
sizes the bench runs — config 4 at 1e9 tuples, config 2 at 1e7, config 3 at 1e8, config 5 at 1e7
with three Watch batches — one 65,536-check batch each (rotated seeds, deep positives), bit-exact
against the C oracle (oracle/check_oracle.c) on the same CSR arrays, through the default engine
path and a second path. Each test builds its graph on the GPU in seconds; the oracle checks a
batch in well under a minute on the box's host cores."""
import os

import numpy as np
import pytest
import torch

from oracle import corc
from tests import synth
from tests import synth_configs as S
from tests.test_gpu_configs import load as load_config
from tests.test_gpu_mixed import load as load_mixed
from tests.test_gpu_mixed import run as run_mixed
from tests.test_gpu_scale import load_engine, run
from tests.test_synth import _oracle

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
N = 65536


def _diff(gp, ge, cp, ce):
    bad = np.nonzero((gp != cp) | (ge != ce))[0]
    return [(int(i), int(gp[i]), int(cp[i]), int(ge[i]), int(ce[i])) for i in bad[:6]], len(bad)


def test_config4_1e9_full_batch():
    G = synth.build(1e9, device="cuda")
    items = synth.checks(G, N, seed=4242)  # positives descend up to 24 group layers
    e = load_engine(G)
    assert e.tuple_count == G.n_tuples and G.n_tuples > 9e8
    gp, ge = run(e, items)
    st = e.stats()
    footprint = e.device_bytes
    e.close()
    # the wave-bundle search over the same batch (with the membership index a default engine does
    # not build above 4 GB: engine.hip want_mhash)
    e2 = load_engine(G, closure=False, big_membership_hash=True)
    gp2, ge2 = run(e2, items)
    e2.close()
    _, prog, tab = _oracle(G)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    cp, ce, _ = corc.check(prog, tab, hi, threads=THREADS)
    first, n_bad = _diff(gp, ge, cp, ce)
    assert n_bad == 0, first
    assert np.array_equal(gp2, gp) and np.array_equal(ge2, ge)
    assert st["closure_checks"] == N  # every check answered by the closure join
    assert st["slot_checks"] > N // 2  # most from the user / resource slots alone
    assert 0.3 < np.mean(cp == 2) < 0.7
    # the snapshot without the 17 GB membership index of group#member@user: <= 40 B per tuple
    print(f"config 4 footprint: {footprint / 1e9:.1f} GB, {footprint / G.n_tuples:.1f} B per tuple")
    assert footprint <= 40 * G.n_tuples, footprint


def test_config4_1e9_partitioned_rccl_one_rank():
    """Config 4 in partitioned mode (BASELINE config 4's "graph partitioned by resource ID") at
    1e9 tuples through gck_part_check — the partitioned label join with its RCCL exchange, then
    the level loop for what it leaves — on a one-rank communicator (the test box has one GPU):
    one 64K batch bit-exact against the C oracle, every check decided by the label join."""
    from gochugaru_amd.engine import Engine
    from gochugaru_amd.partition import RcclPartitionedChecker
    G = synth.build(1e9, device="cuda")
    items = synth.checks(G, N, seed=4243)
    e = Engine(device=0, max_batch=N)
    e.set_partition(0, 1)
    e.load_schema(synth.SCHEMA)
    e.reserve_objects(synth.T_USER, G.n_users)
    e.reserve_objects(synth.T_GROUP, G.n_groups)
    e.reserve_objects(synth.T_DOC, G.n_docs)
    e.begin_snapshot(1)
    keep = []
    for rel, st, sr, n_rows, off, nbr in G.csrs():
        off32 = off.to(torch.int32).contiguous()
        keep.append(off32)
        e.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    torch.cuda.synchronize()
    e.commit_snapshot()
    pc = RcclPartitionedChecker(e)
    e.reset_stats()
    perm, err = pc.check(items, N)
    gp, ge = perm.cpu().numpy(), err.cpu().numpy()
    st = e.stats()
    e.close()
    _, prog, tab = _oracle(G)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    cp, ce, _ = corc.check(prog, tab, hi, threads=THREADS)
    first, n_bad = _diff(gp, ge, cp, ce)
    assert n_bad == 0, first
    assert st["label_checks"] == N, st["label_checks"]


@pytest.mark.parametrize("name,scale", [("gdocs", 1.0), ("github", 1.0)], ids=["config2-1e7", "config3-1e8"])
def test_config2_config3_full_batch(name, scale):
    W = S.CONFIGS[name](scale, device=torch.device("cuda", 0))
    items = S.checks(W, N, seed=4243)
    prog, tab = W.oracle()
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    cp, ce, _ = corc.check(prog, tab, hi, threads=THREADS)
    for kw in ({}, {"wide_only": True}):
        e = load_config(W, **kw)
        gp, ge = run(e, items)
        e.close()
        first, n_bad = _diff(gp, ge, cp, ce)
        assert n_bad == 0, (kw, first)
    assert (cp == 2).sum() > N // 20 and (cp == 1).sum() > N // 4


def test_config5_full_with_three_watch_batches():
    M = S.Mixed(1.0, device=torch.device("cuda", 0))
    e, cav = load_mixed(M)
    items = M.checks(N, seed=4244)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    n_tuples = M.W.n_tuples
    seen = {1: 0, 2: 0, 3: 0}
    for step in range(4):
        if step:
            e.apply_updates(1 + step, M.churn(n_tuples // 1000, cav))  # 0.1 % churn, as the bench
        gp, ge = run_mixed(e, items)
        cp, ce = M.expected(hi, threads=THREADS)
        first, n_bad = _diff(gp, ge, cp, ce)
        assert n_bad == 0, (step, first)
        for k in seen:
            seen[k] += int((gp == k).sum())
    assert all(v > 0 for v in seen.values()), seen
    e.close()
