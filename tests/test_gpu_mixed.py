"""BASELINE.json config 5 at reduced scale: caveated tuples (10 % of the folder / doc viewer and
editor user tuples ``with only_on_tuesday``), check-time contexts (tuesday / monday / none) and
Watch churn at a moving revision (CREATE / TOUCH / DELETE, TOUCH toggling the caveat). After
every update batch the engine's answers are compared bit-exactly with the C oracle over the
rebuilt snapshot (tests/synth_configs.py Mixed.expected)."""
import numpy as np
import pytest
import torch

from gochugaru_amd.engine import Engine
from oracle import corc
from tests import synth_configs as S

pytestmark = pytest.mark.gpu


def load(M, **kw):
    e = Engine(device=0, **kw)
    e.load_schema(M.W.schema)
    for t, n in M.W.counts.items():
        e.reserve_objects(M.W.t(t), n)
    e.begin_snapshot(1)
    cav = e.add_caveat_instance("only_on_tuesday", "")
    keep = []

    def loader(rid, st, sr, n_rows, off, nbr):
        off32 = off.to(torch.int32).contiguous()
        nbr32 = nbr.contiguous()
        keep.append((off32, nbr32))
        e.load_csr(rid, st, sr, n_rows, off32.data_ptr(), nbr32.data_ptr(), nbr32.numel(), device=True)

    M.load(e, loader, cav)
    torch.cuda.synchronize()
    e.commit_snapshot()
    return e, cav


def run(e, items):
    n = items.shape[0]
    perm = torch.zeros(n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(n, dtype=torch.int32, device="cuda")
    e.check_bulk_device(items.data_ptr(), n, perm.data_ptr(), err.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream, contexts=S.CONTEXTS)
    return perm.cpu().numpy(), err.cpu().numpy()


@pytest.mark.parametrize("path", ["bundle", "wide"])
def test_mixed_caveats_and_churn(path):
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M, **({"wide_only": True} if path == "wide" else {}))
    items = M.checks(16384, seed=9)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    n_tuples = M.W.n_tuples
    seen = {1: 0, 2: 0, 3: 0}
    for step in range(4):
        if step:
            ups = M.churn(n_tuples // 100, cav)
            e.apply_updates(1 + step, ups)
            assert e.revision == 1 + step
        gp, ge = run(e, items)
        cp, ce = M.expected(hi)
        bad = np.nonzero((gp != cp) | (ge != ce))[0]
        assert len(bad) == 0, (step, [(int(i), int(hi[i]["context_slot"]), int(gp[i]), int(cp[i])) for i in bad[:6]])
        for k in seen:
            seen[k] += int((gp == k).sum())
    assert all(v > 0 for v in seen.values()), seen  # NO, HAS and CONDITIONAL all occur
    e.close()


def test_label_tables_hold_under_a_long_watch_stream():
    """BASELINE config 5's Watch stream (client/client.go:370-413 is unbounded) at reduced scale:
    200 batches of 0.1 % of the tuples each (CREATE / TOUCH / DELETE of folder and document
    viewers and editors, TOUCH toggling the caveat). The label tables are kept throughout: a
    subject whose grants changed is still answered by the join unless a changed object is the
    resource or one of its folders (labels.inc round 2, the arrow forest). Bit-exact against the
    C oracle after 1, 50 and 200 batches, with at least 95 % of the checks through the join at
    the end."""
    M = S.Mixed(0.05, device=torch.device("cuda", 0))
    e, cav = load(M)
    n = 16384
    items = M.checks(n, seed=12)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    frac = {}
    for step in range(1, 201):
        e.apply_updates(1 + step, M.churn(max(1, M.W.n_tuples // 1000), cav))
        if step in (1, 50, 200):
            e.reset_stats()
            gp, ge = run(e, items)
            st = e.stats()
            cp, ce = M.expected(hi)
            bad = np.nonzero((gp != cp) | (ge != ce))[0]
            assert len(bad) == 0, (step, [(int(i), int(gp[i]), int(cp[i])) for i in bad[:6]])
            frac[step] = st["label_checks"] / n
    print("label-join share after 1 / 50 / 200 batches:", frac)
    assert frac[200] >= 0.95, frac
    e.close()
