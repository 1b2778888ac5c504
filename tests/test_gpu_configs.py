"""Scale parity for BASELINE.json configs 2 (Google-Docs schema) and 3 (GitHub schema with
exclusion, intersection and all()): tests/synth_configs.py graphs at reduced scale, one batch
through several engine paths, bit-exact against the C oracle on the same CSR arrays."""
import numpy as np
import pytest
import torch

from gochugaru_amd.engine import Engine
from oracle import corc
from tests import synth_configs as S

pytestmark = pytest.mark.gpu

PATHS = {"bundle": {}, "wide": {"wide_only": True}, "giant": {"bundle_budget": 8}, "nobidir": {"bidir": False}}


def load(W, **kw):
    e = Engine(device=0, **kw)
    e.load_schema(W.schema)
    for t, n in W.counts.items():
        e.reserve_objects(W.t(t), n)
    e.begin_snapshot(1)
    keep = []
    for rel, st, sr, n_rows, off, nbr in W.csrs:
        off32 = off.to(torch.int32).contiguous()
        keep.append(off32)
        e.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    torch.cuda.synchronize()
    e.commit_snapshot()
    return e


@pytest.fixture(scope="module", params=[("gdocs", 0.2), ("github", 0.05)], ids=["config2-gdocs", "config3-github"])
def workload(request):
    name, scale = request.param
    W = S.CONFIGS[name](scale, device=torch.device("cuda", 0))
    items = S.checks(W, 16384, seed=11)
    prog, tab = W.oracle()
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    cp, ce, _ = corc.check(prog, tab, hi, threads=16)
    return W, items, cp, ce


@pytest.mark.parametrize("path", sorted(PATHS))
def test_config_parity(workload, path):
    W, items, cp, ce = workload
    e = load(W, **PATHS[path])
    n = items.shape[0]
    perm = torch.zeros(n, dtype=torch.uint8, device="cuda")
    err = torch.zeros(n, dtype=torch.int32, device="cuda")
    e.check_bulk_device(items.data_ptr(), n, perm.data_ptr(), err.data_ptr(),
                        stream=torch.cuda.current_stream().cuda_stream)
    gp, ge = perm.cpu().numpy(), err.cpu().numpy()
    bad = np.nonzero((gp != cp) | (ge != ce))[0]
    assert len(bad) == 0, [(int(i), int(gp[i]), int(cp[i]), int(ge[i]), int(ce[i])) for i in bad[:5]]
    assert (cp == 2).sum() > n // 20 and (cp == 1).sum() > n // 4  # both answers well represented
    e.close()
