"""The scale generator (tests/synth.py) on CPU at toy size: CSR invariants and that the
'positive' half of the check batch is positive under the C oracle."""
import numpy as np

from oracle import corc
from oracle import spicedb_ref as ref
from tests import synth


def _oracle(G):
    H = synth.host_arrays(G)
    ids = corc.Ids(ref.Schema(synth.SCHEMA))
    assert ids.type_id == {"user": synth.T_USER, "group": synth.T_GROUP, "doc": synth.T_DOC}
    assert ids.rel_id[("doc", "view")] == synth.R_VIEW
    idx = {(synth.R_MEMBER, synth.T_USER, synth.ELLIPSIS, False): 0,
           (synth.R_MEMBER, synth.T_GROUP, synth.R_MEMBER, False): 1,
           (synth.R_VIEWER, synth.T_GROUP, synth.R_MEMBER, False): 2}
    prog = corc.encode_program(ids, idx)
    tab = corc.make_csr_table([(H["mem_user_off"], H["mem_user_nbr"], None, None, G.n_groups),
                               (H["mem_group_off"], H["mem_group_nbr"], None, None, G.n_groups),
                               (H["viewer_off"], H["viewer_nbr"], None, None, G.n_docs)])
    return H, prog, tab


def test_synth_invariants_and_positive_half():
    G = synth.build(1e6, device="cpu")
    H, prog, tab = _oracle(G)
    for off_name, nbr_name, n_rows, bound in [("mem_user_off", "mem_user_nbr", G.n_groups, G.n_users),
                                              ("mem_group_off", "mem_group_nbr", G.n_groups, G.n_groups),
                                              ("viewer_off", "viewer_nbr", G.n_docs, G.n_groups)]:
        off = H[off_name].astype(np.int64)
        nbr = H[nbr_name].astype(np.int64)
        assert len(off) == n_rows + 1 and off[0] == 0 and off[-1] == len(nbr)
        assert np.all(np.diff(off) >= 0) and nbr.max() < bound
        for r in np.random.default_rng(0).integers(0, n_rows, 200):
            row = nbr[off[r]:off[r + 1]]
            assert np.all(np.diff(row) > 0)
    # group edges only go one layer down (acyclic)
    ls = G.layer_start.numpy()
    goff, gnbr = H["mem_group_off"].astype(np.int64), H["mem_group_nbr"].astype(np.int64)
    parent = np.repeat(np.arange(G.n_groups), np.diff(goff))
    assert np.all(np.searchsorted(ls, gnbr, side="right") == np.searchsorted(ls, parent, side="right") + 1)
    items = synth.checks(G, 2048, seed=5, positive_frac=1.0).numpy().view(corc.ITEM_DTYPE).reshape(-1)
    perm, err, _ = corc.check(prog, tab, items, threads=4)
    assert np.all(err == 0) and np.all(perm == 2)  # positive by construction
    items = synth.checks(G, 2048, seed=6, positive_frac=0.0).numpy().view(corc.ITEM_DTYPE).reshape(-1)
    perm, err, _ = corc.check(prog, tab, items, threads=4)
    assert np.mean(perm == 1) > 0.8
