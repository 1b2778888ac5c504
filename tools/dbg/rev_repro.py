"""Variants of test_evaluated_revision_across_a_watch_publication (one process per variant)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from gochugaru_amd import engine as E  # noqa: E402
from tests import gen  # noqa: E402
from tests.helpers import parse_check  # noqa: E402

variant = sys.argv[1]
kw = {}
if variant == "nolabels":
    kw["labels"] = False
if variant == "noclosure":
    kw["closure"] = False
e = E.Engine(device=0, **kw)
e.load_schema(gen.GDOCS)
_, tuples, _ = gen.gdocs(7)
e.load_snapshot_text(1, "\n".join(tuples))
cands = [f"doc:d{d}#view@user:u{u}" for d in range(5) for u in range(40)]
perm, _ = e.check_bulk(e.make_items([parse_check(c) for c in cands]), now_us=gen.NOW_US)
c = cands[int(np.flatnonzero(perm == E.PERM_NO)[0])]
d, u = c.split("#")[0], c.split("@")[1]
items = e.make_items([parse_check(c)])
if variant != "noinflight":
    b = e.submit(items)
e.apply_updates_text(2, f"CREATE {d}#viewer@{u}")
if variant != "noinflight":
    p1, _ = b.wait()
st0 = e.stats()
perm, err, rev = e.check_bulk_at(items)
st = e.stats()
delta = {k: st[k] - st0[k] for k in ("label_checks", "closure_checks", "slot_checks", "queries", "batches") if k in st}
print(variant, c, "rev", rev, "perm", int(perm[0]), "err", int(err[0]), delta, flush=True)
perm2, err2 = e.check_bulk(e.make_items([parse_check(c)] * 40), now_us=gen.NOW_US)
print(variant, "x40", perm2.tolist()[:4], flush=True)
e.close()
