"""Which check after a Watch publication answers from stale data (one process per variant)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from gochugaru_amd import engine as E  # noqa: E402
from tests import gen  # noqa: E402
from tests.helpers import parse_check  # noqa: E402

variant = sys.argv[1]
kw = {"membership_hash": False} if variant == "nomhash" else {}
e = E.Engine(device=0, **kw)
e.load_schema(gen.GDOCS)
_, tuples, _ = gen.gdocs(7)
e.load_snapshot_text(1, "\n".join(tuples))
cands = [f"doc:d{d}#view@user:u{u}" for d in range(5) for u in range(40)]
perm, _ = e.check_bulk(e.make_items([parse_check(c) for c in cands]), now_us=gen.NOW_US)
c = cands[int(np.flatnonzero(perm == E.PERM_NO)[0])]
d, u = c.split("#")[0], c.split("@")[1]
one = e.make_items([parse_check(c)])
forty = e.make_items([parse_check(c)] * 40)
e.apply_updates_text(2, f"CREATE {d}#viewer@{u}")
out = []
seq = {"x40first": ["40", "1", "1"], "single2": ["1", "1", "40"], "sync": ["S", "1", "1"], "nomhash": ["1", "1", "40"],
       "sleep": ["Z", "1", "1"]}[variant]
for s in seq:
    if s == "S":
        torch.cuda.synchronize()
        continue
    if s == "Z":
        import time
        time.sleep(0.5)
        continue
    p, _ = e.check_bulk(one if s == "1" else forty, now_us=gen.NOW_US)
    out.append((s, p.tolist()[:3]))
print(variant, c, out, flush=True)
e.close()
