# debug: deferral counts on one random-graph family through the default bundle path
import sys
sys.path.insert(0, ".")
from tests import gen
from tests.test_gpu_parity import make_engine, device_results
fam, seed = sys.argv[1], int(sys.argv[2])
schema, tuples, checks = gen.FAMILIES[fam](seed)
e = make_engine(schema, tuples)
device_results(e, checks, now_us=gen.NOW_US)
st = e.stats()
print(fam, seed, {k: st[k] for k in ("deferred", "deferred_wide", "entries_expanded", "bidir_checks")})
