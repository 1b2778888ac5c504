"""Debug helper: run one check through a 1-check bundle with GCK_DEBUG_BUNDLE=1."""
import sys
sys.path.insert(0, ".")
from tests import gen
from tests.test_gpu_parity import device_results, make_engine
schema, tuples, checks = gen.caveated(1)
c = ["doc:d32#strict@user:u5"]
e = make_engine(schema, tuples, bundle_checks=1)
print(device_results(e, c, now_us=gen.NOW_US))
