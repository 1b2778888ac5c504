"""ShardedEngine on the GPU: replicas on one device (the box has one GPU; an 8-GPU node runs one
per device) answer one request — sliced, submitted without waiting, concatenated in request
order — exactly as a single engine and the oracle do, also across Watch batches."""
import numpy as np
import pytest

from gochugaru_amd import engine as E
from gochugaru_amd.sharded import ShardedEngine
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("replicas", [2, 3])
def test_sharded_equals_single_engine_and_oracle(replicas):
    schema, tuples, checks = gen.gdocs(4)
    checks = checks * 40  # 16,000 checks: several max_batch chunks per slice below
    se = ShardedEngine([0] * replicas, max_batch=2048)
    se.load_schema(schema)
    se.load_snapshot_text(1, "\n".join(tuples))
    items = se.make_items([parse_check(c) for c in checks])
    perm, err = se.check_bulk(items, now_us=gen.NOW_US)
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks[:400]]
    got = [(int(p), int(x)) for p, x in zip(perm, err)]
    assert all(got[i] == want[i % 400] for i in range(len(got)))
    one = E.Engine()
    one.load_schema(schema)
    one.load_snapshot_text(1, "\n".join(tuples))
    p1, e1 = one.check_bulk(items, now_us=gen.NOW_US)
    assert np.array_equal(p1, perm) and np.array_equal(e1, err)
    # a Watch batch reaches every replica
    gone = [t for t in tuples if "#viewer@" in t][:10]
    se.apply_updates_text(2, "\n".join("DELETE " + t for t in gone))
    one.apply_updates_text(2, "\n".join("DELETE " + t for t in gone))
    assert se.revision == 2
    perm2, err2 = se.check_bulk(items, now_us=gen.NOW_US)
    p12, e12 = one.check_bulk(items, now_us=gen.NOW_US)
    assert np.array_equal(p12, perm2) and np.array_equal(e12, err2)
    one.close()
    se.close()


def test_sharded_bounds_batches_in_flight():
    """A slice of more chunks than a replica's workspace pool: the sharded engine waits for a
    replica's oldest batch before its next submit (never more outstanding batches than
    workspaces, include/gck.h), so the request completes; max_batch=0 means the default."""
    schema, tuples, checks = gen.gdocs(4)
    checks = checks * 30
    se = ShardedEngine([0, 0], max_batch=256, workspaces=2)  # 6,000 checks per slice = 24 chunks
    se.load_schema(schema)
    se.load_snapshot_text(1, "\n".join(tuples))
    items = se.make_items([parse_check(c) for c in checks])
    perm, err = se.check_bulk(items, now_us=gen.NOW_US)
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks[:400]]
    assert all((int(perm[i]), int(err[i])) == want[i % 400] for i in range(len(checks)))
    se.close()
    se0 = ShardedEngine([0], max_batch=0)
    assert se0.max_batch == 65536
    se0.close()
