"""Host-buffer batches (BASELINE.md:40-41's step: items H2D, kernels, results D2H): the zero-copy
path, where the join reads the items in place from pinned or staged host memory and writes the
results back across PCIe, and its request checks. A host item whose context_slot exceeds the
call's contexts fails the request (include/gck.h gck_check_bulk_ctx); the join of a zero-copy batch
finds it on the device, the other paths on the host — the same error either way."""
import numpy as np
import pytest

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu

FAMILIES = {"nested": gen.nested, "gdocs": gen.gdocs, "github": gen.github}


def _setup(family, **kw):
    schema, tuples, checks = FAMILIES[family](3)
    e = E.Engine(**kw)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    return e, e.make_items([parse_check(c) for c in checks]), want


def _pinned(e, items):
    a = e.host_array(len(items), E.ITEM_DTYPE)
    a[:] = items
    return a, e.host_array(len(items), np.uint8), e.host_array(len(items), np.int32)


@pytest.mark.parametrize("family", sorted(FAMILIES))
@pytest.mark.parametrize("zero_copy", [True, False], ids=["zero-copy", "dma"])
def test_context_slot_beyond_contexts_fails_the_request(family, zero_copy):
    # (a profiled engine moves host batches by DMA through its workspace buffers: the host check)
    e, items, want = _setup(family, profile=not zero_copy)
    bad_at = min(37, len(items) - 1)
    for n_ctx, slot in ((0, 1), (1, 2)):
        bad = items.copy()
        bad[bad_at]["context_slot"] = slot
        bad[-1]["context_slot"] = slot + 5  # (a later offender: the first one is reported)
        contexts = ['{"x": 1}'] * n_ctx
        with pytest.raises(E.GckError) as ei:  # pageable buffers, synchronous
            e.check_bulk(bad, now_us=gen.NOW_US, contexts=contexts or None)
        assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
        assert f"item {bad_at}: context_slot {slot} beyond the {n_ctx} contexts" in str(ei.value), str(ei.value)
        pi, pp, pe = _pinned(e, bad)  # pinned buffers, asynchronous: the wait reports it
        with pytest.raises(E.GckError) as ei:
            e.submit_into(pi, pp, pe, now_us=gen.NOW_US, contexts=contexts or None).wait()
        assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
        assert f"item {bad_at}:" in str(ei.value), str(ei.value)
    # the engine is still usable, and the good batch answers as the oracle on either buffer kind
    perm, err = e.check_bulk(items, now_us=gen.NOW_US)
    assert [(int(p), int(x)) for p, x in zip(perm, err)] == want
    pi, pp, pe = _pinned(e, items)
    e.submit_into(pi, pp, pe, now_us=gen.NOW_US).wait()
    assert [(int(p), int(x)) for p, x in zip(pp, pe)] == want
    e.close()


@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_pipelined_host_batches_match_the_oracle(family):
    """8 host batches in flight over pinned buffers through the compiled loop (what bench.py times
    as `value`): every batch's results equal the oracle, and the joins ran zero-copy."""
    e, items, want = _setup(family, workspaces=8)
    rng = np.random.default_rng(11)
    orders = [rng.permutation(len(items)) for _ in range(24)]
    bufs = [_pinned(e, items[o]) for o in orders]
    e.reset_stats()
    run = e.prepare_batches([b[0].ctypes.data for b in bufs], [b[1].ctypes.data for b in bufs],
                            [b[2].ctypes.data for b in bufs], len(items), 8, host=True, now_us=gen.NOW_US)
    run.run()
    for o, (_, pp, pe) in zip(orders, bufs):
        assert [(int(p), int(x)) for p, x in zip(pp, pe)] == [want[j] for j in o]
    st = e.stats()
    # (a join that left checks makes the next batches chain the bundles behind it through HIP)
    assert st["aql_batches"] > 0, st["aql_batches"]
    e.close()
