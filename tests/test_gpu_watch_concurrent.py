"""A Watch batch no longer stops the checks (client/client.go:370-413 UpdatesSinceRevision beside
client/client.go:238-284 Check; delta.inc device_apply_build / device_apply_publish): the next
snapshot is merged and derived while the engine lock is held shared, and the exclusive lock is
taken only to finish the batches in flight, patch the membership indexes and swap the snapshot.
A checker thread keeps checking a 4K batch in a loop while a 0.1 % batch touching the group
hierarchy applies to a 1e8-tuple config-4 graph: no check waits longer than 50 ms, checks complete
during the apply, and every one of them answers for one revision — the old one before the swap,
the new one after it — bit-exact against the C oracle of that revision."""
import os
import threading
import time

import numpy as np
import pytest
import torch

from oracle import corc
from tests import synth
from tests.test_gpu_scale import load_engine

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)


@pytest.mark.timeout(900)
def test_checks_run_while_a_hierarchy_batch_applies():
    G = synth.build(1e8, device="cuda")
    C = synth.NestedChurn(G, seed=7)
    items = synth.checks(G, 4096, seed=31)
    hi = items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1)
    prog, tab = C.oracle()
    want_old = corc.check(prog, tab, hi, threads=THREADS)[:2]
    ups = C.batch(max(1000, int(G.n_tuples * 0.001)), cycle=False)  # memberships, nesting, viewers
    prog, tab = C.oracle()
    want_new = corc.check(prog, tab, hi, threads=THREADS)[:2]
    assert (want_old[0] != want_new[0]).any(), "the batch must change some answer"
    e = load_engine(G)
    stop = threading.Event()
    log = []  # (start, seconds, matches old, matches new)
    errors = []

    def checker():
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            perm = torch.zeros(len(hi), dtype=torch.uint8, device="cuda")
            err = torch.zeros(len(hi), dtype=torch.int32, device="cuda")
            while not stop.is_set():
                t0 = time.perf_counter()
                e.check_bulk_device(items.data_ptr(), len(hi), perm.data_ptr(), err.data_ptr(), stream=s.cuda_stream)
                dt = time.perf_counter() - t0
                p, x = perm.cpu().numpy(), err.cpu().numpy()
                log.append((t0, dt, bool((p == want_old[0]).all() and (x == want_old[1]).all()),
                            bool((p == want_new[0]).all() and (x == want_new[1]).all())))
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(repr(ex))

    th = threading.Thread(target=checker)
    th.start()
    time.sleep(1.0)
    t_a = time.perf_counter()
    e.apply_updates(2, ups)
    t_b = time.perf_counter()
    time.sleep(0.5)
    stop.set()
    th.join()
    e.close()
    assert not errors, errors
    during = [r for r in log if t_a <= r[0] <= t_b]
    worst = max(r[1] for r in log)
    print({"apply_s": round(t_b - t_a, 3), "checks": len(log), "during_apply": len(during),
           "worst_check_ms": round(worst * 1e3, 2),
           "median_check_ms": round(float(np.median([r[1] for r in log])) * 1e3, 3)})
    assert all(r[2] or r[3] for r in log), "a check answered for neither revision"
    assert all(r[2] for r in log if r[0] + r[1] < t_a) and all(r[3] for r in log if r[0] > t_b)
    assert len(during) >= 10, "checks must keep completing while the batch applies"
    assert worst < 0.05, f"a check waited {worst * 1e3:.1f} ms"
