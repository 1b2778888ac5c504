"""bench.py's multi-rank launcher on CPU (no HIP): `bench.py --gpus N` without WORLD_SIZE starts
N rank processes with the torch.distributed environment and passes rank 0's JSON line through;
it refuses (non-zero status) to run fewer ranks than asked for. The driver's scaling run uses
`torch.distributed.run ... bench.py --gpus N`, which sets WORLD_SIZE itself."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    if env:
        e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_forms_n_ranks(n):
    r = _run(["--gpus", str(n), "--selftest", "--batch", "1000"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # rank 0's JSON line and nothing else
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["max_over_ranks"] == float(n)  # every rank took part in the MAX reduction
    # the node figure: one 1000-check request shared by the n ranks in contiguous slices, in rank
    # order, covering it exactly (strong scaling); weak scaling checks n x 1000 per step
    assert out["global_batch"] == 1000
    sl = out["slices"]
    assert len(sl) == n and sl[0][0] == 0 and sl[-1][1] == 1000
    assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
    assert max(e - b for b, e in sl) - min(e - b for b, e in sl) <= 1
    assert out["slice"] == sl[0]
    assert out["checks_per_step"] == {"strong": 1000, "weak": 1000 * n}


def test_launcher_refuses_missing_gpus():
    # this container has no GPU: asking for 2 must fail loudly rather than run one rank
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs visible")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "refusing" in r.stderr


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2", "--steps", "1"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
