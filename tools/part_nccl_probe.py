"""Probe: can two RCCL ranks share one GPU on this box? Runs the partitioned parity case
(tests/test_gpu_partition.py) with the nccl backend; prints the outcome."""
import os
import sys
import tempfile
import pathlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_partition as T  # noqa: E402

if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        outs = T._run(pathlib.Path(d), 2, "nested", 1, backend="nccl")
        print("nccl 2 ranks on one GPU: ok", outs[0]["levels"])
