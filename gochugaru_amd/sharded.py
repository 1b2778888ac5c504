"""Replicated-graph multi-GPU checks ("replicated graph, batch sharded over G
GPUs"; BASELINE.json configs 2-4 when the graph fits one GPU).

Two drivers of the same contract — one CheckBulkPermissions request split into G contiguous
slices, each slice checked against a full replica of the snapshot, the pairs returned in request
order (the order ``Client.Check`` maps them in, client/client.go:271-283):

* :class:`ShardedEngine` — one process driving G devices (how a Go server embeds the engine: one
  ``gck_engine`` per GPU). Every snapshot / Watch call goes to every replica; a
  check request is cut into G slices, each slice submitted to its device without waiting
  (``gck_check_submit``), then all are waited for and concatenated. No collective: the graph is
  replicated, the results come back by D2H.
* :class:`DistributedChecker` — one process per GPU (torch.distributed, as ``bench.py --gpus N``
  runs): every rank checks its own contiguous slice of the global request; ``gather`` collects the
  slices in rank order when a caller needs the whole answer on one rank.
"""
from __future__ import annotations

from collections import deque
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .engine import CONSISTENCY_MIN_LATENCY, ITEM_DTYPE, Engine


def slices(n: int, g: int) -> List[Tuple[int, int]]:
    """The G contiguous [begin, end) slices of n items (sizes differ by at most one)."""
    base, extra = divmod(n, g)
    out, pos = [], 0
    for k in range(g):
        ln = base + (1 if k < extra else 0)
        out.append((pos, pos + ln))
        pos += ln
    return out


class ShardedEngine:
    """G replicas of one snapshot, one engine per device (devices may repeat: several replicas on
    one GPU rehearse the protocol)."""

    def __init__(self, devices: Sequence[int], **engine_kw):
        if not devices:
            raise ValueError("at least one device")
        self.devices = list(devices)
        self.engines = [Engine(device=d, **engine_kw) for d in self.devices]
        self.max_batch = engine_kw.get("max_batch") or 65536  # 0 = the engine's default
        # batches one replica may have in flight: its workspace pool (gck_config.workspaces,
        # 0 = 4). A submit beyond it would wait for a workspace its own caller holds.
        self.depth = engine_kw.get("workspaces") or 4

    def close(self):
        for e in self.engines:
            e.close()

    # ---- everything that changes the snapshot goes to every replica -----------------------
    def load_schema(self, text: str):
        for e in self.engines:
            e.load_schema(text)

    def load_snapshot_text(self, revision: int, text: str):
        for e in self.engines:
            e.load_snapshot_text(revision, text)

    def apply_updates_text(self, revision: int, text: str):
        for e in self.engines:
            e.apply_updates_text(revision, text)

    def apply_updates(self, revision: int, updates: np.ndarray):
        for e in self.engines:
            e.apply_updates(revision, updates)

    def set_head_revision(self, revision: int):
        for e in self.engines:
            e.set_head_revision(revision)

    @property
    def revision(self) -> int:
        revs = {e.revision for e in self.engines}
        if len(revs) != 1:
            raise RuntimeError(f"replicas at different revisions: {sorted(revs)}")
        return revs.pop()

    def make_items(self, rels) -> np.ndarray:
        # every replica interns the same names to the same ids (same snapshot, same order)
        return self.engines[0].make_items(rels)

    def make_request(self, rels):
        return self.engines[0].make_request(rels)

    # ---- checks ------------------------------------------------------------------------------
    def check_bulk(self, items: np.ndarray, requirement: int = CONSISTENCY_MIN_LATENCY, revision: int = 0,
                   now_us: int = 0, contexts: Optional[Sequence] = None) -> Tuple[np.ndarray, np.ndarray]:
        """One request over all replicas: slice k (contiguous) on replica k, in chunks of
        max_batch. Chunks are submitted round-robin over the replicas with at most `depth` in
        flight per replica (the oldest of a replica is waited for before its next submit: never
        more outstanding batches than its workspace pool, include/gck.h); results in request
        order."""
        items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
        n = len(items)
        perm = np.zeros(n, dtype=np.uint8)
        err = np.zeros(n, dtype=np.int32)
        if n == 0:
            self.engines[0].check_bulk(items, requirement, revision, now_us, contexts)  # consistency errors
            return perm, err
        chunks = [[(c, min(en, c + self.max_batch)) for c in range(b, en, self.max_batch)]
                  for b, en in slices(n, len(self.engines))]
        inflight = [deque() for _ in self.engines]

        def finish(q):
            c, ce, bt = q.popleft()
            p, x = bt.wait()
            perm[c:ce] = p
            err[c:ce] = x

        try:
            for k in range(max(len(ch) for ch in chunks)):
                for r, e in enumerate(self.engines):
                    if k >= len(chunks[r]):
                        continue
                    if len(inflight[r]) >= self.depth:
                        finish(inflight[r])
                    c, ce = chunks[r][k]
                    inflight[r].append((c, ce, e.submit(items[c:ce], requirement=requirement, revision=revision,
                                                        now_us=now_us, contexts=contexts)))
            for q in inflight:
                while q:
                    finish(q)
        finally:  # an error leaves no batch holding a workspace
            for q in inflight:
                for _, _, bt in q:
                    try:
                        bt.wait()
                    except Exception:
                        pass
        return perm, err


class DistributedChecker:
    """One rank's share of a global request (torch.distributed; gloo or nccl): rank r checks the
    r-th contiguous slice on its own engine (a full replica); ``gather`` returns the whole answer
    in request order on every rank."""

    def __init__(self, checker, group=None):
        import torch.distributed as dist
        self.checker = checker  # anything with check_bulk(items) -> (perm, err) (an Engine)
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def my_slice(self, n: int) -> Tuple[int, int]:
        return slices(n, self.world)[self.rank]

    def check_slice(self, items: np.ndarray, **kw) -> Tuple[np.ndarray, np.ndarray]:
        """This rank's slice of the global request `items` (the same array on every rank)."""
        b, e = self.my_slice(len(items))
        return self.checker.check_bulk(items[b:e], **kw)

    def gather(self, n: int, perm: np.ndarray, err: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Every rank's slice, in request order, on every rank (gloo: host tensors; nccl/RCCL:
        the rank's current GPU, which that backend requires)."""
        import torch
        parts = slices(n, self.world)
        width = max(e - b for b, e in parts)
        dev = (torch.device("cuda", torch.cuda.current_device())
               if self.dist.get_backend(self.group) == "nccl" else torch.device("cpu"))
        buf = torch.zeros(width, 5, dtype=torch.uint8)
        k = len(perm)
        buf[:k, 0] = torch.from_numpy(perm)
        buf[:k, 1:] = torch.from_numpy(err.astype(np.int32).view(np.uint8).reshape(k, 4))
        buf = buf.to(dev)
        out = [torch.zeros_like(buf) for _ in range(self.world)]
        self.dist.all_gather(out, buf, group=self.group)
        out = [t.cpu() for t in out]
        perm_all = np.zeros(n, dtype=np.uint8)
        err_all = np.zeros(n, dtype=np.int32)
        for (b, e), t in zip(parts, out):
            a = t.numpy()[: e - b]
            perm_all[b:e] = a[:, 0]
            err_all[b:e] = a[:, 1:].copy().view(np.int32).reshape(-1)
        return perm_all, err_all
