"""Host driver of partitioned checks: one BFS level per round, exchanged over torch.distributed.

SURVEY.md §8e (BASELINE.json config 4, partitioned mode): graphs above one GPU's 288 GB are
split by resource id — rank r keeps the CSR rows of the objects it owns
(``gck_partition_owner``) — and every rank checks the same global batch together. The engine
(``gck_part_*``, include/gck.h; partition.inc) does the device work of a level; this module moves
data between ranks:

* the entries a rank produced for objects it does not own: counts, then the 12-byte entries,
  ``all_to_all_single`` — RCCL over xGMI with the ``nccl`` backend (one process per GPU), or
  host-staged with ``gloo`` (CPU rehearsals, several ranks sharing one GPU);
* the per-check flag planes (found / conditional / depth error / alive, 4n+1 bytes):
  ``all_reduce(MAX)``, after which every rank resolves every check identically, so the loop
  ends on every rank in the same round without another collective.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .engine import PART_ENTRY_BYTES, PART_JOIN_RECORD_BYTES, Engine, part_flag_bytes

_WORDS = PART_ENTRY_BYTES // 4  # an entry is three 32-bit words on the wire
_RWORDS = PART_JOIN_RECORD_BYTES // 4  # a label-join record (check index, 3 reserved, subject slot): 20 words


class PartitionedChecker:
    """Checks global batches on a partitioned engine (``Engine.set_partition`` before the
    snapshot). Every rank of ``group`` calls :meth:`check` with the same items."""

    def __init__(self, engine: Engine, group=None):
        import torch
        import torch.distributed as dist

        self.engine = engine
        self.group = group
        self.dist = dist
        self.torch = torch
        self.world = dist.get_world_size(group)
        assert engine.part_world == self.world and engine.part_rank == dist.get_rank(group), \
            "engine partition (set_partition) must match the process group"
        self.staged = dist.get_backend(group) != "nccl"  # gloo: exchange through host memory
        # the engine's device (a CPU model of the protocol sets torch_device, tests/part_model.py)
        self.device = getattr(engine, "torch_device", None) or torch.device("cuda", torch.cuda.current_device())
        self.cuda = self.device.type == "cuda"
        self._send = torch.empty(0, dtype=torch.int32, device=self.device)
        self.levels = 0

    def _sync(self):
        if self.cuda:
            self.torch.cuda.synchronize(self.device)

    def _coll_tensor(self, t):
        return t.cpu() if self.staged else t

    def _back(self, t_coll, t_dev):
        if self.staged:
            t_dev.copy_(t_coll)

    def check(self, d_items, n: int, now_us: int = 0) -> Tuple["torch.Tensor", "torch.Tensor"]:
        """``d_items``: a device tensor holding n gck_item records (20 bytes each). Returns
        (permissionship uint8[n], item error int32[n]) on the device, identical on every rank.
        First the label join (one all-to-all of (check, subject slot) records to the owners of
        the resources, an all-reduce MAX of the decided result bytes), then the level loop over
        what no rank decided, in batch order."""
        torch, dist = self.torch, self.dist
        eng = self.engine
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.cuda else None
        perm = torch.zeros(n, dtype=torch.uint8, device=self.device)
        err = torch.zeros(n, dtype=torch.int32, device=self.device)
        send = torch.empty(max(n, 1) * _RWORDS, dtype=torch.int32, device=self.device)
        self._sync()
        counts = eng.part_join_pack(d_items.data_ptr(), n, send.data_ptr(), max(n, 1), stream)
        send_cnt = torch.from_numpy(counts.astype(np.int64))
        recv_cnt = torch.zeros(self.world, dtype=torch.int64)
        if not self.staged:
            send_cnt, recv_cnt = send_cnt.to(self.device), recv_cnt.to(self.device)
        dist.all_to_all_single(recv_cnt, send_cnt, group=self.group)
        rc = recv_cnt.cpu().numpy()
        n_recv = int(rc.sum())
        recv = torch.empty(max(n_recv, 1) * _RWORDS, dtype=torch.int32, device=self.device)
        s_send = self._coll_tensor(send[: int(counts.sum()) * _RWORDS])
        s_recv = self._coll_tensor(recv[: n_recv * _RWORDS])
        dist.all_to_all_single(s_recv, s_send, output_split_sizes=[int(c) * _RWORDS for c in rc],
                               input_split_sizes=[int(c) * _RWORDS for c in counts], group=self.group)
        self._back(s_recv, recv[: n_recv * _RWORDS])
        self._sync()
        eng.part_join_decide(d_items.data_ptr(), n, recv.data_ptr(), n_recv, perm.data_ptr(), err.data_ptr(), stream)
        f = self._coll_tensor(perm)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        self._back(f, perm)
        self._sync()
        self.joined = int((perm != 0).sum())
        left = torch.nonzero(perm == 0).flatten()
        if left.numel() == 0:
            self.levels = 0
            return perm, err
        items2 = d_items.reshape(n, 20)[left].contiguous()
        p2, e2 = self._loop(items2, int(left.numel()), now_us)
        perm[left] = p2
        err[left] = e2
        return perm, err

    def _loop(self, d_items, n: int, now_us: int = 0):
        """The level-synchronous loop (gck_part_begin .. gck_part_finish) over d_items."""
        torch, dist = self.torch, self.dist
        eng = self.engine
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.cuda else None
        flags = torch.zeros(part_flag_bytes(n), dtype=torch.uint8, device=self.device)
        perm = torch.zeros(n, dtype=torch.uint8, device=self.device)
        err = torch.zeros(n, dtype=torch.int32, device=self.device)
        self._sync()
        eng.part_begin(d_items.data_ptr(), n, now_us, stream)
        self.levels = 0
        while True:
            counts = eng.part_expand()
            total = int(counts.sum())
            if self._send.numel() < total * _WORDS:
                self._send = torch.empty(max(total * _WORDS, 2 * self._send.numel()), dtype=torch.int32,
                                         device=self.device)
            if total:
                eng.part_pack(self._send.data_ptr(), total)
            send_cnt = torch.from_numpy(counts.astype(np.int64))
            recv_cnt = torch.zeros(self.world, dtype=torch.int64)
            if not self.staged:
                send_cnt, recv_cnt = send_cnt.to(self.device), recv_cnt.to(self.device)
            dist.all_to_all_single(recv_cnt, send_cnt, group=self.group)
            rc = recv_cnt.cpu().numpy()
            n_recv = int(rc.sum())
            recv = torch.empty(max(n_recv, 1) * _WORDS, dtype=torch.int32, device=self.device)
            s_send = self._coll_tensor(self._send[: total * _WORDS])
            s_recv = self._coll_tensor(recv[: n_recv * _WORDS])
            dist.all_to_all_single(s_recv, s_send, output_split_sizes=[int(c) * _WORDS for c in rc],
                                   input_split_sizes=[int(c) * _WORDS for c in counts], group=self.group)
            self._back(s_recv, recv[: n_recv * _WORDS])
            self._sync()
            eng.part_ingest(recv.data_ptr(), n_recv, flags.data_ptr())
            f = self._coll_tensor(flags)
            dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
            self._back(f, flags)
            self._sync()
            active = eng.part_resolve(flags.data_ptr())
            self.levels += 1
            if active == 0:
                break
        eng.part_finish(perm.data_ptr(), err.data_ptr())
        return perm, err


class RcclPartitionedChecker:
    """Checks global batches on a partitioned engine with the level loop and its exchange inside
    libgck (``gck_part_check``: grouped RCCL send / receive + all-reduce over xGMI, one process
    per GPU). ``group`` (any torch.distributed backend) only carries the communicator id from
    rank 0 to the others, once."""

    def __init__(self, engine: Engine, group=None):
        import torch
        import torch.distributed as dist

        self.engine = engine
        self.torch = torch
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        assert engine.part_world == world and engine.part_rank == rank, \
            "engine partition (set_partition) must match the process group"
        box = [Engine.part_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0, group=group)
        engine.part_init(box[0])
        self._stream = None

    def check(self, d_items, n: int, now_us: int = 0, out=None):
        """`out`: (perm uint8[n], err int32[n]) device tensors to write into (a caller's
        preallocated result buffers); new ones otherwise."""
        torch = self.torch
        if out is None:
            out = (torch.zeros(n, dtype=torch.uint8, device=d_items.device),
                   torch.zeros(n, dtype=torch.int32, device=d_items.device))
        perm, err = out
        if self._stream is None:
            self._stream = torch.cuda.current_stream(d_items.device).cuda_stream
        self.engine.part_check(d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(), now_us, self._stream)
        return perm, err

