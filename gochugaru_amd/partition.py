"""Partitioned checks across ranks: the exchange of a partitioned engine.

SURVEY.md §8e (BASELINE.json config 4, partitioned mode): a graph above one GPU's 288 GB is split
by object id — rank r keeps the rows of the objects it owns (``gck_partition_owner``: id mod
world), the replicated hub hierarchy and the hub memberships of the subjects it owns
(include/gck.h; partition.inc) — and every rank checks the same batch with the others. The engine
runs the whole batch (the label join, then the exact-depth level loop with joins) inside
``gck_part_check_with``; it only needs two collectives from its caller (``gck_transport``):

* ``alltoallv``: per peer a block of bytes, blocks back to back in rank order on both sides;
* ``allreduce_max_u8``: an element-wise MAX over the ranks of a byte array, in place.

:class:`GlooTransport` implements them with torch.distributed collectives over host-staged copies
(gloo: CPU rehearsals, several ranks sharing one GPU); :class:`RcclPartitionedChecker` uses the
RCCL transport inside libgck (``gck_part_check``; one process per GPU, xGMI).
"""
from __future__ import annotations

import ctypes
import traceback
from typing import Optional

from .engine import ALLREDUCE_MAX_U8_FN, ALLTOALLV_FN, Engine, Transport

_HIP = None


def _hip():
    """The HIP runtime this process already uses (the one libgck and torch resolved to)."""
    global _HIP
    if _HIP is None:
        path = "libamdhip64.so"
        try:
            for line in open("/proc/self/maps"):
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
        except OSError:
            pass
        h = ctypes.CDLL(path)
        h.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        h.hipMemcpyAsync.restype = ctypes.c_int
        h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        h.hipStreamSynchronize.restype = ctypes.c_int
        _HIP = h
    return _HIP


class GlooTransport:
    """gck_transport over torch.distributed collectives on host tensors (any backend that takes
    CPU tensors: gloo). ``device=True``: the engine's buffers are device memory (copied through
    the HIP runtime after the engine's stream is synchronised); ``device=False``: host memory
    (a transport test without a GPU). The first failure is kept in ``error``."""

    def __init__(self, group=None, device: bool = True):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.error: Optional[str] = None
        self.calls = {"alltoallv": 0, "allreduce_max_u8": 0, "bytes": 0}
        # (the callbacks must outlive every call that may use them)
        self._a2a = ALLTOALLV_FN(self._alltoallv)
        self._ar = ALLREDUCE_MAX_U8_FN(self._allreduce)
        self.c = Transport(None, self._a2a, self._ar)

    def _sync(self, stream):
        if self.device:
            rc = _hip().hipStreamSynchronize(stream)
            if rc != 0:
                raise RuntimeError(f"hipStreamSynchronize failed ({rc})")

    def _copy(self, dst: int, src: int, n: int, stream):
        if n == 0:
            return
        if self.device:
            # on the engine's stream, then waited for: the engine's next kernels on that stream are
            # ordered after the copy, and the host buffer may be reused once this returns (a
            # synchronous hipMemcpy runs on the null stream, which a non-blocking stream does not
            # wait for, and may return before a pageable upload has landed)
            rc = _hip().hipMemcpyAsync(dst, src, n, 4, stream)  # hipMemcpyDefault: either side
            if rc != 0:
                raise RuntimeError(f"hipMemcpyAsync failed ({rc})")
            self._sync(stream)
        else:
            ctypes.memmove(dst, src, n)

    def _alltoallv(self, ctx, send, send_bytes, recv, recv_bytes, stream) -> int:
        try:
            torch = self.torch
            sb = [int(send_bytes[i]) for i in range(self.world)]
            rb = [int(recv_bytes[i]) for i in range(self.world)]
            self._sync(stream)
            hs = torch.empty(sum(sb), dtype=torch.uint8)
            hr = torch.empty(sum(rb), dtype=torch.uint8)
            self._copy(hs.data_ptr(), send, sum(sb), stream)
            self.dist.all_to_all_single(hr, hs, output_split_sizes=rb, input_split_sizes=sb, group=self.group)
            self._copy(recv, hr.data_ptr(), sum(rb), stream)
            self.calls["alltoallv"] += 1
            self.calls["bytes"] += sum(sb)
            return 0
        except Exception:  # (an exception may not cross the C ABI)
            self.error = self.error or traceback.format_exc()
            return -1

    def _allreduce(self, ctx, buf, n, stream) -> int:
        try:
            torch = self.torch
            self._sync(stream)
            h = torch.empty(int(n), dtype=torch.uint8)
            self._copy(h.data_ptr(), buf, int(n), stream)
            self.dist.all_reduce(h, op=self.dist.ReduceOp.MAX, group=self.group)
            self._copy(buf, h.data_ptr(), int(n), stream)
            self.calls["allreduce_max_u8"] += 1
            return 0
        except Exception:
            self.error = self.error or traceback.format_exc()
            return -1


class LocalTransport:
    """gck_transport between the ranks of one process: each rank's engine runs its collective call
    (gck_part_intern_with, gck_part_add_tuples_text_with, gck_part_check_with) on its own thread,
    and the blocks meet in host memory behind a barrier per collective. For rehearsals and tests
    of several ranks' engines in one process (one GPU or several); ``endpoint(rank).c`` is the
    struct a rank passes."""

    class _End:
        def __init__(self, hub, rank):
            self.hub, self.rank = hub, rank
            self.error: Optional[str] = None
            self._a2a = ALLTOALLV_FN(self._alltoallv)
            self._ar = ALLREDUCE_MAX_U8_FN(self._allreduce)
            self.c = Transport(None, self._a2a, self._ar)

        def _get(self, src, n, stream):
            buf = (ctypes.c_uint8 * max(1, n))()
            if n:
                rc = _hip().hipMemcpyAsync(ctypes.addressof(buf), src, n, 4, stream)
                if rc != 0 or _hip().hipStreamSynchronize(stream) != 0:
                    raise RuntimeError(f"hipMemcpyAsync failed ({rc})")
            return bytes(buf)[:n]

        def _put(self, dst, data, stream):
            if data:
                src = ctypes.create_string_buffer(data, len(data))
                rc = _hip().hipMemcpyAsync(dst, ctypes.addressof(src), len(data), 4, stream)
                if rc != 0 or _hip().hipStreamSynchronize(stream) != 0:
                    raise RuntimeError(f"hipMemcpyAsync failed ({rc})")

        def _alltoallv(self, ctx, send, send_bytes, recv, recv_bytes, stream) -> int:
            try:
                h, w = self.hub, self.hub.world
                _hip().hipStreamSynchronize(stream)
                sb = [int(send_bytes[i]) for i in range(w)]
                rb = [int(recv_bytes[i]) for i in range(w)]
                flat = self._get(send, sum(sb), stream)
                blocks, at = [], 0
                for k in range(w):
                    blocks.append(flat[at:at + sb[k]])
                    at += sb[k]
                h.box[self.rank] = blocks
                h.barrier.wait()
                got = b"".join(h.box[s][self.rank] for s in range(w))
                h.barrier.wait()
                if len(got) != sum(rb):
                    raise RuntimeError(f"alltoallv: {len(got)} bytes arrived, {sum(rb)} expected")
                self._put(recv, got, stream)
                return 0
            except Exception:  # (an exception may not cross the C ABI)
                self.error = self.error or traceback.format_exc()
                self.hub.barrier.abort()
                return -1

        def _allreduce(self, ctx, buf, n, stream) -> int:
            try:
                h = self.hub
                _hip().hipStreamSynchronize(stream)
                h.box[self.rank] = self._get(buf, int(n), stream)
                h.barrier.wait()
                out = bytes(max(col) for col in zip(*h.box)) if n else b""
                h.barrier.wait()
                self._put(buf, out, stream)
                return 0
            except Exception:
                self.error = self.error or traceback.format_exc()
                self.hub.barrier.abort()
                return -1

    def __init__(self, world: int):
        import threading
        self.world = world
        self.barrier = threading.Barrier(world)
        self.box = [None] * world
        self.ends = [LocalTransport._End(self, r) for r in range(world)]

    def endpoint(self, rank: int) -> "LocalTransport._End":
        return self.ends[rank]

    def run(self, fn):
        """fn(rank) on one thread per rank, together (a collective of every rank); the first
        exception is raised here."""
        import threading
        errs = [None] * self.world

        def body(r):
            try:
                fn(r)
            except BaseException as ex:  # noqa: BLE001
                errs[r] = ex
                self.barrier.abort()
        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        self.barrier.reset()
        for ex in errs:
            if ex is not None:
                raise ex


class PartitionedChecker:
    """Checks batches on a partitioned engine (``Engine.set_partition`` before the snapshot) over
    a torch.distributed group: every rank of ``group`` calls :meth:`check` with the same items and
    gets every result (``gck_part_check_with`` with a :class:`GlooTransport`)."""

    def __init__(self, engine: Engine, group=None):
        import torch
        import torch.distributed as dist

        self.engine = engine
        self.torch = torch
        self.world = dist.get_world_size(group)
        assert engine.part_world == self.world and engine.part_rank == dist.get_rank(group), \
            "engine partition (set_partition) must match the process group"
        self.transport = GlooTransport(group, device=True)

    def check(self, d_items, n: int, now_us: int = 0, out=None):
        """``d_items``: a device tensor holding n gck_item records (20 bytes each). Returns
        (permissionship uint8[n], item error int32[n]) on the device, identical on every rank."""
        torch = self.torch
        if out is None:
            out = (torch.zeros(n, dtype=torch.uint8, device=d_items.device),
                   torch.zeros(n, dtype=torch.int32, device=d_items.device))
        perm, err = out
        stream = torch.cuda.current_stream(d_items.device).cuda_stream
        try:
            self.engine.part_check_with(self.transport.c, d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(),
                                        now_us, stream)
        except Exception as ex:
            if self.transport.error:
                raise RuntimeError(f"{ex}\ntransport failure:\n{self.transport.error}") from ex
            raise
        return perm, err


class RcclPartitionedChecker:
    """Checks batches on a partitioned engine with the exchange inside libgck (``gck_part_check``:
    grouped RCCL send / receive and all-reduce over xGMI, one process per GPU). ``group`` (any
    torch.distributed backend) only carries the communicator id from rank 0 to the others, once."""

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

    def check(self, d_items, n: int, now_us: int = 0, out=None):
        """`out`: (perm uint8[n], err int32[n]) device tensors to write into (a caller's
        preallocated result buffers); new ones otherwise. Ordered on the caller's current stream
        (taken at every call)."""
        torch = self.torch
        if out is None:
            out = (torch.zeros(n, dtype=torch.uint8, device=d_items.device),
                   torch.zeros(n, dtype=torch.int32, device=d_items.device))
        perm, err = out
        stream = torch.cuda.current_stream(d_items.device).cuda_stream
        self.engine.part_check(d_items.data_ptr(), n, perm.data_ptr(), err.data_ptr(), now_us, stream)
        return perm, err
