"""ctypes binding of ``libgck.so`` (the C ABI in ``include/gck.h``).

This is the host-side plumbing a Python caller uses; a Go caller binds the same symbols with
cgo. The shared library is built in-tree by ``__graft_entry__.build()``
(``make -C gochugaru_amd/csrc``). There is deliberately **no fallback**: if the library or a
HIP device is missing, the calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import time
import weakref
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

# GCK_LIBRARY: an instrumented build of the same sources (make TIMING=1 -> libgck_timing.so)
_LIB_PATH = os.environ.get("GCK_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgck.so")

# ---- constants mirrored from include/gck.h ------------------------------------------------
GCK_OK = 0
GCK_E_INVALID_ARGUMENT = -1
GCK_E_SCHEMA = -2
GCK_E_NOT_FOUND = -3
GCK_E_DEVICE = -4
GCK_E_CAPACITY = -5
GCK_E_STATE = -6
GCK_E_REVISION = -7
GCK_E_NO_DEVICE = -8
GCK_E_REVISION_GONE = -9

PERM_UNSPECIFIED, PERM_NO, PERM_HAS, PERM_CONDITIONAL = 0, 1, 2, 3

ITEM_OK = 0
ITEM_ERR_MAX_DEPTH = 1
ITEM_ERR_UNKNOWN_PERMISSION = 2
ITEM_ERR_UNKNOWN_TYPE = 3
ITEM_ERR_UNKNOWN_SUBJECT_RELATION = 4
ITEM_ERR_WILDCARD_SUBJECT = 5
ITEM_ERR_CAVEAT_EVAL = 6

ELLIPSIS = 0xFFFF
ID_WILDCARD = 0xFFFFFFFF
ID_ABSENT = 0xFFFFFFFE
TYPE_INVALID = 0xFFFF
REL_INVALID = 0xFFFE  # an id no schema relation has (never equal to ELLIPSIS)

CONSISTENCY_MIN_LATENCY, CONSISTENCY_FULL, CONSISTENCY_AT_LEAST, CONSISTENCY_SNAPSHOT = 0, 1, 2, 3
CAVEAT_FALSE, CAVEAT_TRUE, CAVEAT_PARTIAL = 0, 1, 2
INTERN_CREATE = 1
MEM_DEVICE = 1
FLAG_PROFILE = 1
FLAG_NO_BUNDLE = 2
FLAG_NO_MHASH = 4
FLAG_NO_GIANT = 8
FLAG_NO_BIDIR = 16
FLAG_NO_CLOSURE = 32
FLAG_LAZY_CAVEATS = 64
FLAG_NO_SLOTS = 128
FLAG_NO_LABELS = 256
FLAG_RESIDENT = 512
FLAG_BIG_MHASH = 1024
SUBMIT_DEVICE = 1
SUBMIT_ENGINE_STREAM = 2

ITEM_DTYPE = np.dtype([
    ("resource_type", "<u2"), ("permission", "<u2"), ("resource_id", "<u4"),
    ("subject_type", "<u2"), ("subject_relation", "<u2"), ("subject_id", "<u4"),
    ("context_slot", "<u4"),
])
assert ITEM_DTYPE.itemsize == 20

TUPLE_DTYPE = np.dtype({
    "names": ["resource_type", "relation", "resource_id", "subject_type", "subject_relation",
              "subject_id", "caveat", "expires_at_us"],
    "formats": ["<u2", "<u2", "<u4", "<u2", "<u2", "<u4", "<u4", "<i8"],
    "offsets": [0, 2, 4, 8, 10, 12, 16, 24],
    "itemsize": 32,
})

UPDATE_CREATE, UPDATE_DELETE, UPDATE_TOUCH = 1, 2, 3  # rel.UpdateType (rel/relationship.go:267-274)
UPDATE_DTYPE = np.dtype({"names": ["op", "reserved", "tuple"], "formats": ["<u4", "<u4", TUPLE_DTYPE],
                         "offsets": [0, 4, 8], "itemsize": 40})

ITEM_ERROR_MESSAGES = {
    ITEM_ERR_MAX_DEPTH: "max depth exceeded: this usually indicates a recursive or too deep data dependency",
    ITEM_ERR_UNKNOWN_PERMISSION: "relation/permission not found",
    ITEM_ERR_UNKNOWN_TYPE: "object definition not found",
    ITEM_ERR_UNKNOWN_SUBJECT_RELATION: "subject relation not found",
    ITEM_ERR_WILDCARD_SUBJECT: "cannot perform check on wildcard subject",
    ITEM_ERR_CAVEAT_EVAL: "evaluation error for caveat",
}


class GckError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"gck error {code}: {message}")
        self.code = code
        self.message = message


class _Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_depth", C.c_uint32), ("max_batch", C.c_uint32),
                ("flags", C.c_uint32), ("visited_capacity", C.c_uint64),
                ("frontier_capacity", C.c_uint64), ("segment_capacity", C.c_uint64),
                ("query_capacity", C.c_uint64), ("bundle_checks", C.c_uint32),
                ("bundle_frontier", C.c_uint32), ("bundle_visited", C.c_uint32),
                ("bundle_waves_per_cu", C.c_uint32), ("bundle_budget", C.c_uint32),
                ("giant_frontier", C.c_uint32), ("giant_visited", C.c_uint32),
                ("giant_slots", C.c_uint32), ("bidir_both", C.c_uint32),
                ("workspaces", C.c_uint32)]


class _Consistency(C.Structure):
    _fields_ = [("requirement", C.c_int32), ("reserved", C.c_uint32), ("revision", C.c_uint64)]


class _Stats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("levels", C.c_uint64), ("entries_expanded", C.c_uint64),
                ("row_lookups", C.c_uint64), ("membership_probes", C.c_uint64),
                ("edges_enumerated", C.c_uint64), ("ext_edges", C.c_uint64),
                ("queries", C.c_uint64), ("joins", C.c_uint64), ("retries", C.c_uint64),
                ("kernel_ms", C.c_double), ("expand_ms", C.c_double), ("edges_ms", C.c_double),
                ("resolve_ms", C.c_double), ("expand_launches", C.c_uint64),
                ("edges_launches", C.c_uint64), ("bundle_ms", C.c_double),
                ("bundle_launches", C.c_uint64), ("deferred", C.c_uint64),
                ("giant_ms", C.c_double), ("deferred_wide", C.c_uint64),
                ("bidir_checks", C.c_uint64), ("bundles", C.c_uint64), ("closure_checks", C.c_uint64),
                ("caveat_evals", C.c_uint64), ("caveat_passes", C.c_uint64), ("slot_checks", C.c_uint64),
                ("label_checks", C.c_uint64), ("aql_batches", C.c_uint64), ("resident_batches", C.c_uint64)]


class Uniform(C.Structure):
    """gck_uniform (include/gck.h): the shared shape of a uniform request's checks."""
    _fields_ = [("resource_type", C.c_uint16), ("permission", C.c_uint16), ("subject_type", C.c_uint16),
                ("subject_relation", C.c_uint16), ("context_slot", C.c_uint32), ("reserved", C.c_uint32)]


# gck_item_error: (index, GCK_ITEM_*) of a uniform request's errored checks
ITEM_ERROR_DTYPE = np.dtype([("index", "<u4"), ("code", "<i4")])


def unpack_results(words: np.ndarray, n: int) -> np.ndarray:
    """The Permissionship of each of n checks from a uniform request's packed words (2 bits per
    check, 32 per little-endian u64 word: include/gck.h gck_check_bulk_uniform)."""
    b = np.ascontiguousarray(words, dtype="<u8").view(np.uint8)
    four = np.stack([(b >> s) & 3 for s in (0, 2, 4, 6)], axis=1).reshape(-1)
    return four[:n].astype(np.uint8)


# symbol -> (restype, argtypes); the ABI test checks this list against include/gck.h
_P = C.c_void_p

# gck_transport (include/gck.h): a caller's exchange between the ranks of a partitioned engine
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, _P, _P, C.POINTER(C.c_uint64), _P, C.POINTER(C.c_uint64), _P)
ALLREDUCE_MAX_U8_FN = C.CFUNCTYPE(C.c_int, _P, _P, C.c_uint64, _P)


class Transport(C.Structure):
    _fields_ = [("ctx", _P), ("alltoallv", ALLTOALLV_FN), ("allreduce_max_u8", ALLREDUCE_MAX_U8_FN)]


_SIGS = {
    "gck_abi_version": (C.c_int, []),
    "gck_last_error": (C.c_char_p, []),
    "gck_create": (C.c_int, [C.POINTER(_Config), C.POINTER(_P)]),
    "gck_destroy": (None, [_P]),
    "gck_load_schema": (C.c_int, [_P, C.c_char_p, C.c_size_t]),
    "gck_type_id": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint16)]),
    "gck_relation_id": (C.c_int, [_P, C.c_uint16, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint16)]),
    "gck_type_count": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "gck_relation_count": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "gck_intern": (C.c_int, [_P, C.c_uint16, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32),
                             C.c_size_t, C.c_uint32, C.POINTER(C.c_uint32)]),
    "gck_object_count": (C.c_int, [_P, C.c_uint16, C.POINTER(C.c_uint32)]),
    "gck_reserve_objects": (C.c_int, [_P, C.c_uint16, C.c_uint32]),
    "gck_object_name": (C.c_int, [_P, C.c_uint16, C.c_uint32, C.c_char_p, C.c_size_t,
                                  C.POINTER(C.c_size_t)]),
    "gck_add_caveat_instance": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                          C.POINTER(C.c_uint32)]),
    "gck_evaluate_caveat": (C.c_int, [_P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p,
                                      C.c_size_t, C.POINTER(C.c_uint8)]),
    "gck_begin_snapshot": (C.c_int, [_P, C.c_uint64]),
    "gck_add_tuples": (C.c_int, [_P, _P, C.c_size_t]),
    "gck_add_tuples_text": (C.c_int, [_P, C.c_char_p, C.c_size_t]),
    "gck_load_csr": (C.c_int, [_P, C.c_uint16, C.c_uint16, C.c_uint16, C.c_uint32, _P, _P,
                               C.c_uint64, C.c_uint32]),
    "gck_commit_snapshot": (C.c_int, [_P]),
    "gck_save_snapshot": (C.c_int, [_P, C.c_char_p]),
    "gck_load_snapshot_file": (C.c_int, [_P, C.c_char_p]),
    "gck_revision": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "gck_set_head_revision": (C.c_int, [_P, C.c_uint64]),
    "gck_tuple_count": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "gck_device_bytes": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "gck_apply_updates": (C.c_int, [_P, C.c_uint64, _P, C.c_size_t]),
    "gck_apply_updates_text": (C.c_int, [_P, C.c_uint64, C.c_char_p, C.c_size_t]),
    "gck_watch_stage": (C.c_int, [_P, _P, C.c_size_t, C.POINTER(C.c_uint64)]),
    "gck_watch_apply_staged": (C.c_int, [_P, C.c_uint64, C.c_uint64]),
    "gck_watch_discard": (C.c_int, [_P, C.c_uint64]),
    "gck_check_bulk": (C.c_int, [_P, C.POINTER(_Consistency), _P, C.c_size_t, C.c_int64, _P, _P]),
    "gck_check_bulk_device": (C.c_int, [_P, _P, C.c_size_t, C.c_int64, _P, _P, _P]),
    "gck_check_bulk_ctx": (C.c_int, [_P, C.POINTER(_Consistency), _P, C.c_size_t, C.POINTER(C.c_char_p),
                                     C.POINTER(C.c_size_t), C.c_size_t, C.c_int64, _P, _P]),
    "gck_check_bulk_device_ctx": (C.c_int, [_P, _P, C.c_size_t, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                            C.c_size_t, C.c_int64, _P, _P, _P]),
    "gck_check_submit": (C.c_int, [_P, C.POINTER(_Consistency), _P, C.c_size_t, C.POINTER(C.c_char_p),
                                   C.POINTER(C.c_size_t), C.c_size_t, C.c_int64, _P, _P, C.c_uint32, _P,
                                   C.POINTER(_P)]),
    "gck_set_profile": (C.c_int, [_P, C.c_uint32]),
    "gck_check_wait": (C.c_int, [_P, _P]),
    "gck_check_bulk_at": (C.c_int, [_P, C.POINTER(_Consistency), _P, C.c_size_t, C.POINTER(C.c_char_p),
                                    C.POINTER(C.c_size_t), C.c_size_t, C.c_int64, _P, _P, C.POINTER(C.c_uint64)]),
    "gck_check_wait_at": (C.c_int, [_P, _P, C.POINTER(C.c_uint64)]),
    "gck_check_bulk_uniform": (C.c_int, [_P, C.POINTER(_Consistency), C.POINTER(Uniform), _P, C.c_size_t,
                                         C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, C.c_int64, _P, _P,
                                         C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_uint64)]),
    "gck_check_submit_uniform": (C.c_int, [_P, C.POINTER(_Consistency), C.POINTER(Uniform), _P, C.c_size_t,
                                           C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, C.c_int64, _P,
                                           _P, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(_P)]),
    "gck_host_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "gck_host_free": (C.c_int, [_P, _P]),
    "gck_last_stats": (C.c_int, [_P, C.POINTER(_Stats)]),
    "gck_lookup_resources": (C.c_int, [_P, C.POINTER(_Consistency), C.c_uint16, C.c_uint16, C.c_uint16,
                                       C.c_uint16, C.c_uint32, C.c_int64, _P, _P, C.c_size_t,
                                       C.POINTER(C.c_size_t)]),
    "gck_lookup_subjects": (C.c_int, [_P, C.POINTER(_Consistency), C.c_uint16, C.c_uint32, C.c_uint16,
                                      C.c_uint16, C.c_uint16, C.c_int64, _P, _P, C.c_size_t,
                                      C.POINTER(C.c_size_t)]),
    "gck_set_partition": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "gck_partition_owner": (C.c_uint32, [C.c_uint32, C.c_uint32]),
    "gck_partition_owner_name": (C.c_uint32, [C.c_uint16, C.c_char_p, C.c_size_t, C.c_uint32]),
    "gck_part_intern_with": (C.c_int, [_P, C.POINTER(Transport), _P, _P, _P, C.c_size_t, C.c_uint32, _P]),
    "gck_part_add_tuples_text_with": (C.c_int, [_P, C.POINTER(Transport), C.c_char_p, C.c_size_t]),
    "gck_interned_names": (C.c_int, [_P, C.c_uint16, C.POINTER(C.c_uint32)]),
    "gck_part_check_with": (C.c_int, [_P, C.POINTER(Transport), _P, C.c_size_t, C.c_int64, _P, _P, _P]),
    "gck_part_unique_id": (C.c_int, [_P]),
    "gck_part_init": (C.c_int, [_P, _P]),
    "gck_part_check": (C.c_int, [_P, _P, C.c_size_t, C.c_int64, _P, _P, _P]),
    "gck_reset_stats": (C.c_int, [_P]),
}

_lib = None


_DRIVER = None


def _cpulist(text: str) -> List[int]:
    out = []
    for tok in text.strip().split(","):
        if tok:
            a, _, b = tok.partition("-")
            out.extend(range(int(a), int(b or a) + 1))
    return out


def device_numa_node(device: int = 0) -> Tuple[int, str]:
    """The NUMA node of the GPU's PCIe root (sysfs), and its PCI address; -1 when unknown."""
    import torch
    p = torch.cuda.get_device_properties(device)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip()), bdf
    except (OSError, ValueError):
        return -1, bdf


def pin_to_device_node(device: int = 0) -> dict:
    """Runs the calling process on the CPUs of the GPU's NUMA node (those of them it may use).

    A host batch's items are read by the GPU across PCIe right after the submitting thread wrote
    them: from a thread on the other socket every line is snooped out of a remote cache, and
    the copy engines and kernels read host memory ~10 % slower (tools/pcie_probe: zero-copy reads
    36 vs 40 GB/s, DMA 28-32 vs 41 GB/s). Pinned buffers already come from the GPU's node
    (hipHostMalloc follows the device). Returns what was done, for the bench line."""
    node, bdf = device_numa_node(device)
    allowed = sorted(os.sched_getaffinity(0))
    info = {"gpu_bdf": bdf, "gpu_numa_node": node, "cpus_allowed": len(allowed), "pinned": False}
    if node < 0:
        return info
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            local = set(_cpulist(f.read()))
    except OSError:
        return info
    use = [c for c in allowed if c in local]
    if use and len(use) < len(allowed):
        os.sched_setaffinity(0, use)
        info.update(pinned=True, cpus_used=len(use))
    elif use:
        info.update(cpus_used=len(use))
    return info


def _driver():
    """libgck_driver.so (csrc/driver.cpp): the compiled submit/wait loop bench.py times through."""
    global _DRIVER
    if _DRIVER is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgck_driver.so")
        if not os.path.exists(path):
            raise OSError(f"{path} is missing: build it with `make -C gochugaru_amd/csrc`")
        d = C.CDLL(path)
        d.gckd_run.restype = C.c_int
        d.gckd_run.argtypes = [C.c_void_p, C.c_void_p, _P, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p, C.c_uint32, C.c_int64,
                               C.POINTER(C.c_double)]
        d.gckd_run_host.restype = C.c_int
        d.gckd_run_host.argtypes = [C.c_void_p, C.c_void_p, _P, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_size_t, C.c_uint32, C.c_int64, C.POINTER(C.c_double)]
        d.gckd_run_uniform.restype = C.c_int
        d.gckd_run_uniform.argtypes = [C.c_void_p, C.c_void_p, _P, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32,
                                       C.c_int64, C.POINTER(C.c_double)]
        d.gckd_set_trace.restype = None
        d.gckd_set_trace.argtypes = [C.c_void_p, C.c_size_t]
        _DRIVER = d
    return _DRIVER


def load_library(path: str = _LIB_PATH):
    """Load libgck.so (raises if it has not been built — there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"libgck.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (make -C gochugaru_amd/csrc); the check engine has no CPU fallback")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME
    # libamdhip64.so.7) and loads it by file name. If libgck were loaded first, the process
    # would end up with two HIP runtimes and torch could not see the GPU. Loading torch first
    # makes libgck's NEEDED libamdhip64.so.7 resolve to the already-loaded runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int):
    if rc != GCK_OK:
        msg = _lib.gck_last_error().decode("utf-8", "replace")
        raise GckError(rc, msg)


class Stats(dict):
    pass


class Engine:
    """One engine = one device-resident snapshot on one GPU (``gck_engine``)."""

    def __init__(self, device: int = 0, max_depth: int = 50, max_batch: int = 65536,
                 visited_capacity: int = 0, frontier_capacity: int = 0,
                 segment_capacity: int = 0, query_capacity: int = 0, profile: bool = False,
                 wide_only: bool = False, bundle_checks: int = 0, bundle_frontier: int = 0,
                 bundle_visited: int = 0, bundle_waves_per_cu: int = 0,
                 membership_hash: bool = True, bundle_budget: int = 0, giant_frontier: int = 0,
                 giant_visited: int = 0, giant_slots: int = 0, giant_stage: bool = True,
                 bidir: bool = True, bidir_both: int = 0, workspaces: int = 0, closure: bool = True,
                 lazy_caveats: bool = False, slots: bool = True, labels: bool = True, resident: bool = False,
                 big_membership_hash: bool = False):
        lib = load_library()
        flags = ((FLAG_PROFILE if profile else 0) | (FLAG_NO_BUNDLE if wide_only else 0)
                 | (0 if membership_hash else FLAG_NO_MHASH) | (0 if giant_stage else FLAG_NO_GIANT)
                 | (0 if bidir else FLAG_NO_BIDIR) | (0 if closure else FLAG_NO_CLOSURE)
                 | (FLAG_LAZY_CAVEATS if lazy_caveats else 0) | (0 if slots else FLAG_NO_SLOTS)
                 | (0 if labels else FLAG_NO_LABELS) | (FLAG_RESIDENT if resident else 0)
                 | (FLAG_BIG_MHASH if big_membership_hash else 0))
        cfg = _Config(device, max_depth, max_batch, flags, visited_capacity, frontier_capacity,
                      segment_capacity, query_capacity, bundle_checks, bundle_frontier,
                      bundle_visited, bundle_waves_per_cu, bundle_budget, giant_frontier,
                      giant_visited, giant_slots, bidir_both, workspaces)
        h = _P()
        _check(lib.gck_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self._lib = lib
        self._pins = 0          # live host_array() buffers (each keeps the engine handle alive)
        self._closing = False
        self._staged = {}       # ticket -> the staged Watch batch's array (kept alive until applied)
        self._type_ids = {}
        self._rel_ids = {}
        self.part_rank, self.part_world = 0, 1

    def close(self):
        """Destroys the engine — once the last host_array() buffer is gone, since gck_destroy
        frees the pinned memory those arrays view."""
        self._closing = True
        if self._h and self._pins == 0:
            self._lib.gck_destroy(self._h)
            self._h = None

    def _unpin(self, p):
        self._pins -= 1
        if self._h:
            self._lib.gck_host_free(self._h, p)
            if self._closing and self._pins == 0:
                self._lib.gck_destroy(self._h)
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- schema --------------------------------------------------------------------------
    def load_schema(self, text: str):
        b = text.encode()
        _check(self._lib.gck_load_schema(self._h, b, len(b)))
        self._type_ids.clear()
        self._rel_ids.clear()

    def type_id(self, name: str) -> int:
        """Type id, or TYPE_INVALID if the type is not defined."""
        t = self._type_ids.get(name)
        if t is None:
            out = C.c_uint16()
            b = name.encode()
            rc = self._lib.gck_type_id(self._h, b, len(b), C.byref(out))
            if rc == GCK_E_NOT_FOUND:
                return TYPE_INVALID
            _check(rc)
            t = self._type_ids[name] = out.value
        return t

    def relation_id(self, type_id: int, name: str) -> int:
        """Global relation id, or REL_INVALID if not defined on the type."""
        key = (type_id, name)
        r = self._rel_ids.get(key)
        if r is None:
            if type_id == TYPE_INVALID:
                return REL_INVALID
            out = C.c_uint16()
            b = name.encode()
            rc = self._lib.gck_relation_id(self._h, type_id, b, len(b), C.byref(out))
            if rc == GCK_E_NOT_FOUND:
                return REL_INVALID
            _check(rc)
            r = self._rel_ids[key] = out.value
        return r

    def counts(self) -> Tuple[int, int]:
        t, r = C.c_uint32(), C.c_uint32()
        _check(self._lib.gck_type_count(self._h, C.byref(t)))
        _check(self._lib.gck_relation_count(self._h, C.byref(r)))
        return t.value, r.value

    # ---- interning -----------------------------------------------------------------------
    def intern(self, type_id: int, ids: Sequence[str], create: bool = False) -> np.ndarray:
        n = len(ids)
        out = np.empty(n, dtype=np.uint32)
        if n == 0:
            return out
        enc = [s.encode() for s in ids]
        arr = (C.c_char_p * n)(*enc)
        lens = (C.c_uint32 * n)(*[len(b) for b in enc])
        _check(self._lib.gck_intern(self._h, type_id, arr, lens, n,
                                    INTERN_CREATE if create else 0,
                                    out.ctypes.data_as(C.POINTER(C.c_uint32))))
        return out

    def object_count(self, type_id: int) -> int:
        out = C.c_uint32()
        _check(self._lib.gck_object_count(self._h, type_id, C.byref(out)))
        return out.value

    def reserve_objects(self, type_id: int, n: int):
        _check(self._lib.gck_reserve_objects(self._h, type_id, n))

    def object_name(self, type_id: int, oid: int) -> str:
        buf = C.create_string_buffer(1100)
        ln = C.c_size_t()
        _check(self._lib.gck_object_name(self._h, type_id, oid, buf, len(buf), C.byref(ln)))
        return buf.value.decode()

    def add_caveat_instance(self, name: str, context_json: str = "") -> int:
        out = C.c_uint32()
        nb, jb = name.encode(), context_json.encode()
        _check(self._lib.gck_add_caveat_instance(self._h, nb, len(nb), jb, len(jb), C.byref(out)))
        return out.value

    def evaluate_caveat(self, name: str, stored=None, context=None) -> int:
        """The host CEL evaluator: CAVEAT_FALSE / CAVEAT_TRUE / CAVEAT_PARTIAL."""
        out = C.c_uint8()
        nb = name.encode()
        sb = _context_json(stored).encode()
        cb = _context_json(context).encode()
        _check(self._lib.gck_evaluate_caveat(self._h, nb, len(nb), sb, len(sb), cb, len(cb), C.byref(out)))
        return out.value

    # ---- snapshot ------------------------------------------------------------------------
    def begin_snapshot(self, revision: int):
        _check(self._lib.gck_begin_snapshot(self._h, revision))

    def add_tuples_text(self, text: str):
        b = text.encode()
        _check(self._lib.gck_add_tuples_text(self._h, b, len(b)))

    def add_tuples(self, tuples: np.ndarray):
        tuples = np.ascontiguousarray(tuples, dtype=TUPLE_DTYPE)
        _check(self._lib.gck_add_tuples(self._h, tuples.ctypes.data, len(tuples)))

    def load_csr(self, relation: int, subject_type: int, subject_relation: int, n_rows: int,
                 offsets, neighbours, n_edges: int, device: bool = False):
        """Bulk ingest of one prebuilt CSR. Host numpy arrays (uint32) or, with device=True,
        raw device pointers (ints) on the engine's GPU."""
        if device:
            po, pn = int(offsets), int(neighbours)
        else:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
            neighbours = np.ascontiguousarray(neighbours, dtype=np.uint32)
            po, pn = offsets.ctypes.data, neighbours.ctypes.data
        _check(self._lib.gck_load_csr(self._h, relation, subject_type, subject_relation, n_rows,
                                      po, pn, n_edges, MEM_DEVICE if device else 0))

    def commit_snapshot(self):
        _check(self._lib.gck_commit_snapshot(self._h))

    def save_snapshot(self, path: str):
        """Writes the committed snapshot to `path` (the on-disk snapshot cache, gck_save_snapshot)."""
        _check(self._lib.gck_save_snapshot(self._h, os.fsencode(path)))

    def load_snapshot_file(self, path: str):
        """Replaces the committed snapshot with one saved under the same schema text."""
        _check(self._lib.gck_load_snapshot_file(self._h, os.fsencode(path)))

    def load_snapshot_text(self, revision: int, text: str):
        self.begin_snapshot(revision)
        self.add_tuples_text(text)
        self.commit_snapshot()

    @property
    def revision(self) -> int:
        out = C.c_uint64()
        _check(self._lib.gck_revision(self._h, C.byref(out)))
        return out.value

    def set_head_revision(self, revision: int):
        """The source's head revision for consistency.Full() (ReadSchema's ReadAt token,
        client/client.go:416-422, or a Watch checkpoint)."""
        _check(self._lib.gck_set_head_revision(self._h, revision))

    @property
    def tuple_count(self) -> int:
        out = C.c_uint64()
        _check(self._lib.gck_tuple_count(self._h, C.byref(out)))
        return out.value

    @property
    def device_bytes(self) -> int:
        out = C.c_uint64()
        _check(self._lib.gck_device_bytes(self._h, C.byref(out)))
        return out.value

    # ---- Watch updates (Client.UpdatesSinceRevision, client/client.go:370-413) -------------
    def apply_updates(self, revision: int, updates: np.ndarray):
        """One batch of interned updates (UPDATE_DTYPE records, stream order) -> `revision`."""
        updates = np.ascontiguousarray(updates, dtype=UPDATE_DTYPE)
        _check(self._lib.gck_apply_updates(self._h, revision, updates.ctypes.data if len(updates) else None,
                                           len(updates)))

    def stage_updates(self, updates: np.ndarray) -> int:
        """Stages a batch (gck_watch_stage): the engine's thread validates and groups it while the
        caller applies the previous one. Returns the ticket for `apply_staged`; the array is held
        until then."""
        updates = np.ascontiguousarray(updates, dtype=UPDATE_DTYPE)
        t = C.c_uint64(0)
        _check(self._lib.gck_watch_stage(self._h, updates.ctypes.data if len(updates) else None, len(updates),
                                         C.byref(t)))
        self._staged[t.value] = updates
        return t.value

    def apply_staged(self, revision: int, ticket: int):
        """Applies a staged batch -> `revision` (gck_watch_apply_staged; the errors of apply_updates)."""
        try:
            _check(self._lib.gck_watch_apply_staged(self._h, revision, ticket))
        finally:
            self._staged.pop(ticket, None)

    def discard_staged(self, ticket: int):
        try:
            _check(self._lib.gck_watch_discard(self._h, ticket))
        finally:
            self._staged.pop(ticket, None)

    def apply_updates_text(self, revision: int, text: str):
        """One batch as text: "<CREATE|TOUCH|DELETE> <rel.Relationship.String>" per line."""
        b = text.encode()
        _check(self._lib.gck_apply_updates_text(self._h, revision, b, len(b)))

    # ---- checks --------------------------------------------------------------------------
    def check_bulk(self, items: np.ndarray, requirement: int = CONSISTENCY_MIN_LATENCY,
                   revision: int = 0, now_us: int = 0,
                   contexts: Optional[Sequence] = None) -> Tuple[np.ndarray, np.ndarray]:
        """`contexts`: check-time caveat contexts (dicts or JSON text); an item's context_slot
        k selects contexts[k-1] (make_request builds both)."""
        items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
        n = len(items)
        perm = np.zeros(n, dtype=np.uint8)
        err = np.zeros(n, dtype=np.int32)
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        _check(self._lib.gck_check_bulk_ctx(self._h, C.byref(cs), items.ctypes.data if n else None, n,
                                            ctx_arr, ctx_lens, n_ctx, now_us,
                                            perm.ctypes.data if n else None,
                                            err.ctypes.data if n else None))
        return perm, err

    def check_bulk_at(self, items: np.ndarray, requirement: int = CONSISTENCY_MIN_LATENCY,
                      revision: int = 0, now_us: int = 0,
                      contexts: Optional[Sequence] = None) -> Tuple[np.ndarray, np.ndarray, int]:
        """check_bulk plus the revision the batch was evaluated at (gck_check_bulk_at): the
        response's CheckedAt."""
        items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
        n = len(items)
        perm = np.zeros(n, dtype=np.uint8)
        err = np.zeros(n, dtype=np.int32)
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        rev = C.c_uint64(0)
        _check(self._lib.gck_check_bulk_at(self._h, C.byref(cs), items.ctypes.data if n else None, n, ctx_arr,
                                           ctx_lens, n_ctx, now_us, perm.ctypes.data if n else None,
                                           err.ctypes.data if n else None, C.byref(rev)))
        return perm, err, rev.value

    def check_uniform(self, header, pairs: np.ndarray, requirement: int = CONSISTENCY_MIN_LATENCY,
                      revision: int = 0, now_us: int = 0, contexts: Optional[Sequence] = None,
                      out_packed: Optional[np.ndarray] = None, out_errs: Optional[np.ndarray] = None):
        """A uniform request (gck_check_bulk_uniform): `header` = (resource_type, permission,
        subject_type, subject_relation, context_slot), `pairs` = (n, 2) u32 (resource id, subject
        id). Returns (packed words, errors as ITEM_ERROR_DTYPE records, evaluated revision);
        unpack_results(words, n) gives the Permissionships. Pinned output arrays (host_array) are
        written in place by the kernels."""
        pairs = np.ascontiguousarray(pairs, dtype=np.uint32).reshape(-1, 2)
        n = len(pairs)
        words = out_packed if out_packed is not None else np.zeros((n + 31) // 32, dtype=np.uint64)
        errs = out_errs if out_errs is not None else np.zeros(n, dtype=ITEM_ERROR_DTYPE)
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        hdr = Uniform(*header[:4], header[4] if len(header) > 4 else 0, 0)
        n_errs = C.c_size_t(0)
        rev = C.c_uint64(0)
        _check(self._lib.gck_check_bulk_uniform(self._h, C.byref(cs), C.byref(hdr), pairs.ctypes.data if n else None,
                                                n, ctx_arr, ctx_lens, n_ctx, now_us,
                                                words.ctypes.data if n else None, errs.ctypes.data if len(errs) else None,
                                                len(errs), C.byref(n_errs), C.byref(rev)))
        return words, errs[:min(n_errs.value, len(errs))].copy(), rev.value

    def submit_uniform(self, header, pairs: np.ndarray, out_packed: np.ndarray, out_errs: np.ndarray,
                       requirement: int = CONSISTENCY_MIN_LATENCY, revision: int = 0, now_us: int = 0,
                       contexts: Optional[Sequence] = None) -> "UniformBatch":
        """gck_check_submit_uniform: the results land in out_packed / out_errs at wait()."""
        n = len(pairs)
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        hdr = Uniform(*header[:4], header[4] if len(header) > 4 else 0, 0)
        b = UniformBatch(self, hdr, pairs, out_packed, out_errs)
        _check(self._lib.gck_check_submit_uniform(self._h, C.byref(cs), C.byref(hdr), pairs.ctypes.data if n else None,
                                                  n, ctx_arr, ctx_lens, n_ctx, now_us,
                                                  out_packed.ctypes.data if n else None,
                                                  out_errs.ctypes.data if len(out_errs) else None, len(out_errs),
                                                  C.byref(b._n_errs), C.byref(b._h)))
        return b

    def prepare_uniform(self, headers, pairs, ns, packed, errs, err_cap: int, depth: int,
                        now_us: int = 0) -> "PreparedUniform":
        """The compiled submit/wait loop over uniform requests (libgck_driver.so gckd_run_uniform),
        its arguments marshalled ahead: request k = headers[k] (gck_uniform fields) and host pointers
        pairs[k] (ns[k] pairs), packed[k], errs[k] (err_cap records), `depth` in flight."""
        return PreparedUniform(self, headers, pairs, ns, packed, errs, err_cap, depth, now_us)

    def run_uniform_batches(self, header, pairs, packed, errs, err_cap: int, n: int, depth: int,
                            now_us: int = 0) -> float:
        """prepare_uniform(...).run() for requests of one header and n checks each; returns the loop's
        wall time in seconds."""
        k = len(pairs)
        return self.prepare_uniform([header] * k, pairs, [n] * k, packed, errs, err_cap, depth, now_us).run()

    def check_bulk_device(self, d_items: int, n: int, d_perm: int, d_err: int,
                          stream: Optional[int] = None, now_us: int = 0,
                          contexts: Optional[Sequence] = None):
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        _check(self._lib.gck_check_bulk_device_ctx(self._h, d_items, n, ctx_arr, ctx_lens, n_ctx, now_us,
                                                   d_perm, d_err, stream))

    def submit(self, items, n: Optional[int] = None, out_perm=None, out_err=None, requirement: int = CONSISTENCY_MIN_LATENCY,
               revision: int = 0, now_us: int = 0, contexts: Optional[Sequence] = None, device: bool = False,
               stream: Optional[int] = None, engine_stream: bool = False) -> "Batch":
        """Starts one batch (n <= max_batch) without waiting (gck_check_submit); Batch.wait()
        completes it. Host batches: `items` is an ITEM_DTYPE array and the results are returned by
        wait(). Device batches (device=True): `items`, `out_perm`, `out_err` are device pointers
        ordered on `stream`."""
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        h = _P()
        if device:
            flags = SUBMIT_DEVICE | (SUBMIT_ENGINE_STREAM if engine_stream else 0)
            _check(self._lib.gck_check_submit(self._h, C.byref(cs), items, n, ctx_arr, ctx_lens, n_ctx, now_us,
                                              out_perm, out_err, flags, stream, C.byref(h)))
            return Batch(self, h, None, None, None)
        items = np.ascontiguousarray(items, dtype=ITEM_DTYPE)
        n = len(items)
        perm = np.zeros(n, dtype=np.uint8)
        err = np.zeros(n, dtype=np.int32)
        _check(self._lib.gck_check_submit(self._h, C.byref(cs), items.ctypes.data if n else None, n, ctx_arr,
                                          ctx_lens, n_ctx, now_us, perm.ctypes.data if n else None,
                                          err.ctypes.data if n else None, 0, None, C.byref(h)))
        return Batch(self, h, perm, err, items)

    def host_array(self, n: int, dtype) -> np.ndarray:
        """A numpy array in pinned host memory (gck_host_alloc): host batches over such arrays
        are copied by DMA directly. The memory is returned (gck_host_free) when the array and
        every view of it are gone; the engine itself stays alive until then, even past close().
        A batch submitted over it reads the items by DMA until its wait (include/gck.h)."""
        if not self._h or self._closing:
            raise GckError(GCK_E_STATE, "engine closed")
        dtype = np.dtype(dtype)
        p = _P()
        _check(self._lib.gck_host_alloc(self._h, max(1, n * dtype.itemsize), C.byref(p)))
        buf = (C.c_char * max(1, n * dtype.itemsize)).from_address(p.value)
        self._pins += 1
        weakref.finalize(buf, self._unpin, p.value)  # numpy views keep `buf` alive
        return np.frombuffer(buf, dtype=dtype, count=n)

    def submit_into(self, items: np.ndarray, perm: np.ndarray, err: np.ndarray,
                    requirement: int = CONSISTENCY_MIN_LATENCY, revision: int = 0, now_us: int = 0,
                    contexts: Optional[Sequence] = None) -> "Batch":
        """A host batch writing its results into caller-provided arrays (pinned ones from
        host_array() skip the engine's staging copies). Items in a host_array() buffer are read by
        DMA while the batch runs: leave them unchanged until wait() returns (include/gck.h
        gck_check_submit); other host items are staged before this returns."""
        cs = _Consistency(requirement, 0, revision)
        ctx_arr, ctx_lens, n_ctx = _context_arrays(contexts)
        h = _P()
        n = len(items)
        _check(self._lib.gck_check_submit(self._h, C.byref(cs), items.ctypes.data if n else None, n, ctx_arr,
                                          ctx_lens, n_ctx, now_us, perm.ctypes.data if n else None,
                                          err.ctypes.data if n else None, 0, None, C.byref(h)))
        return Batch(self, h, perm, err, items)

    def set_profile(self, on: bool):
        """GCK_FLAG_PROFILE for the batches submitted from now on (gck_set_profile)."""
        _check(self._lib.gck_set_profile(self._h, 1 if on else 0))

    def prepare_batches(self, items, perms, errs, n: int, depth: int, streams=None, engine_streams: bool = False,
                        now_us: int = 0, host: bool = False) -> "PreparedRun":
        """The arguments of one compiled submit/wait loop (libgck_driver.so), marshalled ahead, so
        that a timed region holds the C loop alone. host=True: items / perms / errs are host
        pointers (gck_host_alloc memory for DMA in place), batches on the engine's streams."""
        return PreparedRun(self, items, perms, errs, n, depth, streams, engine_streams, now_us, host)

    def run_device_batches(self, items, perms, errs, n: int, depth: int, streams, engine_streams: bool = False,
                           now_us: int = 0) -> float:
        """Checks len(items) device batches of n items each (device pointers items[k], perms[k],
        errs[k]) with up to `depth` in flight, batch k on streams[k % depth] (engine_streams: on
        the engine's workspace streams, GCK_SUBMIT_ENGINE_STREAM), through the compiled
        submit/wait loop of libgck_driver.so (the loop a cgo caller runs; no Python per batch).
        Returns the loop's wall time in seconds."""
        drv = _driver()
        k = len(items)
        arr = lambda xs: (C.c_uint64 * max(1, len(xs)))(*[int(x) for x in xs])
        cs = _Consistency(CONSISTENCY_MIN_LATENCY, 0, 0)
        secs = C.c_double(0.0)
        submit = C.cast(self._lib.gck_check_submit, C.c_void_p)
        wait = C.cast(self._lib.gck_check_wait, C.c_void_p)
        _check(drv.gckd_run(submit, wait, self._h, C.byref(cs), k, arr(items), arr(perms), arr(errs), n, depth,
                            arr(streams), SUBMIT_ENGINE_STREAM if engine_streams else 0, now_us, C.byref(secs)))
        return secs.value

    # ---- lookups (Client.LookupResources / LookupSubjects, client/client.go:508-599) --------
    def _lookup(self, fn, args, requirement, revision):
        cs = _Consistency(requirement, 0, revision)
        n = C.c_size_t(0)
        cap = 1024
        while True:
            ids = np.zeros(cap, dtype=np.uint32)
            perms = np.zeros(cap, dtype=np.uint8)
            rc = fn(self._h, C.byref(cs), *args, ids.ctypes.data, perms.ctypes.data, cap, C.byref(n))
            if rc == GCK_E_CAPACITY and n.value > cap:
                cap = n.value  # the engine kept the result: the retry copies it out
                continue
            _check(rc)
            return ids[: n.value], perms[: n.value]

    def lookup_resources(self, resource_type: int, permission: int, subject_type: int, subject_relation: int,
                         subject_id: int, requirement: int = CONSISTENCY_MIN_LATENCY, revision: int = 0,
                         now_us: int = 0) -> Tuple[np.ndarray, np.ndarray]:
        """Ids (ascending) of the resource_type objects the subject has `permission` on, and
        their permissionship (PERM_HAS / PERM_CONDITIONAL)."""
        # an explicit evaluation time, so that a capacity retry is served from the engine's cache
        now_us = now_us or time.time_ns() // 1000
        return self._lookup(self._lib.gck_lookup_resources,
                            (resource_type, permission, subject_type, subject_relation, subject_id, now_us),
                            requirement, revision)

    def lookup_subjects(self, resource_type: int, resource_id: int, permission: int, subject_type: int,
                        subject_relation: int = ELLIPSIS, requirement: int = CONSISTENCY_MIN_LATENCY,
                        revision: int = 0, now_us: int = 0) -> Tuple[np.ndarray, np.ndarray]:
        """Ids (ascending) of the subject_type subjects that have `permission` on the resource;
        a wildcard grant is one id, ID_WILDCARD (last), instead of every subject of the type."""
        now_us = now_us or time.time_ns() // 1000
        return self._lookup(self._lib.gck_lookup_subjects,
                            (resource_type, resource_id, permission, subject_type, subject_relation, now_us),
                            requirement, revision)

    # ---- partitioned graphs (gck_part_*; driven by gochugaru_amd.partition) -----------------
    def set_partition(self, rank: int, world: int):
        _check(self._lib.gck_set_partition(self._h, rank, world))
        self.part_rank, self.part_world = rank, world

    @staticmethod
    def part_unique_id() -> bytes:
        """gck_part_unique_id: the RCCL communicator id rank 0 hands to every rank."""
        buf = (C.c_uint8 * PART_UNIQUE_ID_BYTES)()
        _check(load_library().gck_part_unique_id(buf))
        return bytes(buf)

    def part_init(self, unique_id: bytes):
        """gck_part_init: join the RCCL communicator of the partition (every rank, same id)."""
        assert len(unique_id) == PART_UNIQUE_ID_BYTES
        buf = (C.c_uint8 * PART_UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        _check(self._lib.gck_part_init(self._h, buf))

    def part_intern(self, transport: "Transport", type_ids, names, create: bool = False) -> np.ndarray:
        """gck_part_intern_with (collective): the ids every rank agrees on for (type, name) pairs,
        each interned by its owner rank (hash of the name)."""
        n = len(names)
        raw = [s.encode() if isinstance(s, str) else bytes(s) for s in names]
        types = np.ascontiguousarray(type_ids, dtype=np.uint16)
        lens = np.array([len(b) for b in raw], dtype=np.uint32)
        bufs = [C.create_string_buffer(b, len(b) + 1) for b in raw]
        ptrs = (C.c_char_p * max(1, n))(*[C.cast(b, C.c_char_p) for b in bufs])
        out = np.zeros(n, dtype=np.uint32)
        _check(self._lib.gck_part_intern_with(self._h, C.byref(transport), types.ctypes.data if n else None,
                                              C.cast(ptrs, C.c_void_p) if n else None,
                                              lens.ctypes.data if n else None, n, INTERN_CREATE if create else 0,
                                              out.ctypes.data if n else None))
        return out

    def interned_names(self, type_id: int) -> int:
        """Names the interner holds for a type (gck_interned_names)."""
        v = C.c_uint32(0)
        _check(self._lib.gck_interned_names(self._h, type_id, C.byref(v)))
        return v.value

    def part_add_tuples_text(self, transport: "Transport", text: str):
        """gck_part_add_tuples_text_with (collective): the export stream's text, the same on every
        rank; each keeps and interns what it owns."""
        b = text.encode()
        _check(self._lib.gck_part_add_tuples_text_with(self._h, C.byref(transport), b, len(b)))

    def part_load_snapshot_text(self, transport: "Transport", revision: int, text: str):
        self.begin_snapshot(revision)
        self.part_add_tuples_text(transport, text)
        self.commit_snapshot()

    def part_make_items(self, transport: "Transport", rels: Iterable) -> np.ndarray:
        """make_items on a partitioned engine (collective): the names resolved by their owners,
        so that every rank builds the same items."""
        rels = list(rels)
        items = np.zeros(len(rels), dtype=ITEM_DTYPE)
        types, names, where = [], [], []
        for i, r in enumerate(rels):
            rt = self.type_id(r.ResourceType)
            st = self.type_id(r.SubjectType)
            items[i]["resource_type"] = rt
            items[i]["permission"] = self.relation_id(rt, r.ResourceRelation)
            items[i]["subject_type"] = st
            items[i]["subject_relation"] = (ELLIPSIS if r.SubjectRelation in ("", "...")
                                            else self.relation_id(st, r.SubjectRelation))
            items[i]["resource_id"] = ID_ABSENT
            items[i]["subject_id"] = ID_WILDCARD if (st == TYPE_INVALID and r.SubjectID == "*") else ID_ABSENT
            if rt != TYPE_INVALID:
                types.append(rt), names.append(r.ResourceID), where.append((i, "resource_id"))
            if st != TYPE_INVALID:
                types.append(st), names.append(r.SubjectID), where.append((i, "subject_id"))
        ids = self.part_intern(transport, types, names, create=False)
        for (i, f), v in zip(where, ids):
            items[i][f] = v
        return items

    def part_check(self, d_items: int, n: int, d_perm: int, d_err: int, now_us: int = 0,
                   stream: Optional[int] = None):
        """gck_part_check: the whole partitioned check, exchanged over RCCL inside libgck."""
        _check(self._lib.gck_part_check(self._h, d_items, n, now_us, d_perm, d_err, stream))

    def part_check_with(self, transport: "Transport", d_items: int, n: int, d_perm: int, d_err: int, now_us: int = 0,
                        stream: Optional[int] = None):
        """gck_part_check_with: the partitioned check over the caller's transport (a
        gochugaru_amd.partition transport: gck_transport's callbacks)."""
        _check(self._lib.gck_part_check_with(self._h, C.byref(transport), d_items, n, now_us, d_perm, d_err, stream))

    def stats(self) -> Stats:
        s = _Stats()
        _check(self._lib.gck_last_stats(self._h, C.byref(s)))
        return Stats({k: getattr(s, k) for k, _ in _Stats._fields_})

    def reset_stats(self):
        _check(self._lib.gck_reset_stats(self._h))

    # ---- string-level convenience --------------------------------------------------------
    def make_request(self, rels: Iterable) -> Tuple[np.ndarray, List[str]]:
        """Items plus their check-time caveat contexts, as Client.Check builds them
        (client/client.go:244-258: Context = MustV1ProtoCaveat().GetContext(), i.e. the
        relationship's caveat context when it names a caveat). Identical contexts share a slot."""
        rels = list(rels)
        items = self.make_items(rels)
        contexts: List[str] = []
        slots = {}
        for i, r in enumerate(rels):
            ctx = r.MustV1ProtoCaveatContext() if hasattr(r, "MustV1ProtoCaveatContext") else None
            if ctx is None:
                continue
            js = _context_json(ctx)
            k = slots.get(js)
            if k is None:
                contexts.append(js)
                k = slots[js] = len(contexts)
            items[i]["context_slot"] = k
        return items, contexts

    def make_items(self, rels: Iterable) -> np.ndarray:
        """rel.Relationship-like items -> interned gck_item array (unknown names map to
        invalid ids so the device reports the per-item error; unknown ids map to ABSENT)."""
        rels = list(rels)
        items = np.zeros(len(rels), dtype=ITEM_DTYPE)
        by_type = {}
        for i, r in enumerate(rels):
            rt = self.type_id(r.ResourceType)
            st = self.type_id(r.SubjectType)
            items[i]["resource_type"] = rt
            items[i]["permission"] = self.relation_id(rt, r.ResourceRelation)
            items[i]["subject_type"] = st
            items[i]["subject_relation"] = (ELLIPSIS if r.SubjectRelation in ("", "...")
                                            else self.relation_id(st, r.SubjectRelation))
            if rt != TYPE_INVALID:
                by_type.setdefault(rt, ([], []))[0].append(i)
            if st != TYPE_INVALID:
                by_type.setdefault(st, ([], []))[1].append(i)
        for t, (ri, si) in by_type.items():
            if ri:
                items["resource_id"][ri] = self.intern(t, [rels[i].ResourceID for i in ri])
            if si:
                items["subject_id"][si] = self.intern(t, [rels[i].SubjectID for i in si])
        for i, r in enumerate(rels):
            if items[i]["resource_type"] == TYPE_INVALID:
                items[i]["resource_id"] = ID_ABSENT
            if items[i]["subject_type"] == TYPE_INVALID:
                items[i]["subject_id"] = ID_WILDCARD if r.SubjectID == "*" else ID_ABSENT
        return items


class PreparedRun:
    """A compiled submit/wait loop with its argument arrays built (Engine.prepare_batches)."""

    def __init__(self, engine, items, perms, errs, n, depth, streams, engine_streams, now_us, host):
        arr = lambda xs: (C.c_uint64 * max(1, len(xs)))(*[int(x) for x in xs])
        self._e, self._k, self._n, self._depth, self._now, self._host = engine, len(items), n, depth, now_us, host
        self._items, self._perms, self._errs = arr(items), arr(perms), arr(errs)
        self._streams = arr(streams or [0])
        self._flags = SUBMIT_ENGINE_STREAM if engine_streams else 0
        self._cs = _Consistency(CONSISTENCY_MIN_LATENCY, 0, 0)
        self._drv = _driver()
        self._submit = C.cast(engine._lib.gck_check_submit, C.c_void_p)
        self._wait = C.cast(engine._lib.gck_check_wait, C.c_void_p)
        self._secs = C.c_double(0.0)

    def run(self) -> float:
        """Runs the loop; returns its wall time in seconds (first submit to last wait)."""
        if self._host:
            _check(self._drv.gckd_run_host(self._submit, self._wait, self._e._h, C.byref(self._cs), self._k,
                                           self._items, self._perms, self._errs, self._n, self._depth, self._now,
                                           C.byref(self._secs)))
        else:
            _check(self._drv.gckd_run(self._submit, self._wait, self._e._h, C.byref(self._cs), self._k, self._items,
                                      self._perms, self._errs, self._n, self._depth, self._streams, self._flags,
                                      self._now, C.byref(self._secs)))
        return self._secs.value


class PreparedUniform:
    """A compiled submit/wait loop over uniform requests with its argument arrays built
    (Engine.prepare_uniform)."""

    def __init__(self, engine, headers, pairs, ns, packed, errs, err_cap, depth, now_us):
        arr = lambda xs: (C.c_uint64 * max(1, len(xs)))(*[int(x) for x in xs])
        self._e, self._k, self._depth, self._now, self._cap = engine, len(pairs), depth, now_us, err_cap
        self._hdrs = (Uniform * max(1, len(headers)))(
            *[Uniform(*h[:4], h[4] if len(h) > 4 else 0, 0) for h in headers])
        self._pairs, self._ns, self._packed, self._errs = arr(pairs), arr(ns), arr(packed), arr(errs)
        self.n_errs = (C.c_size_t * max(1, len(pairs)))()
        self._cs = _Consistency(CONSISTENCY_MIN_LATENCY, 0, 0)
        self._drv = _driver()
        self._submit = C.cast(engine._lib.gck_check_submit_uniform, C.c_void_p)
        self._wait = C.cast(engine._lib.gck_check_wait, C.c_void_p)
        self._secs = C.c_double(0.0)

    def run(self) -> float:
        """Runs the loop; returns its wall time in seconds (first submit to last wait)."""
        _check(self._drv.gckd_run_uniform(self._submit, self._wait, self._e._h, C.byref(self._cs), self._k,
                                          self._hdrs, self._pairs, self._ns, self._packed, self._errs, self._cap,
                                          self.n_errs, self._depth, self._now, C.byref(self._secs)))
        return self._secs.value


class Batch:
    """A submitted batch (gck_batch): wait() completes it exactly once."""

    def __init__(self, engine, handle, perm, err, items):
        self._engine, self._h = engine, handle
        self.perm, self.err = perm, err
        self._items = items  # host items stay alive until the wait (they are staged at submit anyway)
        self.revision = None  # the revision the batch ran on (gck_check_wait_at), after wait()

    def wait(self):
        if self._h is not None:
            h, self._h = self._h, None
            rev = C.c_uint64(0)
            _check(self._engine._lib.gck_check_wait_at(self._engine._h, h, C.byref(rev)))
            self.revision = rev.value
        return self.perm, self.err

    def __del__(self):
        try:
            self.wait()
        except Exception:
            pass


class UniformBatch:
    """A submitted uniform request (gck_check_submit_uniform): wait() completes it exactly once and
    returns (packed words, errors, evaluated revision)."""

    def __init__(self, engine, hdr, pairs, packed, errs):
        self._engine, self._hdr, self._pairs = engine, hdr, pairs
        self.packed, self.errs = packed, errs
        self._h = _P()
        self._n_errs = C.c_size_t(0)
        self.revision = None

    def wait(self):
        if self._h is not None and self._h.value is not None:
            h, self._h = self._h, None
            rev = C.c_uint64(0)
            _check(self._engine._lib.gck_check_wait_at(self._engine._h, h, C.byref(rev)))
            self.revision = rev.value
        m = min(self._n_errs.value, len(self.errs))
        return self.packed, self.errs[:m], self.revision

    def __del__(self):
        try:
            self.wait()
        except Exception:
            pass


def _context_json(ctx) -> str:
    if ctx is None:
        return ""
    if isinstance(ctx, (str, bytes)):
        return ctx.decode() if isinstance(ctx, bytes) else ctx
    return json.dumps(ctx, sort_keys=True, separators=(",", ":"))


class Contexts:
    """Check-time caveat contexts marshalled once for the C ABI (the `contexts` / `context_lens`
    arrays of gck_check_bulk_ctx): pass it wherever `contexts` is taken to reuse the arrays
    across calls (a caller that builds its requests ahead, as a Go caller's slices are)."""

    def __init__(self, contexts):
        self._enc = [_context_json(c).encode() for c in contexts]
        self.arr = (C.c_char_p * len(self._enc))(*self._enc)
        self.lens = (C.c_size_t * len(self._enc))(*[len(b) for b in self._enc])

    def __len__(self):
        return len(self._enc)


def _context_arrays(contexts):
    if contexts is None or len(contexts) == 0:
        return None, None, 0
    if not isinstance(contexts, Contexts):
        contexts = Contexts(contexts)
    return contexts.arr, contexts.lens, len(contexts)


PART_UNIQUE_ID_BYTES = 128  # GCK_PART_UNIQUE_ID_BYTES


def partition_owner(object_id: int, world: int) -> int:
    return load_library().gck_partition_owner(object_id, world)


def partition_owner_name(type_id: int, name: str, world: int) -> int:
    """The rank that owns (and interns) the named object on a partitioned graph."""
    b = name.encode()
    return load_library().gck_partition_owner_name(type_id, b, len(b), world)
