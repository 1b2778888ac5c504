"""Client façade — host-side mirror of gochugaru's check family, answered locally.

Mirrors ``client/client.go``:

* ``Check``      (``:238-284``)  — items in request order; HAS_PERMISSION -> True, NO and
  CONDITIONAL -> False (``:274-277``); the first per-item error returns the results so far
  plus the error (``:279-280``); an empty request returns ``[]`` (``client_test.go:203-207``).
* ``CheckOne``   (``:129-135``), ``CheckAny`` (``:138-145``), ``CheckAll`` (``:148-160``),
  ``CheckIter``  (``:164-180``, chunks of 1000 by default, stops at the first error).
* ``checkOverlap`` (``:182-191``) — raises (Go panics) when ``WithOverlapRequired`` is set and
  the context carries no overlap key.
* ``retryRetriableErrors`` (``:193-211``) — exponential backoff 50 ms -> 2 s on Unavailable
  (``GCK_E_DEVICE``, ``GCK_E_REVISION``) and DeadlineExceeded; anything else is permanent.

The round-trip to SpiceDB (``:261-266``) is replaced by ``Engine.check_bulk`` on the GPU.
Go's ``(results, err)`` return pairs are kept as Python tuples so that callers and tests read
like the reference.
"""
from __future__ import annotations

import random
import time
from typing import Iterable, Iterator, List, Optional, Tuple

from . import consistency as _cs
from . import rel as _rel
from .consistency import Background, Context, Strategy
from .engine import (CONSISTENCY_AT_LEAST, CONSISTENCY_FULL, CONSISTENCY_MIN_LATENCY,
                     CONSISTENCY_SNAPSHOT, ELLIPSIS, GCK_E_DEVICE, GCK_E_NOT_FOUND, GCK_E_REVISION,
                     ID_ABSENT, ID_WILDCARD, ITEM_ERROR_MESSAGES, PERM_HAS, REL_INVALID, TYPE_INVALID, Engine,
                     GckError)

CHECK_ITER_CHUNK = 1000  # client/client.go:166


class OverlapKeyPanic(RuntimeError):
    """Go panics in checkOverlap (client/client.go:190)."""


class CheckItemError(Exception):
    """A CheckBulkPermissionsPair_Error turned into a Go error (client/client.go:279-280)."""


class Unavailable(Exception):
    pass


class InvalidArgument(Exception):
    pass


def WithOverlapRequired():
    """``client/client.go:84-86``."""
    def opt(c: "Client"):
        c.overlapRequired = True
    return opt


def _requirement(cs: Optional[Strategy]) -> Tuple[int, int]:
    if cs is None:
        return CONSISTENCY_MIN_LATENCY, 0
    v = cs.V1Consistency
    if v.requirement == _cs.MINIMIZE_LATENCY:
        return CONSISTENCY_MIN_LATENCY, 0
    if v.requirement == _cs.FULLY_CONSISTENT:
        return CONSISTENCY_FULL, 0
    try:
        rev = int(v.token)
    except (TypeError, ValueError):
        raise InvalidArgument(f"invalid zedtoken {v.token!r}")
    if v.requirement == _cs.AT_LEAST_AS_FRESH:
        return CONSISTENCY_AT_LEAST, rev
    if v.requirement == _cs.AT_EXACT_SNAPSHOT:
        return CONSISTENCY_SNAPSHOT, rev
    raise InvalidArgument(f"unknown consistency requirement {v.requirement!r}")


def _retriable(err: BaseException) -> bool:
    if isinstance(err, GckError):
        return err.code in (GCK_E_DEVICE, GCK_E_REVISION)  # gRPC Unavailable
    msg = str(err)
    return isinstance(err, (Unavailable, TimeoutError)) or \
        "retryable error" in msg or "try restarting transaction" in msg


def retryRetriableErrors(ctx: Context, fn, max_elapsed: float = 15 * 60):
    """``client/client.go:193-211``: backoff.ExponentialBackOff{Initial 50ms, Max 2s,
    default multiplier 1.5 and randomization 0.5}; gives up at the context deadline (or the
    backoff's default 15 min max elapsed time)."""
    interval = 0.05
    start = time.monotonic()
    deadline = getattr(ctx, "deadline", None)
    while True:
        try:
            return fn()
        except Exception as err:  # noqa: BLE001 — classified below
            if not _retriable(err):
                raise
            delay = interval * (1 + random.uniform(-0.5, 0.5))
            now = time.monotonic()
            limit = start + max_elapsed if deadline is None else deadline
            if now + delay > limit:
                raise
            time.sleep(delay)
            interval = min(interval * 1.5, 2.0)


class Client:
    """``client.Client`` (``client/client.go:101-105``) with a local GPU evaluator in place of
    the gRPC connection."""

    def __init__(self, engine: Engine, *opts, chunk: int = 65536):
        self.engine = engine
        self.overlapRequired = False
        self.chunk = chunk
        for o in opts:
            o(self)

    @classmethod
    def NewWithOpts(cls, engine: Engine, *opts) -> Tuple["Client", Optional[Exception]]:
        """``client/client.go:65-75``."""
        return cls(engine, *opts), None

    # ---- overlap guard -------------------------------------------------------------------
    def checkOverlap(self, ctx: Optional[Context]):
        if self.overlapRequired:
            md = (ctx or Background).metadata
            if md.get(_cs.REQUEST_OVERLAP_KEY):
                return
            raise OverlapKeyPanic("failed to configure required overlap key for request")

    # ---- the check family ----------------------------------------------------------------
    def Check(self, ctx: Optional[Context], cs: Optional[Strategy], *rs) -> Tuple[List[bool], Optional[Exception]]:
        self.checkOverlap(ctx)
        rels = [r.Relationship() for r in rs]
        try:
            requirement, revision = _requirement(cs)

            def attempt():
                # interned per attempt, like the server resolving names at evaluation time: an
                # object a Watch batch created while this request waited is found on the retry
                items, contexts = self.engine.make_request(rels)
                return self.engine.check_bulk(items, requirement, revision, contexts=contexts)
            perm, err = retryRetriableErrors(ctx or Background, attempt)
        except Exception as e:  # noqa: BLE001 — Go returns (nil, err)
            return None, e
        results: List[bool] = []
        for p, e in zip(perm.tolist(), err.tolist()):
            if e:
                return results, CheckItemError(ITEM_ERROR_MESSAGES.get(e, f"item error {e}"))
            results.append(p == PERM_HAS)
        return results, None

    def CheckOne(self, ctx, cs, r) -> Tuple[bool, Optional[Exception]]:
        results, err = self.Check(ctx, cs, r)
        if err is not None:
            return False, err
        return results[0], None

    def CheckAny(self, ctx, cs, *rs) -> Tuple[bool, Optional[Exception]]:
        results, err = self.Check(ctx, cs, *rs)
        if err is not None:
            return False, err
        return True in results, None

    def CheckAll(self, ctx, cs, *rs) -> Tuple[bool, Optional[Exception]]:
        results, err = self.Check(ctx, cs, *rs)
        if err is not None:
            return False, err
        for r in results:
            if not r:
                return False, None
        return True, None

    def CheckIter(self, ctx, cs, rs: Iterable, chunk: int = CHECK_ITER_CHUNK) -> Iterator[Tuple[bool, Optional[Exception]]]:
        buf = []
        for r in rs:
            buf.append(r)
            if len(buf) == chunk:
                ok = yield from self._iter_chunk(ctx, cs, buf)
                if not ok:
                    return
                buf = []
        if buf:
            yield from self._iter_chunk(ctx, cs, buf)

    def _iter_chunk(self, ctx, cs, items):
        checks, err = self.Check(ctx, cs, *items)
        if err is not None:
            yield False, err
            return False
        for c in checks:
            yield c, None
        return True

    # ---- lookups (client/client.go:501-599) ------------------------------------------------
    def LookupResources(self, ctx: Optional[Context], cs: Optional[Strategy], permission: str,
                        subject: str) -> Iterator[Tuple[str, Optional[Exception]]]:
        """``client/client.go:508-552``: yields the ids of the objects of ``permission``'s type
        ("document#reader") on which ``subject`` ("user:jimmy" or "team:admin#member") has the
        permission (HAS or CONDITIONAL, as SpiceDB streams both); stops at the first error."""
        self.checkOverlap(ctx)
        try:
            subj_type, subj_id, subj_rel = _rel.ParseObjectSet(subject)
            obj_type, obj_rel = _rel.ParseTypedRelation(permission)
            requirement, revision = _requirement(cs)
            eng = self.engine
            rt = eng.type_id(obj_type)
            st = eng.type_id(subj_type)
            perm = eng.relation_id(rt, obj_rel)
            srel = ELLIPSIS if subj_rel in ("", "...") else eng.relation_id(st, subj_rel)
            if TYPE_INVALID in (rt, st) or REL_INVALID in (perm, srel):
                raise GckError(GCK_E_NOT_FOUND, "object definition or relation not found")
            sid = int(eng.intern(st, [subj_id])[0])  # unknown ids stay ABSENT: wildcards still match
            ids, _ = retryRetriableErrors(ctx or Background, lambda: eng.lookup_resources(
                rt, perm, st, srel, sid, requirement, revision))
            names = [eng.object_name(rt, int(i)) for i in ids]
        except Exception as e:  # noqa: BLE001 — Go yields ("", err) and stops
            yield "", e
            return
        for n in names:
            yield n, None

    def LookupSubjects(self, ctx: Optional[Context], cs: Optional[Strategy], resource: str, permission: str,
                       subject: str) -> Iterator[Tuple[str, Optional[Exception]]]:
        """``client/client.go:560-599``: yields the ids of the subjects of type ``subject``
        ("user" or "team#member") that have ``permission`` on ``resource`` ("document:README");
        a wildcard grant yields "*" once (as SpiceDB streams it), not every subject of the type."""
        self.checkOverlap(ctx)
        try:
            res_type, res_id, _ = _rel.ParseObjectSet(resource)
            subj_type, subj_rel, _ = _rel._cut(subject, "#")
            requirement, revision = _requirement(cs)
            eng = self.engine
            rt = eng.type_id(res_type)
            st = eng.type_id(subj_type)
            perm = eng.relation_id(rt, permission)
            srel = ELLIPSIS if subj_rel in ("", "...") else eng.relation_id(st, subj_rel)
            if TYPE_INVALID in (rt, st) or REL_INVALID in (perm, srel):
                raise GckError(GCK_E_NOT_FOUND, "object definition or relation not found")
            rid = int(eng.intern(rt, [res_id])[0])
            ids, _ = retryRetriableErrors(ctx or Background, lambda: eng.lookup_subjects(
                rt, rid, perm, st, srel, requirement, revision)) if rid != ID_ABSENT else ([], [])
            # a wildcard grant is the subject "*" (SpiceDB's LookupSubjects result for `type:*`)
            names = ["*" if int(i) == ID_WILDCARD else eng.object_name(st, int(i)) for i in ids]
        except Exception as e:  # noqa: BLE001
            yield "", e
            return
        for n in names:
            yield n, None

    # ---- snapshot plumbing (ReadSchema + ExportRelationships at its revision) -------------
    def LoadSnapshot(self, schema: str, revision: int, relationships: Iterable) -> None:
        """Ingest the output of ``ReadSchema`` (client/client.go:416-422) and
        ``ExportRelationships`` at that revision (client/client.go:472-499)."""
        self.engine.load_schema(schema)
        lines = "\n".join(r.String() if hasattr(r, "String") else str(r) for r in relationships)
        self.engine.load_snapshot_text(revision, lines)

    def SetHeadRevision(self, revision: int) -> None:
        """The source's head revision that ``consistency.Full()`` must reach (consistency/
        consistency.go:25-35): ReadSchema's ReadAt token (client/client.go:416-422) or a Watch
        checkpoint. Until ApplyUpdates reaches it, a Full check is Unavailable and retried."""
        self.engine.set_head_revision(revision)

    _UPDATE_OPS = {_rel.UpdateCreate: "CREATE", _rel.UpdateTouch: "TOUCH", _rel.UpdateDelete: "DELETE"}

    def ApplyUpdates(self, revision: int, updates: Iterable) -> None:
        """Fold one Watch response into the local snapshot: the ``rel.Update`` values that
        ``UpdatesSinceRevision`` yields (client/client.go:370-413, rel/relationship.go:291-301)
        up to the response's ChangesThrough revision (which gochugaru's iterator drops; the
        caller passes it here). ``UpdateUnknown`` is rejected, as SpiceDB never sends it."""
        lines = []
        for u in updates:
            op = self._UPDATE_OPS.get(u.UpdateType)
            if op is None:
                raise InvalidArgument(f"unknown update type {u.UpdateType!r}")
            lines.append(op + " " + u.Relationship.String())
        self.engine.apply_updates_text(revision, "\n".join(lines))
