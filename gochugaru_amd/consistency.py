"""Consistency strategies — mirror of gochugaru's ``consistency`` package
(``consistency/consistency.go:15-77``).

A ``Strategy`` names which revision a check must be evaluated at. For the local evaluator
(SURVEY.md §5.1 item 11):

* ``MinLatency``  → the engine's current snapshot as-is;
* ``Full``        → the engine's head revision (the snapshot must be at the source's head);
* ``AtLeast(t)``  → the applied revision must be ≥ t, otherwise the request is rejected
  with ``Unavailable`` so the caller's retry applies (``client/client.go:196``);
* ``Snapshot(t)`` → only if the applied revision == t (no MVCC on the GPU in v1).

ZedTokens are opaque strings here; the engine only compares tokens it issued itself
(``gck_revision_token``), which encode the revision as a decimal integer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

FULLY_CONSISTENT = "fully_consistent"
MINIMIZE_LATENCY = "minimize_latency"
AT_LEAST_AS_FRESH = "at_least_as_fresh"
AT_EXACT_SNAPSHOT = "at_exact_snapshot"

# authzed-go pkg/requestmeta.RequestOverlapKey
REQUEST_OVERLAP_KEY = "io.spicedb.requestoverlapkey"


@dataclass(frozen=True)
class V1Consistency:
    requirement: str
    token: Optional[str] = None


@dataclass(frozen=True)
class Strategy:
    V1Consistency: V1Consistency


def Full() -> Strategy:
    return Strategy(V1Consistency(FULLY_CONSISTENT))


def MinLatency() -> Strategy:
    return Strategy(V1Consistency(MINIMIZE_LATENCY))


def AtLeast(revision: str) -> Strategy:
    return Strategy(V1Consistency(AT_LEAST_AS_FRESH, revision))


def Snapshot(revision: str) -> Strategy:
    return Strategy(V1Consistency(AT_EXACT_SNAPSHOT, revision))


@dataclass(frozen=True)
class Context:
    """Stand-in for Go's ``context.Context`` outgoing gRPC metadata."""
    metadata: Dict[str, str] = field(default_factory=dict)


Background = Context()


def WithOverlapKey(ctx: Optional[Context], key: str) -> Context:
    """``consistency/consistency.go:21-23``."""
    md = dict((ctx or Background).metadata)
    md[REQUEST_OVERLAP_KEY] = key
    return Context(md)
