"""Relationship value type — host-side mirror of gochugaru's ``rel`` package.

Mirrors ``rel/relationship.go`` (``Relationship`` ``:28-38``, ``String`` ``:51-90``,
``WithCaveat``/``WithExpiration`` ``:93-120``, ``FromTriple``/``FromTuple`` ``:220-265``,
``UpdateType``/``Update`` ``:267-306``) and ``rel/strings.go`` (``ParseObjectSet`` ``:19-28``,
``ParseTypedRelation`` ``:31-38``). Method and error names follow the Go API so that callers
(and the parity tests) read like the reference's own code.

A ``Relationship`` is both the check item (``ResourceRelation`` = the permission,
``client/client.go:244-258``) and the snapshot/ingest record (``client/client.go:472-499``).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Any, Dict, Optional


class RelError(ValueError):
    pass


# rel/relationship.go:17-24
ErrInvalidResource = RelError("invalid resource")
ErrInvalidRelation = RelError("invalid relation")
ErrInvalidSubject = RelError("invalid subject")
# rel/strings.go:8-11
ErrInvalidObjectString = RelError(
    "invalid object string: must be in form `objectType:objectID#optionalRelation`")
ErrInvalidTypedRelationString = RelError(
    "invalid typed permission string: must be in form `objectType#relation`")


def _cut(s: str, sep: str):
    i = s.find(sep)
    if i < 0:
        return s, "", False
    return s[:i], s[i + len(sep):], True


def _json_value(v: Any) -> str:
    # structpb.NewStruct stores numbers as float64; protojson prints integral doubles as ints.
    if isinstance(v, bool) or v is None:
        return json.dumps(v)
    if isinstance(v, (int, float)):
        f = float(v)
        return str(int(f)) if f.is_integer() and abs(f) < 1e21 else repr(f)
    if isinstance(v, str):
        return json.dumps(v, ensure_ascii=False)
    if isinstance(v, dict):
        return "{" + ",".join(f"{json.dumps(k, ensure_ascii=False)}:{_json_value(v[k])}"
                              for k in sorted(v)) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_json_value(x) for x in v) + "]"
    raise TypeError(f"unsupported caveat context value {v!r}")


def _rfc3339nano(t: datetime) -> str:
    # Go time.RFC3339Nano: fractional seconds with trailing zeros removed, Z for UTC.
    t = t.astimezone(timezone.utc)
    s = t.strftime("%Y-%m-%dT%H:%M:%S")
    if t.microsecond:
        s += ("." + f"{t.microsecond:06d}").rstrip("0")
    return s + "Z"


@dataclass
class Relationship:
    """``rel.Relationship`` (``rel/relationship.go:28-38``)."""

    ResourceType: str = ""
    ResourceID: str = ""
    ResourceRelation: str = ""
    SubjectType: str = ""
    SubjectID: str = ""
    SubjectRelation: str = ""
    CaveatName: str = ""
    CaveatContext: Optional[Dict[str, Any]] = None
    Expiration: Optional[datetime] = None

    # rel.Interface (:26, :40)
    def Relationship(self) -> "Relationship":
        return self

    def Permission(self) -> str:
        return self.ResourceRelation

    def HasCaveat(self) -> bool:
        return self.CaveatName != ""

    def HasExpiration(self) -> bool:
        # :45-47 — a zero time (Go's time.Time{}) counts as no expiration
        return self.Expiration is not None and self.Expiration != ZERO_TIME

    def Caveat(self):
        return self.CaveatName, self.CaveatContext, self.HasCaveat()

    def String(self) -> str:
        """Canonical text form, ``rel/relationship.go:51-90``."""
        b = [self.ResourceType, ":", self.ResourceID, "#", self.ResourceRelation, "@",
             self.SubjectType, ":", self.SubjectID]
        if self.SubjectRelation:
            b += ["#", self.SubjectRelation]
        if self.HasCaveat():
            b += ["[", self.CaveatName]
            if self.CaveatContext:
                for k in self.CaveatContext:
                    if not isinstance(k, str):
                        raise RelError("caveat created with non-utf8 context key")
                b += [":", _json_value(self.CaveatContext)]
            b.append("]")
        if self.HasExpiration():
            b += ["[expiration:", _rfc3339nano(self.Expiration), "]"]
        return "".join(b)

    __str__ = String

    def WithCaveat(self, name: str, context: Optional[Dict[str, Any]]) -> "Relationship":
        return Relationship(self.ResourceType, self.ResourceID, self.ResourceRelation,
                            self.SubjectType, self.SubjectID, self.SubjectRelation,
                            name, context, self.Expiration)

    def WithExpiration(self, expiration: datetime) -> "Relationship":
        return Relationship(self.ResourceType, self.ResourceID, self.ResourceRelation,
                            self.SubjectType, self.SubjectID, self.SubjectRelation,
                            self.CaveatName, self.CaveatContext, expiration)

    def MustV1ProtoCaveatContext(self) -> Optional[Dict[str, Any]]:
        """The check-time context: ``client/client.go:257`` sends
        ``MustV1ProtoCaveat().GetContext()`` (``rel/relationship.go:174-188``)."""
        if not self.HasCaveat():
            return None
        for k in (self.CaveatContext or {}):
            if not isinstance(k, str):
                raise RelError("caveat created with non-utf8 context key")
        return dict(self.CaveatContext or {})


ZERO_TIME = datetime(1, 1, 1, tzinfo=timezone.utc)


def FromTuple(resource: str, subject: str) -> Relationship:
    """``rel/relationship.go:236-265``; raises the same sentinel errors."""
    r = Relationship()
    resource, r.ResourceRelation, found = _cut(resource, "#")
    if not found or r.ResourceRelation == "":
        raise ErrInvalidRelation
    r.ResourceType, r.ResourceID, found = _cut(resource, ":")
    if not found:
        raise ErrInvalidResource
    subject, r.SubjectRelation, _ = _cut(subject, "#")
    r.SubjectType, r.SubjectID, found = _cut(subject, ":")
    if not found:
        raise ErrInvalidSubject
    return r


def FromTriple(resource: str, relation: str, subject: str) -> Relationship:
    """``rel/relationship.go:228-230``."""
    return FromTuple(resource + "#" + relation, subject)


MustFromTriple = FromTriple  # panics in Go == raises here
MustFromTuple = FromTuple


@dataclass
class Object:
    """``rel.Object`` (``rel/relationship.go:198-206``)."""
    Typ: str
    ID: str
    Relation: str = ""

    def Object(self) -> "Object":
        return self


def FromObjects(resource, subject) -> Relationship:
    r, s = resource.Object(), subject.Object()
    return Relationship(r.Typ, r.ID, r.Relation, s.Typ, s.ID, s.Relation)


# rel/relationship.go:267-294
UpdateUnknown, UpdateCreate, UpdateDelete, UpdateTouch = 0, 1, 2, 3


@dataclass
class Update:
    UpdateType: int
    Relationship: Relationship = field(default_factory=Relationship)


def ParseObjectSet(obj: str):
    """``rel/strings.go:19-28`` → (type, id, relation)."""
    typ, oid, found = _cut(obj, ":")
    if not found:
        raise ErrInvalidObjectString
    oid, rel, _ = _cut(oid, "#")
    return typ, oid, rel


def ParseTypedRelation(perm: str):
    """``rel/strings.go:31-38`` → (type, relation)."""
    typ, rel, found = _cut(perm, "#")
    if not found:
        raise ErrInvalidTypedRelationString
    return typ, rel


def ParseRFC3339(s: str) -> datetime:
    """RFC 3339 (Go time.RFC3339Nano accepts any fraction length; Python 3.10's
    fromisoformat does not)."""
    import re

    m = re.fullmatch(r"(\d{4}-\d{2}-\d{2}[Tt]\d{2}:\d{2}:\d{2})(?:\.(\d+))?([Zz]|[+-]\d{2}:\d{2})", s)
    if not m:
        raise RelError(f"invalid expiration timestamp {s!r}")
    base = datetime.fromisoformat(m.group(1).replace("t", "T"))
    frac = (m.group(2) or "")[:6].ljust(6, "0")
    tz = m.group(3)
    if tz in ("Z", "z"):
        tzinfo = timezone.utc
    else:
        from datetime import timedelta
        sign = -1 if tz[0] == "-" else 1
        tzinfo = timezone(sign * timedelta(hours=int(tz[1:3]), minutes=int(tz[4:6])))
    return base.replace(microsecond=int(frac), tzinfo=tzinfo)


def Parse(line: str) -> Relationship:
    """Inverse of ``String``: parse the canonical text form (fixture/snapshot line format)."""
    import re

    line = line.strip()
    exp = None
    m = re.search(r"\[expiration:([^\]]+)\]$", line)
    if m:
        exp = ParseRFC3339(m.group(1))
        line = line[: m.start()]
    cav, ctx = "", None
    m = re.search(r"\[([A-Za-z_][A-Za-z0-9_/]*)(?::(\{.*\}))?\]$", line)
    if m:
        cav = m.group(1)
        ctx = json.loads(m.group(2)) if m.group(2) else None
        line = line[: m.start()]
    res, subj, found = _cut(line, "@")
    if not found:
        raise ErrInvalidSubject
    r = FromTuple(res, subj)
    r.CaveatName, r.CaveatContext, r.Expiration = cav, ctx, exp
    return r
