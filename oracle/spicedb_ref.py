"""TEST INFRASTRUCTURE ONLY — the pure-Python parity oracle for batched permission checks.

Nothing in the product (``gochugaru_amd``) imports this module. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it, and only as the
checker.

What it restates
----------------
The reference (authzed/gochugaru) computes no permission itself: ``Client.Check``
(``client/client.go:238-284``) ships items to SpiceDB's ``CheckBulkPermissions`` and maps
``Permissionship == HAS_PERMISSION`` to ``true`` (``client/client.go:271-283``). The arithmetic
on the north-star path therefore lives in the SpiceDB *server* (not present in
``/root/reference`` and not a Go dependency of it). This module restates the
server's published check semantics as a small recursive interpreter:

* ``Checker._dispatch``        — SpiceDB dispatch: depth budget, identity filter
  (SURVEY §5.1 items 3, 9).
* ``Checker._check_direct``    — ``checkDirect``: exact subject, wildcard, userset
  re-dispatch (§5.1 item 3).
* ``Checker._eval``            — rewrite evaluation: union / intersection / exclusion /
  computed userset / tuple-to-userset ``->``, ``.any``, ``.all`` / ``nil`` (§5.1 items 4-6).
* tri-state caveat algebra Y/N/C (§5.1 item 7), expiration (§5.1 item 8).

Parity pinning
--------------
Pinned against every known answer the reference's own tests hold for this path:
``client/client_test.go:141-216`` (exampleSchema checks), the README founders example
(``README.md:71-88``) and the canonical ``rel.String`` goldens
(``rel/relationship_test.go:31-100``) — see ``tests/golden/`` and ``tests/test_oracle.py``.
Everything beyond union/computed-userset (arrows, intersection, exclusion, wildcards,
caveats, expiration, depth) is **parity unpinned** by the reference: those rules follow
SpiceDB's public documentation as restated in SURVEY.md §5.1 and are cross-checked against
the independent C restatement in ``oracle/check_oracle.c``.

Defined semantics where SpiceDB is nondeterministic (DESIGN.md §"Semantics"):
union: Y > ERR > C > N; intersection: N > ERR > C > Y; exclusion: base N or any
subtracted Y -> N, else ERR, else C, else Y.
"""
from __future__ import annotations

import datetime
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

ELLIPSIS = "..."
WILDCARD = "*"

# Permissionship values as in authzed v1 CheckPermissionResponse.Permissionship
NO = 1
HAS = 2
COND = 3
ERR = -1  # per-item error (max depth) in the oracle's internal tri-state+error lattice

# per-item error codes (mirrors include/gck.h GCK_ITEM_ERR_*)
ITEM_OK = 0
ITEM_ERR_MAX_DEPTH = 1
ITEM_ERR_UNKNOWN_PERMISSION = 2
ITEM_ERR_UNKNOWN_TYPE = 3
ITEM_ERR_UNKNOWN_SUBJECT_RELATION = 4
ITEM_ERR_WILDCARD_SUBJECT = 5
ITEM_ERR_CAVEAT_EVAL = 6  # a caveat met by the check failed to evaluate under its context

DEFAULT_MAX_DEPTH = 50


class SchemaError(ValueError):
    pass


# ----------------------------------------------------------------------------------------
# Schema DSL (subset of the SpiceDB schema language)
# ----------------------------------------------------------------------------------------

_TOKEN_RE = re.compile(
    r"""
    (?P<ws>\s+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<arrow>->)
  | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<num>\d+(?:\.\d+)?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:/[A-Za-z_][A-Za-z0-9_]*)*)
  | (?P<op>==|!=|<=|>=|&&|\|\||[{}()\[\]:#|=+\-&.,*<>!;/%?])
""",
    re.VERBOSE | re.DOTALL,
)


def _tokenize(text: str) -> List[Tuple[str, str]]:
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m:
            raise SchemaError(f"unexpected character {text[pos]!r} at offset {pos}")
        kind = m.lastgroup
        val = m.group(kind)
        pos = m.end()
        if kind in ("ws", "lcomment", "bcomment"):
            continue
        out.append((kind, val))
    out.append(("eof", ""))
    return out


@dataclass
class AllowedSubject:
    type: str
    relation: str = ELLIPSIS  # "..." for a concrete object
    wildcard: bool = False
    caveat: Optional[str] = None
    expiration: bool = False


@dataclass
class Expr:
    op: str  # union | intersect | exclude | nil | computed | arrow
    children: List["Expr"] = field(default_factory=list)
    name: str = ""  # computed relation, or arrow target
    tupleset: str = ""  # arrow tupleset relation
    func: str = "any"  # arrow: any | all


@dataclass
class Relation:
    name: str
    allowed: Optional[List[AllowedSubject]] = None  # relation
    expr: Optional[Expr] = None  # permission

    @property
    def is_permission(self) -> bool:
        return self.expr is not None


@dataclass
class Definition:
    name: str
    relations: Dict[str, Relation] = field(default_factory=dict)


@dataclass
class Caveat:
    name: str
    params: Dict[str, str]
    expr_text: str
    expr: Any = None


class Schema:
    def __init__(self, text: str):
        self.defs: Dict[str, Definition] = {}
        self.caveats: Dict[str, Caveat] = {}
        self.uses: List[str] = []
        self._toks = _tokenize(text)
        self._i = 0
        self._text = text
        self._parse()
        self._validate()

    # -- token helpers ---------------------------------------------------------------
    def _peek(self, k=0):
        return self._toks[self._i + k]

    def _next(self):
        t = self._toks[self._i]
        self._i += 1
        return t

    def _expect(self, val=None, kind=None):
        t = self._next()
        if (val is not None and t[1] != val) or (kind is not None and t[0] != kind):
            raise SchemaError(f"expected {val or kind}, got {t[1]!r}")
        return t

    def _accept(self, val):
        if self._peek()[1] == val and self._peek()[0] in ("op", "ident", "arrow"):
            self._i += 1
            return True
        return False

    # -- grammar ------------------------------------------------------------------------
    def _parse(self):
        while self._peek()[0] != "eof":
            kw = self._expect(kind="ident")[1]
            if kw == "definition":
                self._parse_definition()
            elif kw == "caveat":
                self._parse_caveat()
            elif kw == "use":
                self.uses.append(self._expect(kind="ident")[1])
            else:
                raise SchemaError(f"unexpected keyword {kw!r}")

    def _parse_definition(self):
        name = self._expect(kind="ident")[1]
        if name in self.defs:
            raise SchemaError(f"duplicate definition {name!r}")
        d = Definition(name)
        self._expect("{")
        while not self._accept("}"):
            kw = self._expect(kind="ident")[1]
            rname = self._expect(kind="ident")[1]
            if rname in d.relations:
                raise SchemaError(f"duplicate relation {name}#{rname}")
            if kw == "relation":
                self._expect(":")
                allowed = [self._parse_allowed()]
                while self._accept("|"):
                    allowed.append(self._parse_allowed())
                d.relations[rname] = Relation(rname, allowed=allowed)
            elif kw == "permission":
                self._expect("=")
                d.relations[rname] = Relation(rname, expr=self._parse_expr())
            else:
                raise SchemaError(f"unexpected {kw!r} in definition {name}")
            self._accept(";")
        self.defs[name] = d

    def _parse_allowed(self) -> AllowedSubject:
        a = AllowedSubject(self._expect(kind="ident")[1])
        if self._accept(":"):
            self._expect("*")
            a.wildcard = True
        elif self._accept("#"):
            a.relation = self._expect(kind="ident")[1]
        if self._peek()[1] == "with":
            self._next()
            w = self._expect(kind="ident")[1]
            if w == "expiration":
                a.expiration = True
            else:
                a.caveat = w
                if self._peek()[1] == "and":
                    self._next()
                    if self._expect(kind="ident")[1] != "expiration":
                        raise SchemaError("expected 'expiration' after 'and'")
                    a.expiration = True
        return a

    # precedence (SpiceDB schemadsl parser, binaryOpDefinitions): '-' loosest, then '&',
    # then '+' tightest; all left-associative. Parity UNPINNED: synthetic schemas use
    # explicit parentheses wherever operators mix.
    def _parse_expr(self) -> Expr:
        return self._parse_binary(0)

    _LEVELS = [("-", "exclude"), ("&", "intersect"), ("+", "union")]

    def _parse_binary(self, level: int) -> Expr:
        if level == len(self._LEVELS):
            return self._parse_primary()
        sym, op = self._LEVELS[level]
        left = self._parse_binary(level + 1)
        while self._peek() == ("op", sym):
            self._next()
            right = self._parse_binary(level + 1)
            if op in ("union", "intersect") and left.op == op:
                left.children.append(right)  # flatten associative chains
            elif op == "exclude" and left.op == "exclude":
                left.children.append(right)  # (a - b) - c == a - b - c
            else:
                left = Expr(op, [left, right])
        return left

    def _parse_primary(self) -> Expr:
        if self._accept("("):
            e = self._parse_expr()
            self._expect(")")
            return e
        name = self._expect(kind="ident")[1]
        if name == "nil":
            return Expr("nil")
        if self._peek()[0] == "arrow":
            self._next()
            target = self._expect(kind="ident")[1]
            return Expr("arrow", tupleset=name, name=target, func="any")
        if self._accept("."):
            func = self._expect(kind="ident")[1]
            if func not in ("any", "all"):
                raise SchemaError(f"unknown arrow function {func!r}")
            self._expect("(")
            target = self._expect(kind="ident")[1]
            self._expect(")")
            return Expr("arrow", tupleset=name, name=target, func=func)
        return Expr("computed", name=name)

    def _parse_caveat(self):
        name = self._expect(kind="ident")[1]
        self._expect("(")
        params = {}
        while not self._accept(")"):
            pname = self._expect(kind="ident")[1]
            ptype = self._expect(kind="ident")[1]
            # generic types like list<string> / map<int>
            if self._accept("<"):
                inner = self._expect(kind="ident")[1]
                self._expect(">")
                ptype = f"{ptype}<{inner}>"
            params[pname] = ptype
            self._accept(",")
        self._expect("{")
        depth, start = 1, self._i
        while depth:
            t = self._next()
            if t[0] == "eof":
                raise SchemaError("unterminated caveat body")
            if t[1] == "{":
                depth += 1
            elif t[1] == "}":
                depth -= 1
        body = self._toks[start : self._i - 1]
        c = Caveat(name, params, " ".join(v for _, v in body))
        c.expr = CelParser(body, params).parse()
        self.caveats[name] = c

    def _validate(self):
        for d in self.defs.values():
            for r in d.relations.values():
                if r.allowed is not None:
                    for a in r.allowed:
                        if a.type not in self.defs:
                            raise SchemaError(f"{d.name}#{r.name}: unknown type {a.type!r}")
                        if a.relation != ELLIPSIS and a.relation not in self.defs[a.type].relations:
                            raise SchemaError(f"{d.name}#{r.name}: unknown relation {a.type}#{a.relation}")
                        if a.caveat and a.caveat not in self.caveats:
                            raise SchemaError(f"{d.name}#{r.name}: unknown caveat {a.caveat!r}")
                else:
                    self._validate_expr(d, r.expr)

    def _validate_expr(self, d: Definition, e: Expr):
        if e.op == "computed":
            if e.name not in d.relations:
                raise SchemaError(f"{d.name}: unknown relation/permission {e.name!r}")
        elif e.op == "arrow":
            ts = d.relations.get(e.tupleset)
            if ts is None or ts.is_permission:
                raise SchemaError(f"{d.name}: arrow tupleset {e.tupleset!r} must be a relation")
            if any(a.wildcard for a in ts.allowed):
                raise SchemaError(f"{d.name}: arrow tupleset {e.tupleset!r} allows a wildcard")
            if not any(e.name in self.defs[a.type].relations for a in ts.allowed):
                raise SchemaError(f"{d.name}: arrow target {e.name!r} exists on no subject type")
        for c in e.children:
            self._validate_expr(d, c)

    # -- lookups ------------------------------------------------------------------------
    def relation(self, typ: str, rel: str) -> Optional[Relation]:
        d = self.defs.get(typ)
        return None if d is None else d.relations.get(rel)


# ----------------------------------------------------------------------------------------
# CEL subset with partial evaluation (caveats)
# ----------------------------------------------------------------------------------------

class _Unknown:
    """A value that depends on a missing caveat parameter (SpiceDB partial evaluation)."""

    def __repr__(self):
        return "UNKNOWN"


UNKNOWN = _Unknown()


class CelParser:
    """Recursive-descent parser for a CEL subset: literals, identifiers, member access on
    maps, lists, ! - unary, * / %, + -, comparisons, in, &&, ||, ?:."""

    def __init__(self, toks, params=None):
        self.t = list(toks) + [("eof", "")]
        self.i = 0
        self.conv = {k: v for k, v in (params or {}).items() if v in ("timestamp", "duration", "ipaddress")}

    def args(self):
        out = []
        while self.peek() != ("op", ")"):
            if self.peek()[0] == "eof":
                raise SchemaError("unterminated argument list")
            out.append(self.ternary())
            if self.peek() == ("op", ","):
                self.nxt()
            elif self.peek() != ("op", ")"):
                raise SchemaError("expected ',' or ')'")
        self.nxt()
        return out

    def peek(self):
        return self.t[self.i]

    def nxt(self):
        v = self.t[self.i]
        self.i += 1
        return v

    def parse(self):
        e = self.ternary()
        if self.peek()[0] != "eof":
            raise SchemaError(f"trailing tokens in caveat expression: {self.peek()[1]!r}")
        return e

    def ternary(self):
        c = self.lor()
        if self.peek() == ("op", "?"):
            self.nxt()
            a = self.ternary()
            if self.nxt() != ("op", ":"):
                raise SchemaError("expected ':' in conditional")
            b = self.ternary()
            return ("?:", c, a, b)
        return c

    def lor(self):
        e = self.land()
        while self.peek() == ("op", "||"):
            self.nxt()
            e = ("||", e, self.land())
        return e

    def land(self):
        e = self.rel()
        while self.peek() == ("op", "&&"):
            self.nxt()
            e = ("&&", e, self.rel())
        return e

    def rel(self):
        e = self.add()
        while self.peek()[1] in ("==", "!=", "<", "<=", ">", ">=") or self.peek() == ("ident", "in"):
            op = self.nxt()[1]
            e = (op, e, self.add())
        return e

    def add(self):
        e = self.mul()
        while self.peek() in (("op", "+"), ("op", "-")):
            op = self.nxt()[1]
            e = (op, e, self.mul())
        return e

    def mul(self):
        e = self.unary()
        while self.peek() in (("op", "*"), ("op", "/"), ("op", "%")):
            op = self.nxt()[1]
            e = (op, e, self.unary())
        return e

    def unary(self):
        if self.peek() == ("op", "!"):
            self.nxt()
            return ("!", self.unary())
        if self.peek() == ("op", "-"):
            self.nxt()
            return ("neg", self.unary())
        return self.member()

    def member(self):
        e = self.primary()
        while True:
            if self.peek() == ("op", "."):
                self.nxt()
                f = self.nxt()[1]
                if self.peek() == ("op", "("):  # method call
                    self.nxt()
                    e = ("call", f, True, [e] + self.args())
                else:
                    e = (".", e, f)
            elif self.peek() == ("op", "["):
                self.nxt()
                k = self.ternary()
                if self.nxt() != ("op", "]"):
                    raise SchemaError("expected ']'")
                e = ("[]", e, k)
            else:
                return e

    def primary(self):
        kind, v = self.nxt()
        if kind == "num":
            return ("lit", float(v) if "." in v else int(v))
        if kind == "str":
            return ("lit", _unescape(v[1:-1]))
        if kind == "ident":
            if v == "true":
                return ("lit", True)
            if v == "false":
                return ("lit", False)
            if v == "null":
                return ("lit", None)
            if self.peek() == ("op", "("):  # global function, or the has() macro
                self.nxt()
                a = self.args()
                if v == "has":
                    if len(a) != 1 or a[0][0] != ".":
                        raise SchemaError("has() takes one field selection")
                    return ("has", a[0][1], a[0][2])
                return ("call", v, False, a)
            return ("var", v, self.conv.get(v))
        if (kind, v) == ("op", "("):
            e = self.ternary()
            if self.nxt() != ("op", ")"):
                raise SchemaError("expected ')'")
            return e
        if (kind, v) == ("op", "["):
            items = []
            while self.peek() != ("op", "]"):
                items.append(self.ternary())
                if self.peek() == ("op", ","):
                    self.nxt()
            self.nxt()
            return ("list", items)
        raise SchemaError(f"unexpected token {v!r} in caveat expression")


_ESCAPES = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", "'": "'", '"': '"'}
_ESCAPE_RE = re.compile(r"\\(x[0-9A-Fa-f]{2}|u[0-9A-Fa-f]{4}|.)", re.DOTALL)


def _unescape(body: str) -> str:
    """CEL string literal body: the common escapes, \\xHH and \\uXXXX as code points; other
    characters (non-ASCII included) stand for themselves."""
    def sub(m):
        t = m.group(1)
        if t[0] in "xu" and len(t) > 1:
            return chr(int(t[1:], 16))
        return _ESCAPES.get(t, "\\" + t)
    return _ESCAPE_RE.sub(sub, body)


def cel_eval(e, env: Dict[str, Any]):
    """Evaluate with partial knowledge: returns a value, or UNKNOWN if the result depends on
    a missing parameter (SpiceDB returns CONDITIONAL_PERMISSION in that case)."""
    op = e[0]
    if op == "lit":
        return e[1]
    if op == "var":
        v = env.get(e[1], UNKNOWN)
        conv = e[2] if len(e) > 2 else None
        if conv is None or v is UNKNOWN or isinstance(v, _CONV_TYPE[conv]):
            return v
        if not isinstance(v, str):
            raise ValueError(f"parameter {e[1]!r} has the wrong type")
        return _CONV_FN[conv](v)
    if op == "has":
        a = cel_eval(e[1], env)
        if a is UNKNOWN:
            return UNKNOWN
        if not isinstance(a, dict):
            raise ValueError("has() on a non-map")
        return e[2] in a
    if op == "call":
        return _cel_call(e, env)
    if op == "list":
        vals = [cel_eval(x, env) for x in e[1]]
        return UNKNOWN if any(v is UNKNOWN for v in vals) else vals
    if op == "&&":
        a, b = cel_eval(e[1], env), cel_eval(e[2], env)
        if a is False or b is False:
            return False
        if a is UNKNOWN or b is UNKNOWN:
            return UNKNOWN
        return bool(a) and bool(b)
    if op == "||":
        a, b = cel_eval(e[1], env), cel_eval(e[2], env)
        if a is True or b is True:
            return True
        if a is UNKNOWN or b is UNKNOWN:
            return UNKNOWN
        return bool(a) or bool(b)
    if op == "?:":
        c = cel_eval(e[1], env)
        if c is UNKNOWN:
            a, b = cel_eval(e[2], env), cel_eval(e[3], env)
            return a if (a is not UNKNOWN and a == b) else UNKNOWN
        return cel_eval(e[2] if c else e[3], env)
    if op == "!":
        a = cel_eval(e[1], env)
        return UNKNOWN if a is UNKNOWN else (not a)
    if op == "neg":
        a = cel_eval(e[1], env)
        return UNKNOWN if a is UNKNOWN else -a
    if op == ".":
        a = cel_eval(e[1], env)
        if a is UNKNOWN:
            return UNKNOWN
        return a.get(e[2], UNKNOWN) if isinstance(a, dict) else UNKNOWN
    a, b = cel_eval(e[1], env), cel_eval(e[2], env)
    if a is UNKNOWN or b is UNKNOWN:
        return UNKNOWN
    if op == "[]":
        return a[b]
    if op == "==":
        return a == b
    if op == "!=":
        return a != b
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    if op == ">=":
        return a >= b
    if op == "in":
        return a in b
    if isinstance(a, (Timestamp, Duration, IPAddress)) or isinstance(b, (Timestamp, Duration, IPAddress)):
        return _cel_temporal(op, a, b)
    if op == "+":
        return a + b
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        return a // b if isinstance(a, int) and isinstance(b, int) else a / b
    if op == "%":
        return a % b
    raise SchemaError(f"unsupported CEL operator {op!r}")


# -- CEL standard functions over timestamps, durations and strings, and SpiceDB's ipaddress ---
# (SURVEY §8 f4). Timestamps and durations are whole microseconds (RFC 3339 fractions and Go
# duration components below 1 us are truncated); accessors are UTC.

@dataclass(frozen=True, order=True)
class Timestamp:
    us: int


@dataclass(frozen=True, order=True)
class Duration:
    us: int


@dataclass(frozen=True)
class IPAddress:
    packed: bytes


_RFC3339 = re.compile(r"^(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2}):(\d{2})(?:\.(\d+))?(?:([Zz])|([+-])(\d{2}):(\d{2}))$")


def parse_timestamp(s: str) -> Timestamp:
    m = _RFC3339.match(s)
    if not m:
        raise ValueError(f"not an RFC 3339 timestamp: {s!r}")
    y, mo, d, h, mi, se = (int(m.group(k)) for k in range(1, 7))
    if h > 23 or mi > 59 or se > 59:
        raise ValueError(f"not an RFC 3339 timestamp: {s!r}")
    day = datetime.date(y, mo, d)  # ValueError on an impossible date
    frac = int((m.group(7) or "")[:6].ljust(6, "0"))
    off = 0
    if m.group(9):
        oh, om = int(m.group(10)), int(m.group(11))
        if oh > 23 or om > 59:
            raise ValueError(f"not an RFC 3339 timestamp: {s!r}")
        off = (1 if m.group(9) == "+" else -1) * (oh * 3600 + om * 60)
    days = (day - datetime.date(1970, 1, 1)).days
    return Timestamp(((days * 86400 + h * 3600 + mi * 60 + se) - off) * 1_000_000 + frac)


_DUR_UNITS = {"ns": 1, "us": 1000, "\u00b5s": 1000, "ms": 1_000_000, "s": 1_000_000_000, "m": 60_000_000_000,
              "h": 3_600_000_000_000}
_DUR_PART = re.compile(r"(\d*)(?:\.(\d*))?(ns|us|\u00b5s|ms|s|m|h)")


def parse_duration(s: str) -> Duration:
    t, neg = s, False
    if t[:1] in ("-", "+"):
        neg, t = t[0] == "-", t[1:]
    if t == "0":
        return Duration(0)
    if not t:
        raise ValueError(f"not a duration: {s!r}")
    ns, pos = 0, 0
    while pos < len(t):
        m = _DUR_PART.match(t, pos)
        if not m or (not m.group(1) and not m.group(2)):
            raise ValueError(f"not a duration: {s!r}")
        unit = _DUR_UNITS[m.group(3)]
        frac = (m.group(2) or "")[:18]
        ns += int(m.group(1) or "0") * unit + (int(frac) * unit // 10 ** len(frac) if frac else 0)
        pos = m.end()
    us = ns // 1000
    if us > (2 ** 63 - 1) // 2:
        raise ValueError(f"duration out of range: {s!r}")
    return Duration(-us if neg else us)


def parse_ipaddress(s: str) -> IPAddress:
    import ipaddress
    if ":" not in s:
        parts = s.split(".")
        if len(parts) != 4 or any(not p.isdigit() or not p.isascii() or len(p) > 3 or (len(p) > 1 and p[0] == "0")
                                  or int(p) > 255 for p in parts):
            raise ValueError(f"not an IP address: {s!r}")
    return IPAddress(ipaddress.ip_address(s).packed)


def _in_cidr(ip: IPAddress, cidr: str) -> bool:
    net, _, bits = cidr.partition("/")
    if not bits or not bits.isdigit() or not bits.isascii() or len(bits) > 3:
        raise ValueError(f"invalid CIDR {cidr!r}")
    n = int(bits)
    base = parse_ipaddress(net).packed
    if n > len(base) * 8:
        raise ValueError(f"invalid CIDR {cidr!r}")
    if len(ip.packed) != len(base):
        return False
    a, b = int.from_bytes(ip.packed, "big"), int.from_bytes(base, "big")
    shift = len(base) * 8 - n
    return (a >> shift) == (b >> shift)


_CONV_TYPE = {"timestamp": Timestamp, "duration": Duration, "ipaddress": IPAddress}
_CONV_FN = {"timestamp": parse_timestamp, "duration": parse_duration, "ipaddress": parse_ipaddress}


def _trunc_div(a: int, b: int) -> int:
    q = abs(a) // b
    return -q if a < 0 else q


def _cel_temporal(op, a, b):
    if op == "+":
        if isinstance(a, Duration) and isinstance(b, Duration):
            return Duration(a.us + b.us)
        if isinstance(a, Timestamp) and isinstance(b, Duration):
            return Timestamp(a.us + b.us)
        if isinstance(a, Duration) and isinstance(b, Timestamp):
            return Timestamp(a.us + b.us)
    if op == "-":
        if isinstance(a, Timestamp) and isinstance(b, Timestamp):
            return Duration(a.us - b.us)
        if isinstance(a, Timestamp) and isinstance(b, Duration):
            return Timestamp(a.us - b.us)
        if isinstance(a, Duration) and isinstance(b, Duration):
            return Duration(a.us - b.us)
    if op in ("<", "<=", ">", ">=") and type(a) is type(b) and not isinstance(a, IPAddress):
        return {"<": a.us < b.us, "<=": a.us <= b.us, ">": a.us > b.us, ">=": a.us >= b.us}[op]
    if op == "in" and isinstance(b, list):
        return any(a == x for x in b)
    raise ValueError(f"{op!r} on incompatible values")


def _cel_call(e, env):
    _, f, method, kids = e
    a = []
    for k in kids:
        v = cel_eval(k, env)
        if v is UNKNOWN:
            return UNKNOWN
        a.append(v)

    def want(n):
        if len(a) != n:
            raise ValueError(f"{f}(): wrong number of arguments")

    if f == "size":
        want(1)
        if isinstance(a[0], (str, list, dict)) and not isinstance(a[0], bool):
            return len(a[0])
        raise ValueError("size() of a value without a size")
    if method and f in ("startsWith", "endsWith", "contains"):
        want(2)
        if not isinstance(a[0], str) or not isinstance(a[1], str):
            raise ValueError(f"{f}() needs strings")
        return {"startsWith": a[0].startswith, "endsWith": a[0].endswith,
                "contains": a[0].__contains__}[f](a[1])
    if not method and f in ("timestamp", "duration", "ipaddress"):
        want(1)
        if isinstance(a[0], _CONV_TYPE[f]):
            return a[0]
        if not isinstance(a[0], str):
            raise ValueError(f"{f}(): needs a string")
        return _CONV_FN[f](a[0])
    if method and f == "in_cidr":
        want(2)
        if not isinstance(a[0], IPAddress) or not isinstance(a[1], str):
            raise ValueError("in_cidr() needs an ipaddress and a string")
        return _in_cidr(a[0], a[1])
    if not method and f == "int":
        want(1)
        x = a[0]
        if isinstance(x, bool):
            raise ValueError("int(): unsupported argument")
        if isinstance(x, int):
            return x
        if isinstance(x, float):
            if not (-9.2e18 < x < 9.2e18):
                raise ValueError("int(): out of range")
            return int(x)
        if isinstance(x, str):
            body = x[1:] if x[:1] in ("-", "+") else x
            if not body or len(body) > 18 or not (body.isdigit() and body.isascii()):
                raise ValueError("int(): not an integer string")
            return int(x)
        if isinstance(x, Timestamp):
            return x.us // 1_000_000
        raise ValueError("int(): unsupported argument")
    if not method and f == "double":
        want(1)
        x = a[0]
        if isinstance(x, float):
            return x
        if isinstance(x, int) and not isinstance(x, bool):
            return float(x)
        raise ValueError("double(): unsupported argument")
    if not method and f == "string":
        want(1)
        x = a[0]
        if isinstance(x, str):
            return x
        if isinstance(x, bool):
            return "true" if x else "false"
        if isinstance(x, int):
            return str(x)
        raise ValueError("string(): unsupported argument")
    if method and len(a) == 1 and isinstance(a[0], Timestamp):
        secs = a[0].us // 1_000_000
        days, sod = secs // 86400, secs % 86400
        day = datetime.date(1970, 1, 1) + datetime.timedelta(days=days)
        acc = {"getFullYear": day.year, "getMonth": day.month - 1, "getDate": day.day,
               "getDayOfMonth": day.day - 1, "getDayOfWeek": (day.weekday() + 1) % 7,
               "getDayOfYear": day.timetuple().tm_yday - 1, "getHours": sod // 3600,
               "getMinutes": sod // 60 % 60, "getSeconds": sod % 60,
               "getMilliseconds": (a[0].us - secs * 1_000_000) // 1000}
        if f in acc:
            return acc[f]
    if method and len(a) == 1 and isinstance(a[0], Duration):
        per = {"getHours": 3_600_000_000, "getMinutes": 60_000_000, "getSeconds": 1_000_000, "getMilliseconds": 1000}
        if f in per:
            return _trunc_div(a[0].us, per[f])
    raise ValueError(f"unknown function {f!r}")


# ----------------------------------------------------------------------------------------
# Tuple store and tri-state algebra
# ----------------------------------------------------------------------------------------

@dataclass(frozen=True)
class Tuple_:
    resource_type: str
    resource_id: str
    relation: str
    subject_type: str
    subject_id: str
    subject_relation: str = ELLIPSIS
    caveat: Optional[str] = None
    caveat_context: Optional[Tuple[Tuple[str, Any], ...]] = None
    expires_at: Optional[float] = None  # unix seconds


def parse_tuple(line: str) -> Tuple_:
    """Parse the canonical ``rel.Relationship.String`` text form
    (``rel/relationship.go:51-90``): ``type:id#rel@type:id[#rel][caveat[:{json}]][expiration:T]``."""
    import json
    from datetime import datetime

    line = line.strip()
    exp = None
    cav = None
    ctx = None
    m = re.search(r"\[expiration:([^\]]+)\]$", line)
    if m:
        mm = re.fullmatch(r"(.{19})(?:\.(\d+))?(Z|[+-]\d{2}:\d{2})", m.group(1))
        base = datetime.fromisoformat(mm.group(1) + ("+00:00" if mm.group(3) == "Z" else mm.group(3)))
        exp = base.timestamp() + float("0." + (mm.group(2) or "0"))
        line = line[: m.start()]
    m = re.search(r"\[([A-Za-z_][A-Za-z0-9_/]*)(?::(\{.*\}))?\]$", line)
    if m:
        cav = m.group(1)
        if m.group(2):
            ctx = tuple(sorted(json.loads(m.group(2)).items()))
        line = line[: m.start()]
    res, subj = line.split("@", 1)
    res, rel = res.split("#", 1)
    rtype, rid = res.split(":", 1)
    srel = ELLIPSIS
    if "#" in subj:
        subj, srel = subj.split("#", 1)
    stype, sid = subj.split(":", 1)
    return Tuple_(rtype, rid, rel, stype, sid, srel, cav, ctx, exp)


def union3(vals) -> int:
    vals = list(vals)
    if HAS in vals:
        return HAS
    if ERR in vals:
        return ERR
    if COND in vals:
        return COND
    return NO


def inter3(vals) -> int:
    vals = list(vals)
    if not vals or NO in vals:
        return NO
    if ERR in vals:
        return ERR
    if COND in vals:
        return COND
    return HAS


def excl3(base: int, subs) -> int:
    subs = list(subs)
    if base == NO or HAS in subs:
        return NO
    if base == ERR or ERR in subs:
        return ERR
    if base == COND or COND in subs:
        return COND
    return HAS


def and3(caveat: int, sub: int) -> int:
    """A caveated edge conditions everything reached through it."""
    if sub == ERR:
        return ERR
    if caveat == HAS:
        return sub
    if caveat == NO or sub == NO:
        return NO
    return COND


class TupleStore:
    def __init__(self, tuples=()):
        self.index: Dict[Tuple[str, str, str], List[Tuple_]] = {}
        self.count = 0
        for t in tuples:
            self.add(t)

    def add(self, t: Tuple_):
        if isinstance(t, str):
            t = parse_tuple(t)
        lst = self.index.setdefault((t.resource_type, t.resource_id, t.relation), [])
        key = (t.subject_type, t.subject_id, t.subject_relation)
        for i, o in enumerate(lst):
            if (o.subject_type, o.subject_id, o.subject_relation) == key:
                lst[i] = t  # TOUCH semantics: one relationship per (resource, rel, subject)
                return
        lst.append(t)
        self.count += 1

    def delete(self, t: Tuple_):
        if isinstance(t, str):
            t = parse_tuple(t)
        lst = self.index.get((t.resource_type, t.resource_id, t.relation), [])
        key = (t.subject_type, t.subject_id, t.subject_relation)
        for i, o in enumerate(lst):
            if (o.subject_type, o.subject_id, o.subject_relation) == key:
                del lst[i]
                self.count -= 1
                return

    def get(self, rtype, rid, rel) -> List[Tuple_]:
        return self.index.get((rtype, rid, rel), [])


# ----------------------------------------------------------------------------------------
# The checker
# ----------------------------------------------------------------------------------------

@dataclass
class Item:
    resource_type: str
    resource_id: str
    permission: str
    subject_type: str
    subject_id: str
    subject_relation: str = ELLIPSIS
    context: Optional[Dict[str, Any]] = None


class Checker:
    def __init__(self, schema: Schema, store: TupleStore, max_depth: int = DEFAULT_MAX_DEPTH,
                 now: float = 0.0, evaluate_caveats: bool = True):
        self.schema = schema
        self.store = store
        self.max_depth = max_depth
        self.now = now
        # False = the device contract: every caveated edge is CONDITIONAL (the host resolves
        # CONDITIONAL items with CEL afterwards)
        self.evaluate_caveats = evaluate_caveats

    # -- validation (per-item errors) -----------------------------------------------------
    def validate(self, it: Item) -> int:
        if it.resource_type not in self.schema.defs or it.subject_type not in self.schema.defs:
            return ITEM_ERR_UNKNOWN_TYPE
        if self.schema.relation(it.resource_type, it.permission) is None:
            return ITEM_ERR_UNKNOWN_PERMISSION
        srel = it.subject_relation or ELLIPSIS
        if srel != ELLIPSIS and self.schema.relation(it.subject_type, srel) is None:
            return ITEM_ERR_UNKNOWN_SUBJECT_RELATION
        if it.subject_id == WILDCARD:
            return ITEM_ERR_WILDCARD_SUBJECT
        return ITEM_OK

    def check(self, it: Item) -> Tuple[int, int]:
        """Returns (permissionship, item_error). permissionship is 0 when item_error != 0."""
        err = self.validate(it)
        if err:
            return 0, err
        self._subj = (it.subject_type, it.subject_id, it.subject_relation or ELLIPSIS)
        self._ctx = dict(it.context or {})
        # Memo of dispatch results keyed by (vertex, remaining depth): for a fixed subject,
        # context and clock, _dispatch is a pure function of its arguments, so this changes no
        # result — it only keeps cyclic and re-converging data polynomial (|vertices| x depth).
        self._memo = {}
        try:
            r = self._dispatch(it.resource_type, it.resource_id, it.permission, self.max_depth)
        except SchemaError:
            raise
        except (ValueError, TypeError):  # cel_eval: a caveat failed on the merged context (CEL type errors)
            return 0, ITEM_ERR_CAVEAT_EVAL
        if r == ERR:
            return 0, ITEM_ERR_MAX_DEPTH
        return r, ITEM_OK

    def check_many(self, items) -> List[Tuple[int, int]]:
        return [self.check(it) for it in items]

    def lookup_subjects(self, rtype, rid, perm, stype, srel=ELLIPSIS, context=None) -> List[Tuple[str, int]]:
        """``Client.LookupSubjects`` (``client/client.go:560-599``) as SpiceDB answers it: the
        subjects of kind (stype, srel) that have ``perm`` on rtype:rid — HAS or CONDITIONAL —
        sorted by id, with a wildcard grant reported once as the subject ``"*"`` (last). The
        candidates are the concrete subjects on the relationships the rewrite's positive operands
        reach from the resource (union and intersection operands, exclusion bases, computed
        usersets, arrows, userset subjects; expired relationships skipped); each is checked, and
        so is one subject that appears nowhere, which stands for the wildcard. Any candidate's
        depth error fails the lookup (ValueError)."""
        found, seen = set(), set()
        todo = [(rtype, rid, perm)]
        while todo:
            t, i, r = todo.pop()
            if (t, i, r) in seen:
                continue
            seen.add((t, i, r))
            rel = self.schema.relation(t, r)
            if rel is None:
                continue
            if not rel.is_permission:
                for tu in self.store.get(t, i, r):
                    if not self._visible(tu) or tu.subject_id == WILDCARD:
                        continue
                    if tu.subject_type == stype and tu.subject_relation == srel:
                        found.add(tu.subject_id)
                    if tu.subject_relation != ELLIPSIS:
                        todo.append((tu.subject_type, tu.subject_id, tu.subject_relation))
                continue
            exprs = [rel.expr]
            while exprs:
                e = exprs.pop()
                if e.op in ("union", "intersect"):
                    exprs.extend(e.children)
                elif e.op == "exclude":
                    exprs.append(e.children[0])
                elif e.op == "computed":
                    todo.append((t, i, e.name))
                elif e.op == "arrow":
                    for tu in self.store.get(t, i, e.tupleset):
                        if self._visible(tu):
                            todo.append((tu.subject_type, tu.subject_id, e.name))
        out = []
        cands = sorted(found) + ([None] if srel == ELLIPSIS else [])
        for sid in cands:
            p, err = self.check(Item(rtype, rid, perm, stype, "\x00absent" if sid is None else sid, srel, context))
            if err == ITEM_ERR_MAX_DEPTH:
                raise ValueError("max depth exceeded")
            if p in (HAS, COND):
                out.append((WILDCARD if sid is None else sid, p))
        return out

    # -- SpiceDB restatement -------------------------------------------------------------
    def _dispatch(self, rtype, rid, rel, depth_remaining) -> int:
        if depth_remaining <= 0:
            return ERR  # dispatch.CheckDepth: "max depth exceeded"
        if (rtype, rid, rel) == self._subj:
            return HAS  # filterForFoundMemberResource (identity)
        r = self.schema.relation(rtype, rel)
        if r is None:
            return NO
        key = (rtype, rid, rel, depth_remaining)
        v = self._memo.get(key)
        if v is None:
            if r.is_permission:
                v = self._eval(r.expr, rtype, rid, depth_remaining)
            else:
                v = self._check_direct(rtype, rid, rel, depth_remaining)
            self._memo[key] = v
        return v

    def _visible(self, t: Tuple_) -> bool:
        return t.expires_at is None or t.expires_at > self.now

    def _caveat(self, t: Tuple_) -> int:
        if not t.caveat:
            return HAS
        if not self.evaluate_caveats:
            return COND
        cav = self.schema.caveats.get(t.caveat)
        if cav is None:
            return COND
        env = dict(self._ctx)
        env.update(dict(t.caveat_context or ()))  # relationship context takes precedence
        v = cel_eval(cav.expr, env)
        if v is UNKNOWN:
            return COND
        return HAS if v is True else NO

    def _check_direct(self, rtype, rid, rel, dr) -> int:
        stype, sid, srel = self._subj
        results = []
        for t in self.store.get(rtype, rid, rel):
            if not self._visible(t):
                continue
            matched = False
            if t.subject_type == stype:
                if t.subject_id == WILDCARD and t.subject_relation == ELLIPSIS and srel == ELLIPSIS:
                    matched = True
                elif t.subject_id == sid and t.subject_relation == srel:
                    matched = True
            if matched:
                results.append(self._caveat(t))
            elif t.subject_relation != ELLIPSIS:
                sub = self._dispatch(t.subject_type, t.subject_id, t.subject_relation, dr - 1)
                results.append(and3(self._caveat(t), sub))
        return union3(results)

    def _computed(self, rtype, rid, rel, dr) -> int:
        if (rtype, rid, rel) == self._subj:
            return HAS
        if self.schema.relation(rtype, rel) is None:
            return NO  # TTU target missing on this subject type: no members
        return self._dispatch(rtype, rid, rel, dr - 1)

    def _eval(self, e: Expr, rtype, rid, dr) -> int:
        if e.op == "union":
            return union3(self._eval(c, rtype, rid, dr) for c in e.children)
        if e.op == "intersect":
            return inter3([self._eval(c, rtype, rid, dr) for c in e.children])
        if e.op == "exclude":
            base = self._eval(e.children[0], rtype, rid, dr)
            return excl3(base, [self._eval(c, rtype, rid, dr) for c in e.children[1:]])
        if e.op == "nil":
            return NO
        if e.op == "computed":
            return self._computed(rtype, rid, e.name, dr)
        if e.op == "arrow":
            results = []
            for t in self.store.get(rtype, rid, e.tupleset):
                if not self._visible(t):
                    continue
                sub = self._computed(t.subject_type, t.subject_id, e.name, dr)
                results.append(and3(self._caveat(t), sub))
            if e.func == "all":
                return inter3(results)  # empty tupleset -> NO
            return union3(results)
        raise SchemaError(f"unknown expression op {e.op}")
