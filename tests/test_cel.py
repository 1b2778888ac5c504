"""Host CEL evaluator (gochugaru_amd/csrc/cel.cpp, exported as gck_evaluate_caveat) against the
oracle's restatement (oracle/spicedb_ref.py cel_eval). CPU only: the evaluator runs on the host,
it decides which caveated relationships count before the device walk.

Parity is pinned to the oracle (and through it to the hand-derived caveat fixtures in
tests/golden/semantics.json); the reference itself carries no caveat evaluator.
"""
import json
import random

import pytest

from gochugaru_amd import engine as E
from oracle import spicedb_ref as ref
from tests.helpers import load_golden

VARS = {"a": "int", "b": "str", "c": "list", "d": "map", "e": "bool"}


def _lit(rng, ty):
    if ty == "int":
        return str(rng.randint(0, 6))
    if ty == "str":
        return rng.choice(['"tuesday"', '"monday"', '"x"', "'y'", '""'])
    if ty == "bool":
        return rng.choice(["true", "false"])
    if ty == "list":
        return "[" + ", ".join(_lit(rng, "int") for _ in range(rng.randint(0, 3))) + "]"
    return "null"


def gen(rng, ty, depth):
    """A random well-typed CEL expression of type `ty` (int / str / bool / list)."""
    if depth == 0 or rng.random() < 0.25:
        opts = [v for v, t in VARS.items() if t == ty]
        if ty == "int":
            opts += ['d.k', 'd["k"]', "c[0]"]
        if ty == "str":
            opts += ["d.s"]
        if opts and rng.random() < 0.6:
            return rng.choice(opts)
        return _lit(rng, ty)
    d = depth - 1
    if ty == "int":
        op = rng.choice(["+", "-", "*", "/", "%", "neg", "?:"])
        if op == "neg":
            return f"-({gen(rng, 'int', d)})"
        if op == "?:":
            return f"({gen(rng, 'bool', d)} ? {gen(rng, 'int', d)} : {gen(rng, 'int', d)})"
        return f"({gen(rng, 'int', d)} {op} {gen(rng, 'int', d)})"
    if ty == "str":
        if rng.random() < 0.5:
            return f"({gen(rng, 'str', d)} + {gen(rng, 'str', d)})"
        return f"({gen(rng, 'bool', d)} ? {gen(rng, 'str', d)} : {gen(rng, 'str', d)})"
    if ty == "list":
        return f"({gen(rng, 'list', d)} + {gen(rng, 'list', d)})"
    # bool
    op = rng.choice(["&&", "||", "!", "cmp", "eq", "in_list", "in_str", "in_map", "?:", "noparen"])
    if op in ("&&", "||"):
        return f"({gen(rng, 'bool', d)} {op} {gen(rng, 'bool', d)})"
    if op == "!":
        return f"!({gen(rng, 'bool', d)})"
    if op == "cmp":
        t = rng.choice(["int", "str"])
        return f"({gen(rng, t, d)} {rng.choice(['<', '<=', '>', '>='])} {gen(rng, t, d)})"
    if op == "eq":
        t = rng.choice(["int", "str", "bool", "list"])
        return f"({gen(rng, t, d)} {rng.choice(['==', '!='])} {gen(rng, t, d)})"
    if op == "in_list":
        return f"({gen(rng, 'int', d)} in {gen(rng, 'list', d)})"
    if op == "in_str":
        return f"({gen(rng, 'str', d)} in {gen(rng, 'str', d)})"
    if op == "in_map":
        key = rng.choice(['"k"', '"s"', '"z"'])
        return f"({key} in d)"
    if op == "?:":
        return f"({gen(rng, 'bool', d)} ? {gen(rng, 'bool', d)} : {gen(rng, 'bool', d)})"
    # precedence without parentheses: a + b * c < a || !e && b == "x"
    return (f"{gen(rng, 'int', 0)} + {gen(rng, 'int', 0)} * {gen(rng, 'int', 0)} < {gen(rng, 'int', 0)}"
            f" || !{gen(rng, 'bool', 0)} && {gen(rng, 'str', 0)} == {gen(rng, 'str', 0)}")


def rand_context(rng):
    ctx = {}
    for v, t in VARS.items():
        if rng.random() < 0.5:
            continue
        if t == "int":
            ctx[v] = rng.randint(-3, 6)
        elif t == "str":
            ctx[v] = rng.choice(["tuesday", "monday", "x", "xy", ""])
        elif t == "bool":
            ctx[v] = rng.random() < 0.5
        elif t == "list":
            ctx[v] = [rng.randint(0, 4) for _ in range(rng.randint(0, 3))]
        else:
            m = {}
            if rng.random() < 0.7:
                m["k"] = rng.randint(0, 4)
            if rng.random() < 0.7:
                m["s"] = rng.choice(["x", "tuesday"])
            ctx[v] = m
    return ctx


def oracle_outcome(expr, stored, context):
    env = dict(context or {})
    env.update(stored or {})  # the relationship's stored context takes precedence
    try:
        v = ref.cel_eval(expr, env)
    except (TypeError, ZeroDivisionError, KeyError, IndexError, ValueError):
        return "error"
    if v is ref.UNKNOWN:
        return E.CAVEAT_PARTIAL
    return E.CAVEAT_TRUE if v is True else E.CAVEAT_FALSE


def engine_outcome(eng, name, stored, context):
    try:
        return eng.evaluate_caveat(name, stored, context)
    except E.GckError as err:
        assert err.code == E.GCK_E_INVALID_ARGUMENT, err
        return "error"


@pytest.fixture()
def eng():
    e = E.Engine(device=0)
    yield e
    e.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_expressions_match_oracle(eng, seed):
    rng = random.Random(1000 + seed)
    bodies = [gen(rng, "bool", rng.randint(1, 4)) for _ in range(40)]
    params = ", ".join(f"{v} {t}" for v, t in VARS.items())
    schema = "".join(f"caveat c{i}({params}) {{ {b} }}\n" for i, b in enumerate(bodies)) + "definition user {}\n"
    eng.load_schema(schema)
    sc = ref.Schema(schema)
    n = 0
    for i, body in enumerate(bodies):
        expr = sc.caveats[f"c{i}"].expr
        for _ in range(12):
            stored = rand_context(rng) if rng.random() < 0.5 else None
            context = rand_context(rng) if rng.random() < 0.8 else None
            want = oracle_outcome(expr, stored, context)
            got = engine_outcome(eng, f"c{i}", stored, context)
            assert got == want, (body, stored, context)
            n += 1
    assert n == 480


def test_golden_caveat_fixtures(eng):
    """tests/golden/semantics.json: the hand-derived caveat cases, evaluated on the host."""
    s = [x for x in load_golden("semantics.json")["suites"] if x["name"] == "caveats-and-expiration"][0]
    eng.load_schema(s["schema"])
    assert eng.evaluate_caveat("only_on_tuesday") == E.CAVEAT_PARTIAL
    assert eng.evaluate_caveat("only_on_tuesday", {"day_of_the_week": "tuesday"}) == E.CAVEAT_TRUE
    assert eng.evaluate_caveat("only_on_tuesday", None, {"day_of_the_week": "monday"}) == E.CAVEAT_FALSE
    # relationship context takes precedence over the check context
    assert eng.evaluate_caveat("only_on_tuesday", {"day_of_the_week": "wednesday"},
                               {"day_of_the_week": "tuesday"}) == E.CAVEAT_FALSE


def test_partial_evaluation_and_short_circuit(eng):
    eng.load_schema('caveat c(a int, b string) { a > 3 || b == "x" }\n'
                    'caveat t(a int) { a > 0 ? true : true }\n'
                    'caveat n(m map<any>) { m.f == 1 }\n'
                    "definition u {}")
    assert eng.evaluate_caveat("c", None, {"a": 5}) == E.CAVEAT_TRUE
    assert eng.evaluate_caveat("c", None, {"a": 1}) == E.CAVEAT_PARTIAL
    assert eng.evaluate_caveat("c", None, {"a": 1, "b": "y"}) == E.CAVEAT_FALSE
    assert eng.evaluate_caveat("c", None, {"b": "x"}) == E.CAVEAT_TRUE
    assert eng.evaluate_caveat("t") == E.CAVEAT_TRUE  # both branches agree
    assert eng.evaluate_caveat("n", None, {"m": {}}) == E.CAVEAT_PARTIAL  # missing field
    assert eng.evaluate_caveat("n", None, {"m": {"f": 1}}) == E.CAVEAT_TRUE


def test_json_contexts(eng):
    eng.load_schema('caveat c(s string, l list<int>, f double) { s == "a\\"b" && 2 in l && f > 1.5 }\n'
                    "definition u {}")
    ctx = json.dumps({"s": 'a"b', "l": [1, 2], "f": 2.0})
    assert eng.evaluate_caveat("c", None, ctx) == E.CAVEAT_TRUE
    assert eng.evaluate_caveat("c", None, '{"s":"a\\u0022b","l":[2],"f":1e1}') == E.CAVEAT_TRUE
    for bad in ['{"s":', "[1]", '{"s" 1}', '{"s":tru}']:
        with pytest.raises(E.GckError) as ei:
            eng.evaluate_caveat("c", None, bad)
        assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    with pytest.raises(E.GckError) as ei:
        eng.evaluate_caveat("nosuch")
    assert ei.value.code == E.GCK_E_NOT_FOUND


def test_evaluation_errors_are_invalid_argument(eng):
    eng.load_schema("caveat c(a int) { 10 / a == 1 }\ncaveat k(m map<int>) { m[\"z\"] == 1 }\ndefinition u {}")
    assert eng.evaluate_caveat("c", None, {"a": 10}) == E.CAVEAT_TRUE
    for name, ctx in (("c", {"a": 0}), ("k", {"m": {}})):
        with pytest.raises(E.GckError) as ei:
            eng.evaluate_caveat(name, None, ctx)
        assert ei.value.code == E.GCK_E_INVALID_ARGUMENT


def test_caveat_instances_deduplicate(eng):
    s = [x for x in load_golden("semantics.json")["suites"] if x["name"] == "caveats-and-expiration"][0]
    eng.load_schema(s["schema"])
    a = eng.add_caveat_instance("only_on_tuesday", "")
    b = eng.add_caveat_instance("only_on_tuesday", "")
    c = eng.add_caveat_instance("only_on_tuesday", '{"day_of_the_week":"tuesday"}')
    assert a == b and a != c and a > 0
    with pytest.raises(E.GckError):
        eng.add_caveat_instance("only_on_tuesday", '{"day_of_the_week":')


# ---- CEL standard functions, timestamps, durations, ipaddress --------------
# Known answers derived by hand (calendar facts, CIDR arithmetic); the oracle must agree with
# them and the engine with both. Parity with SpiceDB itself is unpinned.
F4_SCHEMA = """caveat f(now timestamp, t2 timestamp, win duration, ip ipaddress, s string, n int, m map<any>, l list<int>) { EXPR }
definition user {}"""
F4_CTX = {"now": "2025-10-03T12:34:56.789Z", "t2": "2024-02-29T23:00:00-01:00", "win": "1h30m",
          "ip": "10.1.2.3", "s": "héllo", "n": 7, "m": {"k": 1}, "l": [1, 2, 3]}
F4_CASES = [
    ("now.getFullYear() == 2025 && now.getMonth() == 9 && now.getDate() == 3", True),
    ("now.getDayOfMonth() == 2 && now.getDayOfWeek() == 5", True),  # 2025-10-03 was a Friday
    ("now.getDayOfYear() == 275", True),  # 31+28+31+30+31+30+31+31+30 = 273 days, then day 3 -> index 275
    ("now.getHours() == 12 && now.getMinutes() == 34 && now.getSeconds() == 56 && now.getMilliseconds() == 789", True),
    ("t2.getMonth() == 2 && t2.getDate() == 1 && t2.getHours() == 0", True),  # 23:00 at -01:00 = 00:00Z next day
    ("t2 == timestamp(\"2024-03-01T00:00:00Z\")", True),
    ("now - t2 > duration(\"13000h\") && now - t2 < duration(\"14000h\")", True),
    ("t2 + duration(\"24h\") == timestamp(\"2024-03-02T00:00:00Z\")", True),
    ("now > t2 && t2 < now && !(now < t2)", True),
    ("win == duration(\"90m\") && win.getMinutes() == 90 && win.getHours() == 1", True),
    ("duration(\"1.5s\").getMilliseconds() == 1500 && duration(\"-1.5h\").getMinutes() == -90", True),
    ("duration(\"300ms\") + duration(\"700ms\") == duration(\"1s\")", True),
    ("duration(\"1h\") - duration(\"61m\") < duration(\"0\")", True),
    ("int(timestamp(\"1970-01-01T00:00:10Z\")) == 10 && int(timestamp(\"1969-12-31T23:59:59.5Z\")) == -1", True),
    ("ip.in_cidr(\"10.0.0.0/8\") && !ip.in_cidr(\"10.2.0.0/16\") && ip.in_cidr(\"10.1.2.3/32\")", True),
    ("ipaddress(\"2001:db8::1\").in_cidr(\"2001:db8::/32\") && !ipaddress(\"2001:db8::1\").in_cidr(\"10.0.0.0/8\")", True),
    ("ip == ipaddress(\"10.1.2.3\") && ip != ipaddress(\"10.1.2.4\")", True),
    ("size(s) == 5 && s.size() == 5 && s.startsWith(\"hé\") && s.endsWith(\"llo\") && s.contains(\"él\")", True),
    ("size(l) == 3 && size(m) == 1 && has(m.k) && !has(m.z)", True),
    ("int(\"-42\") == -42 && int(3.9) == 3 && int(-3.9) == -3 && double(n) == 7.0", True),
    ("string(n) == \"7\" && string(true) == \"true\" && string(\"x\") == \"x\"", True),
    ("now.getDayOfWeek() == 1", False),
]
F4_ERRORS = ["timestamp(\"2025-02-30T00:00:00Z\") == now", "duration(\"5 days\") == win", "int(\"1.5\") == 1",
             "ipaddress(\"10.0.0.256\") == ip", "ip.in_cidr(\"10.0.0.0/33\")", "size(n) == 1", "s.startsWith(n)",
             "now < win", "now + now == now", "nosuch(1) == 1"]


def _f4(expr):
    return F4_SCHEMA.replace("EXPR", expr)


@pytest.mark.parametrize("expr,want", F4_CASES)
def test_f4_known_answers(eng, expr, want):
    schema = _f4(expr)
    eng.load_schema(schema)
    expected = E.CAVEAT_TRUE if want else E.CAVEAT_FALSE
    assert oracle_outcome(ref.Schema(schema).caveats["f"].expr, None, F4_CTX) == expected
    assert engine_outcome(eng, "f", None, F4_CTX) == expected
    # the same with every parameter missing: unknown unless the expression needs none of them
    assert engine_outcome(eng, "f", None, {}) == oracle_outcome(ref.Schema(schema).caveats["f"].expr, None, {})


@pytest.mark.parametrize("expr", F4_ERRORS)
def test_f4_errors(eng, expr):
    schema = _f4(expr)
    eng.load_schema(schema)
    assert oracle_outcome(ref.Schema(schema).caveats["f"].expr, None, F4_CTX) == "error"
    assert engine_outcome(eng, "f", None, F4_CTX) == "error"


def test_f4_typed_parameters(eng):
    """Declared timestamp / duration / ipaddress parameters take their context value as text;
    text that does not convert is an evaluation error, a missing parameter stays unknown."""
    schema = _f4("now > timestamp(\"2025-01-01T00:00:00Z\") && win < duration(\"2h\") && ip.in_cidr(\"10.0.0.0/8\")")
    eng.load_schema(schema)
    expr = ref.Schema(schema).caveats["f"].expr
    for ctx, want in (({**F4_CTX}, E.CAVEAT_TRUE), ({**F4_CTX, "win": "3h"}, E.CAVEAT_FALSE),
                      ({**F4_CTX, "now": "yesterday"}, "error"), ({**F4_CTX, "ip": 10}, "error"),
                      ({"win": "3h"}, E.CAVEAT_FALSE), ({"win": "1h"}, E.CAVEAT_PARTIAL)):
        assert oracle_outcome(expr, None, ctx) == want, ctx
        assert engine_outcome(eng, "f", None, ctx) == want, ctx


TS_POOL = ["1970-01-01T00:00:00Z", "2025-10-03T00:00:00Z", "2025-10-03T23:59:59.999999Z", "2024-02-29T12:00:00+05:30",
           "1999-12-31T23:59:59-08:00", "2000-03-01T00:00:00.5Z", "1969-07-20T20:17:40Z", "2038-01-19T03:14:08Z"]
DUR_POOL = ["0", "1h", "90m", "1.5s", "-2h", "300ms", "1h2m3.5s", "250us", "7ns", "36h", "-0.5m", "1000000s"]
IP_POOL = ["10.1.2.3", "10.255.0.1", "192.168.1.1", "127.0.0.1", "2001:db8::1", "::1", "fe80::1"]
CIDR_POOL = ["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/24", "0.0.0.0/0", "127.0.0.1/32", "2001:db8::/32", "::/0"]
ACCESSORS = ["getFullYear", "getMonth", "getDate", "getDayOfMonth", "getDayOfWeek", "getDayOfYear", "getHours",
             "getMinutes", "getSeconds", "getMilliseconds"]


def gen_f4(rng, depth):
    """A random boolean expression over the f4 functions (parameters now/t2 timestamp, win
    duration, ip ipaddress, s string)."""
    def ts():
        return rng.choice(["now", "t2", f'timestamp("{rng.choice(TS_POOL)}")',
                           f'(now + duration("{rng.choice(DUR_POOL)}"))', f'(t2 - duration("{rng.choice(DUR_POOL)}"))'])

    def dur():
        return rng.choice(["win", f'duration("{rng.choice(DUR_POOL)}")', f"({ts()} - {ts()})",
                           f'(win + duration("{rng.choice(DUR_POOL)}"))'])

    def leaf():
        k = rng.randrange(7)
        if k == 0:
            return f"({ts()} {rng.choice(['<', '<=', '>', '>=', '==', '!='])} {ts()})"
        if k == 1:
            return f"({dur()} {rng.choice(['<', '<=', '>', '>=', '==', '!='])} {dur()})"
        if k == 2:
            return f"({ts()}.{rng.choice(ACCESSORS)}() {rng.choice(['<', '==', '>='])} {rng.randint(0, 60)})"
        if k == 3:
            return f"({dur()}.{rng.choice(ACCESSORS[6:])}() {rng.choice(['<', '==', '>='])} {rng.randint(-100, 100)})"
        if k == 4:
            ipx = rng.choice(["ip", f'ipaddress("{rng.choice(IP_POOL)}")'])
            return f'{ipx}.in_cidr("{rng.choice(CIDR_POOL)}")'
        if k == 5:
            lit = rng.choice(['"ab"', '"b"', '""', '"é"', '"xyz"'])
            return f"s.{rng.choice(['startsWith', 'endsWith', 'contains'])}({lit})"
        return f"(size(s) {rng.choice(['<', '==', '>'])} {rng.randint(0, 4)})"

    if depth == 0:
        return leaf()
    op = rng.choice(["&&", "||", "!", "leaf"])
    if op == "!":
        return f"!({gen_f4(rng, depth - 1)})"
    if op == "leaf":
        return leaf()
    return f"({gen_f4(rng, depth - 1)} {op} {gen_f4(rng, depth - 1)})"


def rand_f4_context(rng):
    ctx = {}
    if rng.random() < 0.7:
        ctx["now"] = rng.choice(TS_POOL + ["2025-13-01T00:00:00Z"] if rng.random() < 0.05 else TS_POOL)
    if rng.random() < 0.7:
        ctx["t2"] = rng.choice(TS_POOL)
    if rng.random() < 0.7:
        ctx["win"] = rng.choice(DUR_POOL + ["1d"] if rng.random() < 0.05 else DUR_POOL)
    if rng.random() < 0.7:
        ctx["ip"] = rng.choice(IP_POOL)
    if rng.random() < 0.7:
        ctx["s"] = rng.choice(["abc", "b", "", "é", "xyzab"])
    return ctx


@pytest.mark.parametrize("seed", range(4))
def test_f4_random_expressions_match_oracle(eng, seed):
    rng = random.Random(7000 + seed)
    bodies = [gen_f4(rng, rng.randint(0, 3)) for _ in range(40)]
    params = "now timestamp, t2 timestamp, win duration, ip ipaddress, s string"
    schema = "".join(f"caveat g{i}({params}) {{ {b} }}\n" for i, b in enumerate(bodies)) + "definition user {}\n"
    eng.load_schema(schema)
    sc = ref.Schema(schema)
    seen = set()
    for i, body in enumerate(bodies):
        expr = sc.caveats[f"g{i}"].expr
        for _ in range(10):
            stored = rand_f4_context(rng) if rng.random() < 0.4 else None
            context = rand_f4_context(rng)
            want = oracle_outcome(expr, stored, context)
            got = engine_outcome(eng, f"g{i}", stored, context)
            assert got == want, (body, stored, context)
            seen.add(want)
    assert {E.CAVEAT_TRUE, E.CAVEAT_FALSE, E.CAVEAT_PARTIAL} <= seen
