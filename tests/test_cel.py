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
