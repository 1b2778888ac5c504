"""C ABI checks that need no GPU: libgck.so loads, exports exactly what include/gck.h
declares, and the host-side data plane (schema compiler, interner, text ingest validation)
behaves. No compute calls are made here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from gochugaru_amd import engine as E
from tests.helpers import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gck.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gck_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = E.load_library()
    declared = header_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    # the ctypes signature table covers the header exactly
    assert sorted(E._SIGS) == declared


def test_driver_library_exports_its_loop():
    """bench.py's compiled submit/wait loop (csrc/driver.cpp) loads without a GPU."""
    import ctypes
    import os
    path = os.path.join(os.path.dirname(E.__file__), "libgck_driver.so")
    assert hasattr(ctypes.CDLL(path), "gckd_run")
    assert hasattr(ctypes.CDLL(path), "gckd_run_uniform")


def test_struct_layouts_match_header():
    assert E.ITEM_DTYPE.itemsize == 20
    assert E.TUPLE_DTYPE.itemsize == 32
    assert E.UPDATE_DTYPE.itemsize == 40
    assert C.sizeof(E._Config) == 88
    assert C.sizeof(E._Stats) == 240
    assert C.sizeof(E.Uniform) == 16
    assert E.ITEM_ERROR_DTYPE.itemsize == 8
    assert E.load_library().gck_abi_version() == 13


@pytest.fixture()
def eng():
    e = E.Engine(device=0)
    yield e
    e.close()


def test_schema_compile_and_lookup(eng):
    g = load_golden("semantics.json")["suites"][0]
    eng.load_schema(g["schema"])
    t, r = eng.counts()
    assert t == 4 and r == 1 + 5 + 9
    doc = eng.type_id("doc")
    assert eng.relation_id(doc, "view") != E.REL_INVALID
    assert eng.relation_id(doc, "nosuch") == E.REL_INVALID
    assert eng.type_id("nosuch") == E.TYPE_INVALID


@pytest.mark.parametrize("bad", [
    "definition a { relation r: nosuch }",
    "definition a { permission p = nosuch }",
    "definition a {}\ndefinition a {}",
    "definition a { relation r: a  permission p = r->missing }",
    "definition a { relation r: a:*  permission p = r->p }",
    "definition a { relation r: a with nocaveat }",
    "definition a { relation r: a",
    "definition a { permission p = (r }",
])
def test_schema_errors(eng, bad):
    with pytest.raises(E.GckError) as ei:
        eng.load_schema(bad)
    assert ei.value.code == E.GCK_E_SCHEMA


def test_intern_and_text_staging(eng):
    g = load_golden("semantics.json")["suites"][0]
    eng.load_schema(g["schema"])
    eng.begin_snapshot(1)
    eng.add_tuples_text("\n".join(g["tuples"]))
    user = eng.type_id("user")
    ids = eng.intern(user, ["alice", "bob", "nobody", "*"])
    assert ids[0] != ids[1] and ids[2] == E.ID_ABSENT and ids[3] == E.ID_WILDCARD
    assert eng.object_name(user, int(ids[0])) == "alice"
    new = eng.intern(user, ["nobody"], create=True)
    assert new[0] == eng.object_count(user) - 1
    # validation: relationship to a permission, disallowed subject kind, unknown names
    for bad in ["doc:x#view@user:a", "doc:x#owner@group:g#member", "doc:x#nosuch@user:a",
                "nosuch:x#owner@user:a", "doc:x#owner@user:*", "doc:x#owner", "docx#owner@user:a"]:
        with pytest.raises(E.GckError):
            eng.add_tuples_text(bad)


def test_text_trailers(eng):
    g = load_golden("semantics.json")["suites"][2]
    eng.load_schema(g["schema"])
    eng.begin_snapshot(3)
    eng.add_tuples_text("\n".join(g["tuples"]))
    with pytest.raises(E.GckError):
        eng.add_tuples_text("doc:a#viewer@user:u1[nosuchcaveat]")
    with pytest.raises(E.GckError):
        eng.add_tuples_text("doc:a#editor@user:u1[expiration:not-a-time]")


def test_binary_tuple_staging(eng):
    eng.load_schema("definition user {}\ndefinition group { relation member: user | group#member }")
    user, group = eng.type_id("user"), eng.type_id("group")
    member = eng.relation_id(group, "member")
    eng.reserve_objects(user, 10)
    eng.reserve_objects(group, 4)
    eng.begin_snapshot(9)
    t = np.zeros(3, dtype=E.TUPLE_DTYPE)
    t["resource_type"] = group
    t["relation"] = member
    t["resource_id"] = [0, 1, 1]
    t["subject_type"] = [user, user, group]
    t["subject_relation"] = [E.ELLIPSIS, E.ELLIPSIS, member]
    t["subject_id"] = [3, 4, 2]
    eng.add_tuples(t)
    t2 = t[:1].copy()
    t2["subject_id"] = 99  # never reserved
    with pytest.raises(E.GckError):
        eng.add_tuples(t2)


def test_state_errors(eng):
    with pytest.raises(E.GckError) as ei:
        eng.begin_snapshot(1)
    assert ei.value.code == E.GCK_E_STATE
    eng.load_schema("definition user {}")
    with pytest.raises(E.GckError) as ei:
        eng.add_tuples_text("user:a#x@user:b")
    assert ei.value.code == E.GCK_E_STATE
    with pytest.raises(E.GckError) as ei:
        eng.check_bulk(np.zeros(1, dtype=E.ITEM_DTYPE))
    assert ei.value.code == E.GCK_E_STATE
    # Watch updates need a committed snapshot
    with pytest.raises(E.GckError) as ei:
        eng.apply_updates_text(2, "CREATE user:a#x@user:b")
    assert ei.value.code == E.GCK_E_STATE
    with pytest.raises(E.GckError) as ei:
        eng.apply_updates(2, np.zeros(1, dtype=E.UPDATE_DTYPE))
    assert ei.value.code == E.GCK_E_STATE


def test_uniform_and_revision_entry_points_without_a_snapshot(eng):
    """The ABI-13 entry points validate their arguments on the host: a uniform header whose context
    slot exceeds the contexts given is refused before anything else, an empty request needs a
    snapshot like any check, and a submitted batch's revision is the one at submit."""
    with pytest.raises(E.GckError) as ei:
        eng.check_uniform((0, 0, 0, 0xFFFF, 2), np.zeros((4, 2), dtype=np.uint32), contexts=[{"a": 1}])
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    eng.load_schema("definition user {}")
    with pytest.raises(E.GckError) as ei:
        eng.check_uniform((0, 0, 0, 0xFFFF), np.zeros((0, 2), dtype=np.uint32))
    assert ei.value.code == E.GCK_E_STATE
    with pytest.raises(E.GckError) as ei:
        eng.check_bulk_at(np.zeros(0, dtype=E.ITEM_DTYPE))
    assert ei.value.code == E.GCK_E_STATE


def test_unpack_results_layout():
    """Packed results: check k in bits 2(k mod 32) of little-endian word k / 32."""
    perm = np.array([1, 2, 3, 0] * 20 + [2], dtype=np.uint8)
    words = np.zeros((len(perm) + 31) // 32, dtype=np.uint64)
    for k, p in enumerate(perm):
        words[k // 32] |= np.uint64(int(p) << (2 * (k % 32)))
    assert E.unpack_results(words, len(perm)).tolist() == perm.tolist()


def test_watch_staging_without_a_snapshot():
    """gck_watch_stage works on the host alone (validation and grouping on the engine's thread);
    applying needs a committed snapshot (GCK_E_STATE); four slots; unknown tickets refused."""
    from gochugaru_amd import engine as E
    e = E.Engine()
    e.load_schema("definition user {}\ndefinition group { relation member: user }")
    ups = np.zeros(2, dtype=E.UPDATE_DTYPE)
    ups["op"] = E.UPDATE_CREATE
    ts = [e.stage_updates(ups) for _ in range(4)]
    with pytest.raises(E.GckError) as ei:
        e.stage_updates(ups)
    assert ei.value.code == E.GCK_E_CAPACITY
    with pytest.raises(E.GckError) as ei:
        e.apply_staged(2, ts[0])
    assert ei.value.code == E.GCK_E_STATE
    for t in ts[1:]:
        e.discard_staged(t)
    with pytest.raises(E.GckError) as ei:
        e.discard_staged(ts[1])
    assert ei.value.code == E.GCK_E_INVALID_ARGUMENT
    e.stage_updates(ups)  # (a slot is free again; the engine ends with a batch still staged)
    e.close()
