"""Shared test helpers: fixture loading, check-string parsing, oracle <-> engine glue."""
import json
import os
from datetime import datetime

from gochugaru_amd import rel

from oracle import spicedb_ref as ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

PERM_NAMES = {ref.NO: "NO", ref.HAS: "HAS", ref.COND: "COND"}


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def parse_check(s: str) -> rel.Relationship:
    res, subj = s.split("@", 1)
    r, _ = res.split("#", 1)[0], None
    resource, relation = res.split("#", 1)
    return rel.FromTriple(resource, relation, subj)


def to_oracle_item(r: rel.Relationship, context=None) -> ref.Item:
    return ref.Item(r.ResourceType, r.ResourceID, r.ResourceRelation, r.SubjectType, r.SubjectID,
                    r.SubjectRelation or ref.ELLIPSIS, context)


def iso_to_unix(s: str) -> float:
    return datetime.fromisoformat(s.replace("Z", "+00:00")).timestamp()


def expected_code(label: str):
    """'HAS'/'NO'/'COND' -> (perm, 0); 'ERR:n' -> (0, n)."""
    if label.startswith("ERR:"):
        return 0, int(label[4:])
    return {"HAS": ref.HAS, "NO": ref.NO, "COND": ref.COND}[label], 0


def oracle_for(schema_text, tuples, max_depth=50, now=0.0, evaluate_caveats=True):
    sc = ref.Schema(schema_text)
    st = ref.TupleStore(ref.parse_tuple(t) for t in tuples)
    return ref.Checker(sc, st, max_depth=max_depth, now=now, evaluate_caveats=evaluate_caveats)
