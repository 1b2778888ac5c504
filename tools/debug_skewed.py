"""Reproduces test_gpu_delta.py::test_skewed_batch_on_one_object after the GPU test files that run
before it (its failure needs their leftover device state) and reports, per engine variant, the
checks that disagree with the oracle, the same checks on a fresh engine loaded from the final
store, and on the Watch-applied engine one at a time.
    python tools/debug_skewed.py [variant ...]        (on the GPU box, from the repo root)"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pytest  # noqa: E402

PREFIX = ["tests/test_gpu_caveat_scale.py", "tests/test_gpu_cel.py", "tests/test_gpu_concurrency.py",
          "tests/test_gpu_configs.py"]
VARIANTS = {"default": {}, "nolabels": {"labels": False}, "noclosure": {"closure": False},
            "noslots": {"slots": False}, "nobidir": {"bidir": False}, "nohash": {"membership_hash": False},
            "wide": {"wide_only": True}}


def run(variant, kw):
    from gochugaru_amd import engine as E
    from tests import gen
    from tests.test_gpu_delta import apply_to_store, engine_results, oracle_results
    schema, tuples, checks = gen.nested(3)
    e = E.Engine(**kw)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    store = {}
    apply_to_store(store, [("CREATE", t) for t in tuples])
    rng = random.Random(11)
    for rnd in range(3):
        ups = []
        for k in rng.sample(range(200), 150):
            ups.append(("CREATE", f"group:g{rnd}#member@user:u{k}"))
        tail = [("DELETE", f"group:g{rnd}#member@user:u{k}") for k in rng.sample(range(200), 100)]
        tail += [("TOUCH", f"group:g{rnd}#member@user:u{k}") for k in rng.sample(range(200), 60)]
        tail += [(rng.choice(["CREATE", "DELETE"]), f"group:g{rnd + 10}#member@user:u{rng.randrange(200)}")
                 for _ in range(40)]
        rng.shuffle(tail)
        ups += tail
        e.apply_updates_text(2 + rnd, "\n".join(f"{op} {line}" for op, line in ups))
        apply_to_store(store, ups)
        probe = checks + [f"group:g{rnd}#member@user:u{k}" for k in range(200)] + \
            [f"group:g{rnd + 10}#member@user:u{k}" for k in range(200)]
        bad = [i for i, (a, b) in enumerate(zip(engine_results(e, probe), oracle_results(schema, store, probe)))
               if a != b]
        print(f"[{variant}] round {rnd}: {len(bad)} mismatches", flush=True)
    ups = [(rng.choice(["CREATE", "DELETE", "TOUCH"]), f"group:g{rng.randrange(120)}#member@user:u{rng.randrange(200)}")
           for _ in range(5000)]
    ups += [(rng.choice(["CREATE", "DELETE"]), f"doc:d{rng.randrange(80)}#viewer@group:g{rng.randrange(30)}#member")
            for _ in range(600)]
    st0 = e.stats()
    e.apply_updates_text(9, "\n".join(f"{op} {line}" for op, line in ups))
    apply_to_store(store, ups)
    got = engine_results(e, checks)
    want = oracle_results(schema, store, checks)
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    print(f"[{variant}] final: {len(bad)} mismatches of {len(checks)}", flush=True)
    if bad:
        f = E.Engine(**kw)
        f.load_schema(schema)
        f.load_snapshot_text(9, "\n".join(store.values()))
        fresh = engine_results(f, [checks[i] for i in bad])
        alone = [engine_results(e, [checks[i]])[0] for i in bad]
        again = engine_results(e, checks)
        for k, i in enumerate(bad[:12]):
            print(f"   {checks[i]}: got {got[i]} want {want[i]} fresh {fresh[k]} alone {alone[k]} again {again[i]}")
        f.close()
        st = e.stats()
        print("   stats:", {k: st[k] - st0.get(k, 0) for k in st if isinstance(st[k], (int, float))}, flush=True)
    e.close()


def main():
    names = sys.argv[1:] or list(VARIANTS)
    for v in names:
        rc = pytest.main(["-q", "-m", "gpu", "-p", "no:cacheprovider", "--timeout", "300", *PREFIX])
        print(f"[{v}] prefix rc={rc}", flush=True)
        run(v, VARIANTS[v])


if __name__ == "__main__":
    main()
