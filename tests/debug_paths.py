"""Debug helper (not collected by pytest): compare engine paths against the oracle and print
per-check mismatches. Usage: python tests/debug_paths.py"""
import sys

sys.path.insert(0, ".")

from tests import gen  # noqa: E402
from tests.helpers import load_golden, oracle_for, parse_check, to_oracle_item  # noqa: E402
from tests.test_gpu_parity import PATHS, device_results, make_engine  # noqa: E402

SEM = load_golden("semantics.json")


def main():
    cases = []
    s = SEM["suites"][0]
    cases.append(("sem-rewrites", s["schema"], s["tuples"], [c[0] for c in s["checks"]]))
    for fam in sorted(gen.FAMILIES):
        sc, t, ch = gen.FAMILIES[fam](1)
        cases.append((fam, sc, t, ch))
    for name, schema, tuples, checks in cases:
        ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
        want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
        for path, kw in sorted(PATHS.items()):
            e = make_engine(schema, tuples, **kw)
            got = device_results(e, checks, now_us=gen.NOW_US)
            bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != g]
            st = e.stats()
            print(f"{name:14s} {path:16s} mismatches={len(bad):4d}/{len(checks)} deferred={st['deferred']}", bad[:4])
            e.close()


if __name__ == "__main__":
    main()
