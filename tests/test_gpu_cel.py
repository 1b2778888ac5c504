"""Caveats over CEL timestamps, durations, IP addresses and string functions
through the whole check path: stored relationship contexts plus check-time contexts, evaluated
by the host CEL evaluator into the per-call outcome table the device walk reads. Bit-exact
against the oracle (whose CEL restatement tests/test_cel.py pins to hand-derived answers)."""
import random

import pytest

from tests.helpers import oracle_for, parse_check, to_oracle_item
from tests.test_gpu_parity import device_results, make_engine

pytestmark = pytest.mark.gpu

SCHEMA = """
caveat in_window(now timestamp, start timestamp, ttl duration) { now >= start && now - start < ttl }
caveat from_network(ip ipaddress, cidr string) { ip.in_cidr(cidr) }
caveat tagged(tag string) { tag.startsWith("team-") && size(tag) <= 9 }
definition user {}
definition group { relation member: user | user with tagged }
definition doc {
  relation viewer: user with in_window | user with from_network | group#member
  relation editor: user with from_network
  permission view = viewer + editor
}
"""

NOW_US = 1759449600 * 1_000_000  # 2025-10-03T00:00:00Z (expiration clock; caveats use contexts)


def graph(seed):
    rng = random.Random(seed)
    users = [f"u{i}" for i in range(30)]
    tuples = []
    for d in range(20):
        for u in rng.sample(users, 4):
            k = rng.randrange(4)
            if k == 0:
                start = rng.choice(["2025-10-01T00:00:00Z", "2025-10-02T12:00:00Z", "2025-09-01T00:00:00Z"])
                tuples.append(f'doc:d{d}#viewer@user:{u}[in_window:{{"start":"{start}"}}]')
            elif k == 1:
                cidr = rng.choice(["10.0.0.0/8", "192.168.0.0/16", "2001:db8::/32"])
                tuples.append(f'doc:d{d}#viewer@user:{u}[from_network:{{"cidr":"{cidr}"}}]')
            elif k == 2:
                tuples.append(f'doc:d{d}#editor@user:{u}[from_network:{{"cidr":"10.1.0.0/16","ip":"10.1.2.3"}}]')
            else:
                tuples.append(f"doc:d{d}#viewer@group:g{d % 5}#member")
    for g in range(5):
        for u in rng.sample(users, 5):
            tag = rng.choice(["team-a", "team-blue", "ops", None])
            tuples.append(f"group:g{g}#member@user:{u}" + (f'[tagged:{{"tag":"{tag}"}}]' if tag else "[tagged]"))
    checks = [f"doc:d{rng.randrange(20)}#view@user:{rng.choice(users)}" for _ in range(300)]
    return tuples, checks


def contexts(seed, n):
    rng = random.Random(seed + 99)
    opts = [None,
            {"now": "2025-10-03T00:00:00Z", "ttl": "48h"},
            {"now": "2025-10-03T00:00:00Z", "ttl": "1h"},
            {"ip": "10.1.2.3"}, {"ip": "192.168.7.7", "now": "2025-10-02T13:00:00Z"},
            {"ip": "2001:db8::5", "tag": "team-xyzw"},
            {"now": "2025-10-02T12:30:00Z", "ttl": "45m", "ip": "8.8.8.8", "tag": "team-a"}]
    return [rng.choice(opts) for _ in range(n)]


@pytest.mark.parametrize("path", [{}, {"wide_only": True}, {"bidir": False}])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_temporal_and_network_caveats_match_oracle(seed, path):
    tuples, checks = graph(seed)
    ctxs = contexts(seed, len(checks))
    ck = oracle_for(SCHEMA, tuples, now=NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c), x)) for c, x in zip(checks, ctxs)]
    e = make_engine(SCHEMA, tuples, **path)
    got = device_results(e, checks, now_us=NOW_US, contexts=ctxs)
    bad = [(c, x, w, g) for c, x, w, g in zip(checks, ctxs, want, got) if w != g]
    assert not bad, bad[:10]
    kinds = {w[0] for w in want}
    assert {1, 2, 3} <= kinds  # NO, HAS and CONDITIONAL all occur
    e.close()
