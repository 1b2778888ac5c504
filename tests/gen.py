"""Seeded synthetic schemas + relationship graphs for parity tests (small sizes: the Python
oracle must finish in seconds). Most families are acyclic and far below the depth budget;
``cyclic`` and ``near_budget`` exercise SpiceDB's depth semantics:
cyclic userset / arrow data, caveats on the way into cycles, and re-converging paths that
straddle a small budget (FAMILY_DEPTH)."""
import random

GDOCS = """
definition user {}
definition group {
  relation member: user | group#member
}
definition folder {
  relation parent: folder
  relation viewer: user | group#member
  relation editor: user | group#member
  permission edit = editor + parent->edit
  permission view = viewer + edit + parent->view
}
definition doc {
  relation parent: folder
  relation owner: user
  relation viewer: user | user:* | group#member
  relation editor: user | group#member
  permission edit = owner + editor + parent->edit
  permission view = viewer + edit + parent->view
}
"""

GITHUB = """
definition user {}
definition team {
  relation maintainer: user
  relation direct_member: user | team#member
  permission member = maintainer + direct_member
}
definition org {
  relation admin: user
  relation member: user | team#member
  permission is_member = admin + member
}
definition repo {
  relation org: org
  relation reader: user | team#member
  relation writer: user | team#member
  relation admin: user | team#member
  relation banned: user
  permission read = (reader + writer + admin + org->is_member) - banned
  permission write = (writer + admin) & org->is_member
  permission admin_all = org.all(is_member)
}
"""

CAVEATED = """
caveat only_on_tuesday(day_of_the_week string) {
  day_of_the_week == "tuesday"
}
definition user {}
definition group {
  relation member: user | group#member | user with only_on_tuesday
}
definition doc {
  relation viewer: user | group#member | user with only_on_tuesday | user with expiration
  relation editor: user | user with expiration
  permission edit = editor
  permission view = viewer + edit
  permission strict = viewer & editor
}
use expiration
"""

NESTED = """
definition user {}
definition group {
  relation member: user | group#member
}
definition doc {
  relation viewer: group#member
  permission view = viewer
}
"""


def _pick(rng, n):
    return rng.randrange(n)


def gdocs(seed, n_users=60, n_groups=25, n_folders=30, n_docs=60):
    rng = random.Random(seed)
    t = []
    for g in range(n_groups):
        for _ in range(rng.randint(0, 4)):
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}")
        for _ in range(rng.randint(0, 2)):
            h = rng.randrange(g + 1, n_groups + 1)
            if h < n_groups:
                t.append(f"group:g{g}#member@group:g{h}#member")
    for f in range(n_folders):
        if f > 0 and rng.random() < 0.8:
            t.append(f"folder:f{f}#parent@folder:f{rng.randrange(f)}")
        for rel in ("viewer", "editor"):
            for _ in range(rng.randint(0, 2)):
                if rng.random() < 0.5:
                    t.append(f"folder:f{f}#{rel}@user:u{_pick(rng, n_users)}")
                else:
                    t.append(f"folder:f{f}#{rel}@group:g{_pick(rng, n_groups)}#member")
    for d in range(n_docs):
        if rng.random() < 0.8:
            t.append(f"doc:d{d}#parent@folder:f{_pick(rng, n_folders)}")
        if rng.random() < 0.5:
            t.append(f"doc:d{d}#owner@user:u{_pick(rng, n_users)}")
        for rel in ("viewer", "editor"):
            for _ in range(rng.randint(0, 2)):
                x = rng.random()
                if x < 0.5:
                    t.append(f"doc:d{d}#{rel}@user:u{_pick(rng, n_users)}")
                elif x < 0.97 or rel == "editor":
                    t.append(f"doc:d{d}#{rel}@group:g{_pick(rng, n_groups)}#member")
                else:
                    t.append(f"doc:d{d}#viewer@user:*")
    checks = []
    for _ in range(400):
        x = rng.random()
        if x < 0.45:
            checks.append(f"doc:d{_pick(rng, n_docs + 3)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users + 3)}")
        elif x < 0.75:
            checks.append(f"folder:f{_pick(rng, n_folders)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users)}")
        elif x < 0.9:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@user:u{_pick(rng, n_users)}")
        else:
            checks.append(f"doc:d{_pick(rng, n_docs)}#view@group:g{_pick(rng, n_groups)}#member")
    return GDOCS, t, checks


def github(seed, n_users=50, n_teams=20, n_orgs=6, n_repos=50):
    rng = random.Random(seed)
    t = []
    for tm in range(n_teams):
        for _ in range(rng.randint(0, 2)):
            t.append(f"team:t{tm}#maintainer@user:u{_pick(rng, n_users)}")
        for _ in range(rng.randint(0, 3)):
            t.append(f"team:t{tm}#direct_member@user:u{_pick(rng, n_users)}")
        if rng.random() < 0.5:
            h = rng.randrange(tm + 1, n_teams + 1)
            if h < n_teams:
                t.append(f"team:t{tm}#direct_member@team:t{h}#member")
    for o in range(n_orgs):
        t.append(f"org:o{o}#admin@user:u{_pick(rng, n_users)}")
        for _ in range(rng.randint(1, 6)):
            if rng.random() < 0.6:
                t.append(f"org:o{o}#member@user:u{_pick(rng, n_users)}")
            else:
                t.append(f"org:o{o}#member@team:t{_pick(rng, n_teams)}#member")
    for r in range(n_repos):
        for _ in range(rng.randint(1, 2)):
            t.append(f"repo:r{r}#org@org:o{_pick(rng, n_orgs)}")
        for rel in ("reader", "writer", "admin"):
            for _ in range(rng.randint(0, 2)):
                if rng.random() < 0.6:
                    t.append(f"repo:r{r}#{rel}@user:u{_pick(rng, n_users)}")
                else:
                    t.append(f"repo:r{r}#{rel}@team:t{_pick(rng, n_teams)}#member")
        if rng.random() < 0.3:
            t.append(f"repo:r{r}#banned@user:u{_pick(rng, n_users)}")
    checks = []
    for _ in range(400):
        x = rng.random()
        if x < 0.8:
            checks.append(f"repo:r{_pick(rng, n_repos)}#{rng.choice(['read', 'write', 'admin_all'])}@user:u{_pick(rng, n_users)}")
        else:
            checks.append(f"team:t{_pick(rng, n_teams)}#member@user:u{_pick(rng, n_users)}")
    return GITHUB, t, checks


def caveated(seed, n_users=40, n_groups=15, n_docs=40):
    """Caveated and expiring tuples; ~half of the expiring ones are already expired at
    NOW_US (2025-10-03)."""
    rng = random.Random(seed)
    t = []
    past, future = "2020-01-01T00:00:00Z", "2999-01-01T00:00:00Z"
    for g in range(n_groups):
        for _ in range(rng.randint(0, 4)):
            cav = "[only_on_tuesday]" if rng.random() < 0.2 else ""
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}{cav}")
        if rng.random() < 0.5:
            h = rng.randrange(g + 1, n_groups + 1)
            if h < n_groups:
                t.append(f"group:g{g}#member@group:g{h}#member")
    for d in range(n_docs):
        for _ in range(rng.randint(0, 3)):
            x = rng.random()
            u = _pick(rng, n_users)
            if x < 0.3:
                t.append(f"doc:d{d}#viewer@user:u{u}")
            elif x < 0.5:
                t.append(f"doc:d{d}#viewer@user:u{u}[only_on_tuesday]")
            elif x < 0.6:
                t.append(f'doc:d{d}#viewer@user:u{u}[only_on_tuesday:{{"day_of_the_week":"tuesday"}}]')
            elif x < 0.75:
                t.append(f"doc:d{d}#viewer@user:u{u}[expiration:{rng.choice([past, future])}]")
            else:
                t.append(f"doc:d{d}#viewer@group:g{_pick(rng, n_groups)}#member")
        for _ in range(rng.randint(0, 2)):
            u = _pick(rng, n_users)
            if rng.random() < 0.5:
                t.append(f"doc:d{d}#editor@user:u{u}")
            else:
                t.append(f"doc:d{d}#editor@user:u{u}[expiration:{rng.choice([past, future])}]")
    # bias half of the checks towards subjects that appear on the document
    users_of = {}
    for s in t:
        if s.startswith("doc:") and "@user:" in s:
            d = s[4:s.index("#")]
            u = s.split("@user:")[1].split("[")[0]
            users_of.setdefault(d, []).append(u)
    checks = []
    for _ in range(300):
        d = _pick(rng, n_docs)
        perm = rng.choice(['view', 'edit', 'strict'])
        if rng.random() < 0.6 and users_of.get(f"d{d}"):
            u = rng.choice(users_of[f"d{d}"])
        else:
            u = f"u{_pick(rng, n_users)}"
        checks.append(f"doc:d{d}#{perm}@user:{u}")
    return CAVEATED, t, checks


def nested(seed, n_users=200, n_groups=120, layers=8, n_docs=80):
    """Layered group DAG (config 4 shape at toy scale)."""
    rng = random.Random(seed)
    t = []
    per = n_groups // layers
    for g in range(n_groups):
        layer = g // per
        for _ in range(rng.randint(0, 5)):
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}")
        if layer + 1 < layers:
            for _ in range(rng.randint(0, 3)):
                h = (layer + 1) * per + _pick(rng, per)
                if h < n_groups:
                    t.append(f"group:g{g}#member@group:g{h}#member")
    for d in range(n_docs):
        for _ in range(rng.randint(1, 3)):
            t.append(f"doc:d{d}#viewer@group:g{_pick(rng, per * 2)}#member")
    checks = [f"doc:d{_pick(rng, n_docs)}#view@user:u{_pick(rng, n_users)}" for _ in range(400)]
    # the closure-join shapes besides doc#view@user: a group's own members, userset subjects,
    # subjects of an unlisted type (left to the bundles), unknown objects
    checks += [f"group:g{_pick(rng, n_groups)}#member@user:u{_pick(rng, n_users)}" for _ in range(60)]
    checks += [f"doc:d{_pick(rng, n_docs)}#view@group:g{_pick(rng, n_groups)}#member" for _ in range(40)]
    checks += [f"group:g{_pick(rng, n_groups)}#member@group:g{_pick(rng, n_groups)}#member" for _ in range(30)]
    checks += [f"doc:d{_pick(rng, n_docs)}#viewer@group:g{_pick(rng, n_groups)}#member" for _ in range(20)]
    checks += [f"doc:d{_pick(rng, n_docs + 5)}#view@user:u{_pick(rng, n_users + 5)}" for _ in range(20)]
    checks += [f"doc:d{_pick(rng, n_docs)}#view@doc:d{_pick(rng, n_docs)}" for _ in range(5)]
    return NESTED, t, checks


def gdocs_deep(seed, n_users=80, n_groups=40, n_folders=40, n_docs=60):
    """GDocs schema without wildcards (every doc/folder permission is a plain union, so checks
    run bidirectionally) and long group / folder chains; a fifth of the checks have a userset
    subject."""
    rng = random.Random(seed)
    t = []
    for g in range(n_groups):
        for _ in range(rng.randint(0, 3)):
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}")
        if g + 1 < n_groups and rng.random() < 0.7:  # a chain with occasional branches
            t.append(f"group:g{g}#member@group:g{g + 1 + (rng.random() < 0.2)}#member".replace(f"g{n_groups}#", f"g{n_groups - 1}#"))
    for f in range(n_folders):
        if f > 0 and rng.random() < 0.9:
            t.append(f"folder:f{f}#parent@folder:f{max(0, f - 1 - _pick(rng, 2))}")
        for rel in ("viewer", "editor"):
            for _ in range(rng.randint(0, 1)):
                if rng.random() < 0.4:
                    t.append(f"folder:f{f}#{rel}@user:u{_pick(rng, n_users)}")
                else:
                    t.append(f"folder:f{f}#{rel}@group:g{_pick(rng, n_groups)}#member")
    for d in range(n_docs):
        if rng.random() < 0.9:
            t.append(f"doc:d{d}#parent@folder:f{_pick(rng, n_folders)}")
        if rng.random() < 0.3:
            t.append(f"doc:d{d}#owner@user:u{_pick(rng, n_users)}")
        for rel in ("viewer", "editor"):
            if rng.random() < 0.4:
                if rng.random() < 0.5:
                    t.append(f"doc:d{d}#{rel}@user:u{_pick(rng, n_users)}")
                else:
                    t.append(f"doc:d{d}#{rel}@group:g{_pick(rng, n_groups)}#member")
    t = sorted(set(x for x in t if "#member@group:g" not in x or x.split("#")[0] != x.split("@")[1].split("#")[0]))
    checks = []
    for _ in range(400):
        x = rng.random()
        if x < 0.5:
            checks.append(f"doc:d{_pick(rng, n_docs + 2)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users + 2)}")
        elif x < 0.65:
            checks.append(f"folder:f{_pick(rng, n_folders)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users)}")
        elif x < 0.8:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@user:u{_pick(rng, n_users)}")
        elif x < 0.9:
            checks.append(f"doc:d{_pick(rng, n_docs)}#view@group:g{_pick(rng, n_groups)}#member")
        else:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@group:g{_pick(rng, n_groups)}#member")
    return GDOCS, t, checks


CYCLIC = """
caveat only_on_tuesday(day_of_the_week string) {
  day_of_the_week == "tuesday"
}
definition user {}
definition group {
  relation member: user | group#member | user with only_on_tuesday | group#member with only_on_tuesday
}
definition folder {
  relation parent: folder | folder with only_on_tuesday
  relation viewer: user | group#member
  relation banned: user | group#member
  permission view = (viewer + parent->view) - banned
  permission every = parent.all(view)
}
definition doc {
  relation parent: folder
  relation viewer: user | group#member | group#member with only_on_tuesday
  relation editor: user | group#member
  permission edit = editor + parent->view
  permission view = viewer + edit
  permission strict = viewer & edit
}
"""


def cyclic(seed, n_users=30, n_groups=18, n_folders=16, n_docs=30):
    """Cyclic group membership and folder parents (self-loops included), some of the cycle
    edges caveated: a check that never reaches its subject ends in the depth error, one that
    reaches it first is HAS, and a caveat on the way into a cycle must not hide the error
    (and3(false, ERR) = ERR in the oracle)."""
    rng = random.Random(seed)
    t = []
    tue = "[only_on_tuesday]"
    for g in range(n_groups):
        for _ in range(rng.randint(0, 2)):
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}" + (tue if rng.random() < 0.2 else ""))
        for _ in range(rng.randint(0, 2)):
            h = _pick(rng, n_groups)  # any direction: cycles and self-loops
            t.append(f"group:g{g}#member@group:g{h}#member" + (tue if rng.random() < 0.25 else ""))
    for f in range(n_folders):
        for _ in range(rng.randint(0, 2)):
            t.append(f"folder:f{f}#parent@folder:f{_pick(rng, n_folders)}" + (tue if rng.random() < 0.2 else ""))
        for rel in ("viewer", "banned"):
            for _ in range(rng.randint(0, 1 if rel == "banned" else 2)):
                if rng.random() < 0.5:
                    t.append(f"folder:f{f}#{rel}@user:u{_pick(rng, n_users)}")
                else:
                    t.append(f"folder:f{f}#{rel}@group:g{_pick(rng, n_groups)}#member")
    for d in range(n_docs):
        if rng.random() < 0.7:
            t.append(f"doc:d{d}#parent@folder:f{_pick(rng, n_folders)}")
        for rel in ("viewer", "editor"):
            for _ in range(rng.randint(0, 2)):
                x = rng.random()
                if x < 0.4:
                    t.append(f"doc:d{d}#{rel}@user:u{_pick(rng, n_users)}")
                elif x < 0.8 or rel == "editor":
                    t.append(f"doc:d{d}#{rel}@group:g{_pick(rng, n_groups)}#member")
                else:
                    t.append(f"doc:d{d}#viewer@group:g{_pick(rng, n_groups)}#member{tue}")
    t = sorted(set(t))
    checks = []
    for _ in range(300):
        x = rng.random()
        if x < 0.4:
            checks.append(f"doc:d{_pick(rng, n_docs + 2)}#{rng.choice(['view', 'edit', 'strict'])}@user:u{_pick(rng, n_users + 2)}")
        elif x < 0.65:
            checks.append(f"folder:f{_pick(rng, n_folders)}#{rng.choice(['view', 'every'])}@user:u{_pick(rng, n_users)}")
        elif x < 0.85:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@user:u{_pick(rng, n_users)}")
        elif x < 0.93:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@group:g{_pick(rng, n_groups)}#member")
        else:
            checks.append(f"doc:d{_pick(rng, n_docs)}#view@group:g{_pick(rng, n_groups)}#member")
    return CYCLIC, t, checks


def near_budget(seed, n_users=40, n_groups=48, n_folders=24, n_docs=40):
    """Acyclic, but with re-converging paths of different lengths around a small depth budget
    (FAMILY_DEPTH: 8): a vertex is reachable both within and beyond the budget, so the answer
    depends on SpiceDB's exact depth accounting (every dispatch path counts, not the shortest)."""
    rng = random.Random(seed)
    t = []
    for g in range(n_groups):  # chains g -> g+1 (long paths) plus skips g -> g+k (short ones)
        for _ in range(rng.randint(0, 2)):
            t.append(f"group:g{g}#member@user:u{_pick(rng, n_users)}")
        if g + 1 < n_groups and rng.random() < 0.85:
            t.append(f"group:g{g}#member@group:g{g + 1}#member")
        if rng.random() < 0.4:
            h = g + rng.randint(2, 6)
            if h < n_groups:
                t.append(f"group:g{g}#member@group:g{h}#member")
    for f in range(n_folders):
        if f > 0 and rng.random() < 0.9:
            t.append(f"folder:f{f}#parent@folder:f{f - 1}")
        if f > 2 and rng.random() < 0.3:
            t.append(f"folder:f{f}#parent@folder:f{f - rng.randint(2, 3)}")
        if rng.random() < 0.5:
            t.append(f"folder:f{f}#viewer@group:g{_pick(rng, n_groups)}#member")
        if rng.random() < 0.3:
            t.append(f"folder:f{f}#editor@user:u{_pick(rng, n_users)}")
    for d in range(n_docs):
        t.append(f"doc:d{d}#parent@folder:f{_pick(rng, n_folders)}")
        if rng.random() < 0.5:
            t.append(f"doc:d{d}#viewer@group:g{_pick(rng, n_groups)}#member")
        if rng.random() < 0.3:
            t.append(f"doc:d{d}#editor@user:u{_pick(rng, n_users)}")
    t = sorted(set(t))
    checks = []
    for _ in range(300):
        x = rng.random()
        if x < 0.5:
            checks.append(f"doc:d{_pick(rng, n_docs)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users)}")
        elif x < 0.75:
            checks.append(f"folder:f{_pick(rng, n_folders)}#{rng.choice(['view', 'edit'])}@user:u{_pick(rng, n_users)}")
        else:
            checks.append(f"group:g{_pick(rng, n_groups)}#member@user:u{_pick(rng, n_users)}")
    return GDOCS_NOWILD, t, checks


GDOCS_NOWILD = GDOCS.replace("relation viewer: user | user:* | group#member", "relation viewer: user | group#member")


HUB_ARROW = """
definition user {
  relation manager: user
}
definition org {
  relation member: user
  permission member_mgr = member->manager
}
definition repo {
  relation org: org
  relation reader: user
  permission read = reader + org->member
  permission audit = org->member_mgr
}
"""


def hub_arrow(seed, n_users=60, n_orgs=10, n_repos=50):
    """A hub relation (org#member: arrows point at it) whose rows are also read as an arrow's
    tupleset outside the hub (org#member_mgr = member->manager). A partitioned graph keeps a hub's
    direct tuples with their subjects' owners, so such a relation must not be a hub there
    (labels.inc partition_rules)."""
    rng = random.Random(seed)
    t = []
    for u in range(n_users):
        if rng.random() < 0.6:
            t.append(f"user:u{u}#manager@user:u{_pick(rng, n_users)}")
    for o in range(n_orgs):
        for _ in range(rng.randint(1, 6)):
            t.append(f"org:o{o}#member@user:u{_pick(rng, n_users)}")
    for r in range(n_repos):
        if rng.random() < 0.9:
            t.append(f"repo:r{r}#org@org:o{_pick(rng, n_orgs)}")
        for _ in range(rng.randint(0, 2)):
            t.append(f"repo:r{r}#reader@user:u{_pick(rng, n_users)}")
    t = sorted(set(t))
    checks = []
    for _ in range(300):
        x = rng.random()
        if x < 0.35:
            checks.append(f"repo:r{_pick(rng, n_repos)}#read@user:u{_pick(rng, n_users)}")
        elif x < 0.65:
            checks.append(f"repo:r{_pick(rng, n_repos)}#audit@user:u{_pick(rng, n_users)}")
        elif x < 0.85:
            checks.append(f"org:o{_pick(rng, n_orgs)}#member_mgr@user:u{_pick(rng, n_users)}")
        else:
            checks.append(f"org:o{_pick(rng, n_orgs)}#member@user:u{_pick(rng, n_users)}")
    return HUB_ARROW, t, checks


def check_contexts(seed, n):
    """Check-time caveat contexts for n checks (CheckBulkPermissionsRequestItem.Context):
    none, a satisfying one or a failing one for only_on_tuesday, and an unrelated key."""
    rng = random.Random(seed * 7919 + 17)
    opts = [None, None, {"day_of_the_week": "tuesday"}, {"day_of_the_week": "monday"}, {"other": 1}]
    return [rng.choice(opts) for _ in range(n)]


FAMILIES = {"gdocs": gdocs, "github": github, "caveated": caveated, "nested": nested,
            "gdocs_deep": gdocs_deep, "cyclic": cyclic, "near_budget": near_budget, "hub_arrow": hub_arrow}
# the dispatch depth budget a family is checked under (default: SpiceDB's 50)
FAMILY_DEPTH = {"near_budget": 8}
NOW_US = 1759449600 * 1_000_000  # 2025-10-03T00:00:00Z
