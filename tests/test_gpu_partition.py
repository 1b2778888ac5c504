"""Partitioned graphs on the GPU (include/gck.h gck_part_check_with / gck_part_check,
gochugaru_amd/csrc/partition.inc): ranks that each hold only the rows of the objects they own, the
replicated hub hierarchy and the hub memberships of their own subjects check one batch together —
the label join, then the exact-depth level loop with joins — through the engine's own exchange
protocol over a transport. On the one-GPU test box the ranks share cuda:0 and the transport is
gloo (host-staged, gochugaru_amd/partition.py GlooTransport); on a multi-GPU node the same engine
path runs over RCCL. Bar: every rank returns the oracle's results bit-exactly; a rank's load stays
well below the replicated snapshot."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from gochugaru_amd import engine as E
from tests import gen
from tests.helpers import oracle_for, parse_check, to_oracle_item

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _family_engine(rank, world, family, seed, transport):
    # the export stream as text on every rank: each keeps and interns what it owns (names owned by
    # hash, interned by their owner: gck_part_add_tuples_text_with), and the check items are built
    # through the owners too, so every rank holds the same items
    schema, tuples, checks = gen.FAMILIES[family](seed)
    e = E.Engine(device=0, max_depth=gen.FAMILY_DEPTH.get(family, 50))
    e.set_partition(rank, world)
    e.load_schema(schema)
    e.part_load_snapshot_text(transport.c, 1, "\n".join(tuples))
    items = e.part_make_items(transport.c, [parse_check(c) for c in checks])
    return e, torch.from_numpy(items.view(np.uint8).copy()).cuda(), len(items)


def _names_held(e):
    n_types = E.C.c_uint32(0)
    e._lib.gck_type_count(e._h, E.C.byref(n_types))
    return sum(e.interned_names(t) for t in range(n_types.value))


def _synth_engine(rank, world, tuples):
    from tests import synth
    G = synth.build(tuples, device=torch.device("cuda", 0))
    e = E.Engine(device=0)
    e.set_partition(rank, world)
    e.load_schema(synth.SCHEMA)
    e.reserve_objects(synth.T_USER, G.n_users)
    e.reserve_objects(synth.T_GROUP, G.n_groups)
    e.reserve_objects(synth.T_DOC, G.n_docs)
    e.begin_snapshot(1)
    keep = []
    for rel, st, sr, n_rows, off, nbr in G.csrs():
        off32 = off.to(torch.int32).contiguous()
        keep.append(off32)
        e.load_csr(rel, st, sr, n_rows, off32.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
    torch.cuda.synchronize()
    e.commit_snapshot()
    return e, G


def _worker(rank, world, port, family, seed, out_dir, watch):
    import torch.distributed as dist

    from gochugaru_amd.partition import PartitionedChecker

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        if family == "synth":
            from tests import synth
            e, G = _synth_engine(rank, world, seed)
            d_items = synth.checks(G, 4096, seed=77)
            n = 4096
            pc = PartitionedChecker(e)
            if watch:
                C = synth.NestedChurn(G, seed=7)
                e.apply_updates(2, C.batch(max(1000, int(G.n_tuples * 0.001)), cycle=False))
                res["revision"] = e.revision
        else:
            from gochugaru_amd.partition import GlooTransport
            tr = GlooTransport(None, device=True)
            e, d_items, n = _family_engine(rank, world, family, seed, tr)
            res["names"] = _names_held(e)
            pc = PartitionedChecker(e)
        e.reset_stats()
        perm, err = pc.check(d_items, n, now_us=gen.NOW_US)
        st = e.stats()
        perm2, err2 = pc.check(d_items, n, now_us=gen.NOW_US)  # the buffers and the exchange are reused
        assert perm2.cpu().tolist() == perm.cpu().tolist() and err2.cpu().tolist() == err.cpu().tolist()
        with pytest.raises(E.GckError):  # a partitioned engine refuses single-rank checks
            e.check_bulk(np.zeros(1, dtype=E.ITEM_DTYPE))
        res.update({"perm": perm.cpu().tolist(), "err": err.cpu().tolist(), "tuples": e.tuple_count,
                    "label_checks": int(st["label_checks"]), "n": n, "levels": int(st["levels"]),
                    "transport": pc.transport.calls})
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(res, f)
        e.close()
    finally:
        dist.destroy_process_group()


def _run(tmp_path, world, family, seed, watch=False):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), family, seed, str(tmp_path), watch), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    for o in outs[1:]:
        assert o["perm"] == outs[0]["perm"] and o["err"] == outs[0]["err"]
    return outs


FAMILIES = [("nested", 1), ("gdocs", 2), ("gdocs_deep", 3), ("github", 1), ("github", 4), ("cyclic", 2),
            ("near_budget", 3), ("caveated", 2), ("hub_arrow", 1)]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("family,seed", FAMILIES)
def test_partitioned_matches_oracle(tmp_path, world, family, seed):
    """Every family — exclusion / intersection / all() (github), cycles with caveats (cyclic),
    SpiceDB's exact depth accounting under a small budget (near_budget), caveats and expiration
    (caveated) — bit-exact on every rank; no rank holds the whole graph."""
    outs = _run(tmp_path, world, family, seed)
    schema, tuples, checks = gen.FAMILIES[family](seed)
    ck = oracle_for(schema, tuples, max_depth=gen.FAMILY_DEPTH.get(family, 50), now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    got = list(zip(outs[0]["perm"], outs[0]["err"]))
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]
    total = len(set(tuples))
    assert all(o["tuples"] < total for o in outs), [o["tuples"] for o in outs]
    # names interned by their owners only: no rank holds every object's name
    rep = E.Engine(device=0)
    rep.load_schema(schema)
    rep.load_snapshot_text(1, "\n".join(tuples))
    all_names = _names_held(rep)
    rep.close()
    # (names are interned by their owners; on these small dense graphs a rank's rows still reference
    # nearly every object: test_partitioned_ranks_intern_their_own_names measures the fraction)
    assert all(o["names"] <= all_names for o in outs), ([o["names"] for o in outs], all_names)
    print(json.dumps({"family": family, "world": world, "names_held": [o["names"] for o in outs],
                      "replicated_names": all_names}))
    if family == "github":  # the term conjunction (exclusion, intersection) partitions too
        assert outs[0]["label_checks"] > 0


def test_partitioned_config4_shape_matches_replicated(tmp_path):
    """The config-4 graph shape at 2e6 tuples over 3 ranks: every check through the partitioned
    label join (label_checks == N), equal to the single-GPU engine."""
    from tests import synth
    from tests.test_gpu_scale import load_engine, run
    outs = _run(tmp_path, 3, "synth", 2e6)
    G = synth.build(2e6, device=torch.device("cuda", 0))
    e = load_engine(G)
    p, x = run(e, synth.checks(G, 4096, seed=77))
    e.close()
    assert outs[0]["perm"] == p.tolist() and outs[0]["err"] == x.tolist()
    assert sum(1 for v in p if v == E.PERM_HAS) > 1000
    assert all(o["label_checks"] == o["n"] for o in outs), [o["label_checks"] for o in outs]


def test_partitioned_after_watch_matches_oracle(tmp_path):
    """A Watch batch (0.1 % of the tuples: memberships, nesting, viewers; CREATE / TOUCH / DELETE)
    applied on every rank — each keeps what it owns — then a partitioned check: bit-exact against
    the C oracle over the updated graph, and still every check through the label join."""
    from oracle import corc
    from tests import synth
    outs = _run(tmp_path, 2, "synth", 2e6, watch=True)
    G = synth.build(2e6, device=torch.device("cuda", 0))
    C = synth.NestedChurn(G, seed=7)
    C.batch(max(1000, int(G.n_tuples * 0.001)), cycle=False)
    items = synth.checks(G, 4096, seed=77)
    prog, tab = C.oracle()
    cp, ce, _ = corc.check(prog, tab, items.cpu().numpy().view(corc.ITEM_DTYPE).reshape(-1), threads=16)
    assert outs[0]["perm"] == cp.tolist() and outs[0]["err"] == ce.tolist()
    assert all(o["revision"] == 2 for o in outs)
    assert all(o["label_checks"] == o["n"] for o in outs), [o["label_checks"] for o in outs]


_LOAD_PROBE = r"""
import json, sys, torch
sys.path.insert(0, {root!r})
from gochugaru_amd import engine as E
from tests import synth
torch.cuda.set_device(0)
G = synth.build({tuples}, device="cuda")
offs = [(rel, st, sr, n_rows, off.to(torch.int32).contiguous(), nbr) for rel, st, sr, n_rows, off, nbr in G.csrs()]
torch.cuda.synchronize()
free0 = torch.cuda.mem_get_info(0)[0]
e = E.Engine(device=0, workspaces=1)
if {world} > 1:
    e.set_partition({rank}, {world})
e.load_schema(synth.SCHEMA)
e.reserve_objects(synth.T_USER, G.n_users); e.reserve_objects(synth.T_GROUP, G.n_groups); e.reserve_objects(synth.T_DOC, G.n_docs)
e.begin_snapshot(1)
for rel, st, sr, n_rows, off, nbr in offs:
    e.load_csr(rel, st, sr, n_rows, off.data_ptr(), nbr.data_ptr(), nbr.numel(), device=True)
e.commit_snapshot()
torch.cuda.synchronize()
free1 = torch.cuda.mem_get_info(0)[0]
print(json.dumps({{"peak": free0 - free1, "device_bytes": e.device_bytes, "tuples": e.tuple_count}}))
"""


def _load_probe(tuples, rank, world):
    code = _LOAD_PROBE.format(root=ROOT, tuples=tuples, rank=rank, world=world)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_rank_loads_a_fraction(world):
    """Each rank alone in its process (the device's free memory before the engine and after its
    commit: everything the load took and its stream-ordered pool kept — the peak of the load, its
    temporaries included): at most 0.6x the replicated engine's, which holds the whole graph (and
    one workspace, as the partitioned rank's probe does not)."""
    rep = _load_probe(2e6, 0, 1)
    parts = [_load_probe(2e6, r, world) for r in range(world)]
    for p in parts:
        assert p["peak"] <= 0.6 * rep["peak"], (p, rep)
        assert p["tuples"] < rep["tuples"]
    print(json.dumps({"world": world, "replicated": rep, "ranks": parts}))


@pytest.mark.parametrize("family,seed", [("nested", 1), ("gdocs", 2), ("gdocs_deep", 3), ("github", 1)])
def test_rccl_single_rank_matches_oracle(family, seed):
    """gck_part_check over RCCL inside libgck. The one-GPU test box can only hold a one-rank
    communicator (RCCL refuses two ranks on one GPU: "Duplicate GPU detected"), so this runs the RCCL
    path with world 1; the multi-rank protocol — the same engine code over another transport — is
    covered by the gloo tests above."""
    from gochugaru_amd.partition import RcclPartitionedChecker
    schema, tuples, checks = gen.FAMILIES[family](seed)
    e = E.Engine(device=0)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    d_items = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    pc = RcclPartitionedChecker(e)
    perm, err = pc.check(d_items, len(items), now_us=gen.NOW_US)
    got = list(zip(perm.cpu().tolist(), err.cpu().tolist()))
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]
    perm2, err2 = pc.check(d_items, len(items), now_us=gen.NOW_US)  # the communicator is reused
    assert perm2.cpu().tolist() == perm.cpu().tolist() and err2.cpu().tolist() == err.cpu().tolist()
    e.close()


def test_invalid_update_rejected_on_every_rank():
    """A Watch batch with an update only one rank keeps (part_keep) and the schema rejects: every
    rank refuses the whole batch and stays at the old revision (each validates the batch before
    it keeps its own updates, gck_api.cpp apply_updates), so no rank moves ahead of the others.
    The engines of both ranks live in this process: applying a batch needs no exchange."""
    from gochugaru_amd.partition import LocalTransport
    schema, tuples, _ = gen.FAMILIES["gdocs"](2)
    engines = []
    for r in range(2):
        e = E.Engine(device=0)
        e.set_partition(r, 2)
        e.load_schema(schema)
        engines.append(e)
    lt = LocalTransport(2)  # (both ranks' engines in this process, one thread each)
    lt.run(lambda r: engines[r].part_load_snapshot_text(lt.endpoint(r).c, 1, "\n".join(tuples)))
    e0 = engines[0]
    t_doc, t_user, t_folder = e0.type_id("doc"), e0.type_id("user"), e0.type_id("folder")
    viewer = e0.relation_id(t_doc, "viewer")
    n_docs = e0.object_count(t_doc)
    doc0 = next(d for d in range(n_docs) if E.partition_owner(d, 2) == 0)
    doc1 = next(d for d in range(n_docs) if E.partition_owner(d, 2) == 1)

    def update(doc, stype, sid):
        u = np.zeros(1, dtype=E.UPDATE_DTYPE)
        u["op"] = E.UPDATE_CREATE
        t = u["tuple"]
        t["resource_type"], t["relation"], t["resource_id"] = t_doc, viewer, doc
        t["subject_type"], t["subject_relation"], t["subject_id"] = stype, E.ELLIPSIS, sid
        return u
    good = update(doc0, t_user, 0)                # kept by rank 0 only: valid
    bad = update(doc1, t_folder, 0)               # kept by rank 1 only: doc#viewer allows no folder
    batch = np.concatenate([good, bad])
    for r, e in enumerate(engines):
        with pytest.raises(E.GckError) as ei:
            e.apply_updates(2, batch)
        assert ei.value.code == E.GCK_E_INVALID_ARGUMENT, (r, ei.value)
        assert e.revision == 1, (r, e.revision)
    for e in engines:  # the valid update alone applies on both ranks
        e.apply_updates(2, good)
        assert e.revision == 2
    for e in engines:
        e.close()


def _named_config4(seed=5, n_users=20000, n_groups=800, layers=8, n_docs=3000):
    """The config-4 shape with names (users dominate, a layered group DAG, documents granting
    groups), as text: what a partitioned engine reads from the export stream."""
    import random
    rng = random.Random(seed)
    t, per = [], n_groups // layers
    members, viewers = {}, {}
    for g in range(n_groups):
        layer = g // per
        for _ in range(rng.randint(0, 60)):
            u = rng.randrange(n_users)
            members.setdefault(g, []).append(u)
            t.append(f"group:g{g}#member@user:u{u}")
        if layer + 1 < layers:
            for _ in range(rng.randint(0, 3)):
                t.append(f"group:g{g}#member@group:g{(layer + 1) * per + rng.randrange(per)}#member")
    for d in range(n_docs):
        for _ in range(rng.randint(1, 3)):
            g = rng.randrange(n_groups)
            viewers.setdefault(d, []).append(g)
            t.append(f"doc:d{d}#viewer@group:g{g}#member")
    checks = [f"doc:d{rng.randrange(n_docs)}#view@user:u{rng.randrange(n_users)}" for _ in range(1200)]
    for _ in range(300):  # (positives: a direct member of one of the document's groups)
        d = rng.randrange(n_docs)
        g = rng.choice(viewers[d])
        if members.get(g):
            checks.append(f"doc:d{d}#view@user:u{rng.choice(members[g])}")
    checks += [f"group:g{rng.randrange(n_groups)}#member@user:u{rng.randrange(n_users)}" for _ in range(200)]
    checks += [f"doc:d{rng.randrange(n_docs)}#view@group:g{rng.randrange(n_groups)}#member" for _ in range(100)]
    checks += [f"doc:d{rng.randrange(n_docs + 50)}#view@user:u{rng.randrange(n_users + 500)}" for _ in range(100)]
    return gen.NESTED, sorted(set(t)), checks


def _named_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from gochugaru_amd.partition import GlooTransport, PartitionedChecker

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        schema, tuples, checks = _named_config4()
        tr = GlooTransport(None, device=True)
        e, d_items, n = _family_engine_named(rank, world, schema, tuples, checks, tr)
        pc = PartitionedChecker(e)
        e.reset_stats()
        perm, err = pc.check(d_items, n, now_us=gen.NOW_US)
        st = e.stats()
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump({"perm": perm.cpu().tolist(), "err": err.cpu().tolist(), "names": _names_held(e),
                       "tuples": e.tuple_count, "label_checks": int(st["label_checks"]), "n": n}, f)
        e.close()
    finally:
        dist.destroy_process_group()


def _family_engine_named(rank, world, schema, tuples, checks, transport):
    e = E.Engine(device=0)
    e.set_partition(rank, world)
    e.load_schema(schema)
    e.part_load_snapshot_text(transport.c, 1, "\n".join(tuples))
    items = e.part_make_items(transport.c, [parse_check(c) for c in checks])
    return e, torch.from_numpy(items.view(np.uint8).copy()).cuda(), len(items)


def test_partitioned_ranks_intern_their_own_names(tmp_path):
    """Ownership decided before interning (owner = hash(type, name) mod G): the
    config-4 shape read as text by 2 ranks, each keeping its own rows — a group's direct members
    with the members' owner, the hierarchy everywhere — and interning the names of those tuples
    only, through their owners. Each rank's interner holds at most 0.6x the objects the
    replicated engine interns, and every check is bit-exact against the oracle."""
    import torch.multiprocessing as mp
    mp.spawn(_named_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    outs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    assert outs[0]["perm"] == outs[1]["perm"] and outs[0]["err"] == outs[1]["err"]
    schema, tuples, checks = _named_config4()
    rep = E.Engine(device=0)
    rep.load_schema(schema)
    rep.load_snapshot_text(1, "\n".join(tuples))
    all_names = _names_held(rep)
    rep.close()
    ck = oracle_for(schema, tuples, now=gen.NOW_US / 1e6)
    want = [ck.check(to_oracle_item(parse_check(c))) for c in checks]
    got = list(zip(outs[0]["perm"], outs[0]["err"]))
    bad = [(c, w, g) for c, w, g in zip(checks, want, got) if tuple(w) != tuple(g)]
    assert not bad, bad[:5]
    assert sum(1 for p, _ in got if p == E.PERM_HAS) > 200
    print(json.dumps({"names_held": [o["names"] for o in outs], "replicated_names": all_names,
                      "tuples": [o["tuples"] for o in outs], "all_tuples": len(tuples),
                      "label_checks": [o["label_checks"] for o in outs], "n": outs[0]["n"]}))
    for o in outs:
        assert o["names"] <= 0.6 * all_names, (o["names"], all_names)
        assert o["tuples"] <= 0.6 * len(tuples), (o["tuples"], len(tuples))
