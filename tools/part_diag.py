"""Partitioned-engine diagnosis on one GPU (gloo ranks sharing cuda:0): per family / world /
label setting, the mismatches against the oracle and the engine's stats, as JSON lines."""
import json
import os
import socket
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, family, seed, labels, out):
    import torch.distributed as dist
    from gochugaru_amd import engine as E
    from gochugaru_amd.partition import PartitionedChecker
    from tests import gen
    from tests.helpers import parse_check
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    schema, tuples, checks = gen.FAMILIES[family](seed)
    e = E.Engine(device=0, max_depth=gen.FAMILY_DEPTH.get(family, 50), labels=labels)
    if world > 1:
        e.set_partition(rank, world)
    e.load_schema(schema)
    e.load_snapshot_text(1, "\n".join(tuples))
    items = e.make_items([parse_check(c) for c in checks])
    d = torch.from_numpy(items.view(np.uint8).copy()).cuda()
    e.reset_stats()
    if world > 1:
        perm, err = PartitionedChecker(e).check(d, len(items), now_us=gen.NOW_US)
        perm, err = perm.cpu().tolist(), err.cpu().tolist()
    else:
        p, x = e.check_bulk(items, now_us=gen.NOW_US)
        perm, err = p.tolist(), x.tolist()
    st = e.stats()
    json.dump({"perm": perm, "err": err, "tuples": e.tuple_count, "label_checks": int(st["label_checks"]),
               "levels": int(st["levels"]), "retries": int(st["retries"])}, open(f"{out}/r{rank}.json", "w"))
    e.close()
    dist.destroy_process_group()


def main():
    import tempfile
    import torch.multiprocessing as mp
    from tests import gen
    from tests.helpers import oracle_for, parse_check, to_oracle_item
    cfgs = [c.split(":") for c in sys.argv[1:]] or [["nested", "1", "2", "1"]]
    for family, seed, world, labels in cfgs:
        seed, world, labels = int(seed), int(world), labels == "1"
        with tempfile.TemporaryDirectory() as out:
            mp.spawn(_worker, args=(world, _port(), family, seed, labels, out), nprocs=world, join=True)
            outs = [json.load(open(f"{out}/r{r}.json")) for r in range(world)]
        schema, tuples, checks = gen.FAMILIES[family](seed)
        ck = oracle_for(schema, tuples, max_depth=gen.FAMILY_DEPTH.get(family, 50), now=gen.NOW_US / 1e6)
        want = [tuple(ck.check(to_oracle_item(parse_check(c)))) for c in checks]
        got = list(zip(outs[0]["perm"], outs[0]["err"]))
        bad = [(c, w, g) for c, w, g in zip(checks, want, got) if w != tuple(g)]
        same = all(o["perm"] == outs[0]["perm"] and o["err"] == outs[0]["err"] for o in outs)
        print(json.dumps({"family": family, "seed": seed, "world": world, "labels": labels, "n": len(checks),
                          "bad": len(bad), "first": bad[:6], "ranks_agree": same,
                          "label_checks": [o["label_checks"] for o in outs], "levels": [o["levels"] for o in outs],
                          "tuples": [o["tuples"] for o in outs], "total_tuples": len(set(tuples))}), flush=True)


if __name__ == "__main__":
    main()
