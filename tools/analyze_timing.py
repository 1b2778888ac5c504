"""Debug helper: summarise GCK_DEBUG_TIMING=<prefix> records (per-bundle wall-clock spans).
Usage: GCK_DEBUG_TIMING=/tmp/t python bench.py ... ; python tools/analyze_timing.py /tmp/t.bin"""
import sys

import numpy as np

W = 12  # kTimingWords (bundle.inc)
PHASES = ("load", "issue", "claim", "member", "children", "resolve")
TICK_US = 0.01  # wall_clock64 runs at 100 MHz on MI300-class parts


def main(path):
    raw = np.fromfile(path, dtype=np.uint64)
    pos, batches = 0, []
    while pos < len(raw):
        assert raw[pos] == 0xB0DD, "bad header"
        n, B, ndef = int(raw[pos + 1]), int(raw[pos + 2]), int(raw[pos + 3])
        words = W * (n + 1) * 2
        rec = raw[pos + 4: pos + 4 + words].reshape(2, n + 1, W)
        batches.append((n, B, ndef, rec))
        pos += 4 + words
    n, B, ndef, rec = batches[-1]
    print(f"batches={len(batches)} n={n} B={B} deferred={ndef}")
    for stage, name in ((0, "A wavefront bundles"), (1, "B workgroup bundles")):
        r = rec[stage]
        r = r[r[:, 1] > 0].astype(np.float64)
        if not len(r):
            continue
        t0 = r[:, 0].min()
        dur = (r[:, 1] - r[:, 0]) * TICK_US
        lv = r[:, 2]
        ent = r[:, 3]
        span = (r[:, 1].max() - t0) * TICK_US
        start = (r[:, 0] - t0) * TICK_US
        print(f"stage {name}: bundles={len(r)} span={span:.1f}us")
        for q in (50, 90, 99, 99.9, 100):
            print(f"   p{q:<5} dur={np.percentile(dur, q):8.1f}us levels={np.percentile(lv, q):5.1f} "
                  f"entries={np.percentile(ent, q):7.1f} start={np.percentile(start, q):7.1f}us")
        per_level = dur / np.maximum(lv, 1)
        print(f"   us/level p50={np.percentile(per_level, 50):.2f} p90={np.percentile(per_level, 90):.2f}")
        tot = r[:, 4:4 + len(PHASES)].sum(axis=0) * TICK_US
        lvl = lv.sum()
        print("   phase us/level (lane 0): " + " ".join(
            f"{nm}={t / lvl:.2f}" for nm, t in zip(PHASES, tot)))
        # what ends last
        k = np.argsort(r[:, 1])[-5:]
        for i in k:
            print(f"   late: start={start[i]:.1f} dur={dur[i]:.1f} levels={lv[i]:.0f} entries={ent[i]:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
