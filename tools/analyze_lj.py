"""Per-wave phase timing of k_label_join (GCK_DEBUG_TIMING=<prefix> with the TIMING=1 build writes
<prefix>_lj.bin): where a launch's time goes. wall_clock64 ticks at 100 MHz (10 ns).
    python tools/analyze_lj.py <prefix>_lj.bin"""
import sys

import numpy as np

TICK_US = 0.01
W = 11  # labels.inc kLjTimingWords: start, items + table staged, slot lines staged, decided, end, list / ext checks,
#        deferred: no root / slot overflow / dirty without overlay / overlay hit


def launches(path):
    raw = np.fromfile(path, dtype=np.uint64)
    at = 0
    while at + 2 <= raw.size:
        assert raw[at] == 0x1AB0, "bad record"
        nw = int(raw[at + 1])
        rec = raw[at + 2: at + 2 + W * nw].reshape(nw, W).astype(np.int64)
        at += 2 + W * nw
        yield rec


def pct(x):
    return " ".join(f"{q}:{np.percentile(x, q):7.2f}" for q in (10, 50, 90, 99, 100))


def main(path):
    spans, recs = [], []
    for r in launches(path):
        r = r[r[:, 0] > 0]
        if not len(r):
            continue
        t0 = r[:, 0].min()
        spans.append((r[:, 4].max() - t0) * TICK_US)
        recs.append(np.column_stack([(r[:, 0] - t0) * TICK_US, (r[:, 1] - r[:, 0]) * TICK_US,
                                     (r[:, 2] - r[:, 1]) * TICK_US, (r[:, 3] - r[:, 2]) * TICK_US,
                                     (r[:, 4] - r[:, 3]) * TICK_US, (r[:, 4] - t0) * TICK_US, r[:, 5], r[:, 6],
                                     r[:, 7], r[:, 8], r[:, 9], r[:, 10]]))
    a = np.concatenate(recs)
    print(f"launches {len(spans)}  span us (first wave start -> last wave end): {pct(np.array(spans))}")
    names = ["start offset", "items + table", "slot lines", "decide", "results + summary", "wave end offset"]
    for k, nm in enumerate(names):
        print(f"{nm:>18}: {pct(a[:, k])}")
    # the decide phase by what the wave's checks read
    dec, nl, ne = a[:, 3], a[:, 6], a[:, 7]
    for nm, m in (("plain waves", (nl == 0) & (ne == 0)), ("with a cover list", (nl > 0) & (ne == 0)),
                  ("with an ext record", (ne > 0) & (nl == 0)), ("with both", (nl > 0) & (ne > 0))):
        if m.any():
            print(f"{'decide, ' + nm:>30} ({m.mean() * 100:5.1f} % of waves): {pct(dec[m])}")
    slow = a[:, 5] >= np.percentile(a[:, 5], 99)
    print(f"slowest 1 % of waves: list checks {nl[slow].mean():.2f} ext checks {ne[slow].mean():.2f} "
          f"(all waves: {nl.mean():.2f} / {ne.mean():.2f})")
    n_launch = max(1, len(spans))
    print("deferred checks per launch: no label root %.1f, slot overflow %.1f, dirty subject (no overlay) %.1f, "
          "overlay hit %.1f" % tuple(a[:, 8 + k].sum() / n_launch for k in range(4)))


if __name__ == "__main__":
    main(sys.argv[1])
