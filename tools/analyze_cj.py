"""Per-wave phase timing of k_closure_join (GCK_DEBUG_TIMING=<prefix> with the TIMING=1 build
writes <prefix>_cj.bin): where a launch's time goes. wall_clock64 ticks at 100 MHz (10 ns)."""
import sys

import numpy as np

TICK_US = 0.01
W = 11  # closure.inc kCjTimingWords


def launches(path):
    raw = np.fromfile(path, dtype=np.uint64)
    at = 0
    while at + 2 <= raw.size:
        assert raw[at] == 0xC10C, "bad record"
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
        t0 = r[:, 0].min()
        spans.append((r[:, 4].max() - t0) * TICK_US)
        recs.append(np.column_stack([(r[:, 0] - t0) * TICK_US, (r[:, 1] - r[:, 0]) * TICK_US,
                                     (r[:, 8] - r[:, 1]) * TICK_US, (r[:, 10] - r[:, 8]) * TICK_US,
                                     (r[:, 9] - r[:, 10]) * TICK_US,
                                     (r[:, 2] - r[:, 9]) * TICK_US, (r[:, 3] - r[:, 2]) * TICK_US,
                                     (r[:, 4] - r[:, 3]) * TICK_US, (r[:, 4] - t0) * TICK_US,
                                     r[:, 5], r[:, 6], r[:, 7]]))
    a = np.concatenate(recs)
    print(f"launches {len(spans)}  span us (first wave start -> last wave end): {pct(np.array(spans))}")
    names = ["start offset", "table copy", "items", "slots", "lists", "extents", "tasks", "end", "wave end offset"]
    for k, nm in enumerate(names):
        print(f"{nm:>16} us  {pct(a[:, k])}")
    print(f"{'tasks/wave':>16}     {pct(a[:, 9])}")
    print(f"{'probes/wave':>16}     {pct(a[:, 10])}")


if __name__ == "__main__":
    main(sys.argv[1])
