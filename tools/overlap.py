"""Kernel concurrency in a window of a rocprofv3 rocpd database: how much of
the wall time each kernel class was running, how much of it overlapped other
classes, and the share of the window with k kernels in flight.

usage: overlap.py run_results.db [t_from_ms t_to_ms]   (times from the first dispatch)
Without a window: the longest stretch with no gap > 2 ms (a run of proves)."""
import collections
import sqlite3
import sys

CLASSES = [("k_accum_range<gg::Fp2>", "accum_g2"), ("k_accum_range", "accum_g1"), ("k_ntt_pass", "ntt"),
           ("k_digits_hist", "sort"), ("k_bin_scatter", "sort"), ("k_seg_", "sort"), ("k_scan", "sort"),
           ("k_bin_starts", "sort"), ("k_set_total", "sort"), ("k_bucket_max", "sort"),
           ("k_bucket_combine", "level2"), ("k_range_tree", "level2"), ("k_reduce", "reduce"),
           ("k_gather_items", "reduce")]


def cls(name):
    for k, v in CLASSES:
        if k in name:
            return v
    return "other"


def main(db, a=None, b=None):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    t0 = rows[0][1]
    ev = [((s - t0) / 1e6, (e - t0) / 1e6, cls(n)) for n, s, e in rows]
    if a is None:  # longest stretch without a gap > 2 ms
        best, cur, end = (0, 0), 0, ev[0][1]
        for i in range(1, len(ev)):
            if ev[i][0] - end > 2.0:
                if ev[i - 1][1] - ev[cur][0] > best[1] - best[0]:
                    best = (ev[cur][0], ev[i - 1][1])
                cur = i
            end = max(end, ev[i][1])
        if end - ev[cur][0] > best[1] - best[0]:
            best = (ev[cur][0], end)
        a, b = best
    a, b = float(a), float(b)
    ev = [(max(s, a), min(e, b), c) for s, e, c in ev if e > a and s < b]
    pts = sorted({a, b} | {s for s, _, _ in ev} | {e for _, e, _ in ev})
    busy = collections.Counter()
    alone = collections.Counter()
    depth = collections.Counter()
    dur = collections.Counter()
    for s, e, c in ev:
        dur[c] += e - s
    for x, y in zip(pts, pts[1:]):
        live = [c for s, e, c in ev if s <= x and e >= y]
        depth[min(len(live), 6)] += y - x
        for c in set(live):
            busy[c] += y - x
        if len(set(live)) == 1:
            alone[live[0]] += y - x
    wall = b - a
    print(f"window {a:.1f} .. {b:.1f} ms ({wall:.1f} ms), {len(ev)} dispatches")
    print(f"{'class':10s} {'sum dur':>9s} {'busy':>9s} {'alone':>9s}")
    for c in sorted(dur, key=lambda k: -dur[k]):
        print(f"{c:10s} {dur[c]:9.1f} {busy[c]:9.1f} {alone[c]:9.1f}")
    print("kernels in flight: " + ", ".join(f"{k}: {100 * v / wall:.1f}%" for k, v in sorted(depth.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
