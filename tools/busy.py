"""GPU busy fraction of the last K gaps-separated runs in a rocpd database:
the union of kernel intervals over the span of each run (a run = dispatches
with no gap > GAP ms), and the idle gaps longer than 50 us inside it.
usage: busy.py run_results.db [gap_ms] [last_runs]"""
import sqlite3
import sys


def main(db, gap=5.0, last=2):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    runs, cur = [], [rows[0]]
    end = rows[0][2]
    for r in rows[1:]:
        if (r[1] - end) / 1e6 > gap:
            runs.append(cur)
            cur = []
        cur.append(r)
        end = max(end, r[2])
    runs.append(cur)
    for run in runs[-last:]:
        t0, busy, hi, gaps = run[0][1], 0.0, run[0][1], []
        for n, s, e in run:
            if s > hi:
                if (s - hi) / 1e3 > 50:
                    gaps.append(((hi - t0) / 1e6, (s - hi) / 1e3, prev))
                busy += (e - s)
                hi = e
            elif e > hi:
                busy += e - hi
                hi = e
            prev = n[:60]
        span = (hi - t0) / 1e6
        print("run: span %.2f ms, busy %.2f ms (%.1f%%), %d dispatches" % (span, busy / 1e6, 100 * busy / 1e6 / span,
                                                                       len(run)))
        for at, g, after in sorted(gaps, key=lambda x: -x[1])[:12]:
            print("   gap %.0f us at %.2f ms after %s" % (g, at, after))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], float(a[1]) if len(a) > 1 else 5.0, int(a[2]) if len(a) > 2 else 2)
