"""Timeline of one proof in a rocprofv3 kernel trace (rocpd sqlite): kernels
longer than min_ms within [before, after] ms of the LAST dispatch whose name
contains `anchor`, with start / duration in ms from the first listed kernel,
stream and hardware queue -- to see which task waits for which.
usage: timeline.py run_results.db anchor [before_ms] [after_ms] [min_ms] [nth_from_last]"""
import sqlite3
import sys


def main(argv):
    db, anchor = argv[0], argv[1]
    before = float(argv[2]) if len(argv) > 2 else 40.0
    after = float(argv[3]) if len(argv) > 3 else 10.0
    min_ms = float(argv[4]) if len(argv) > 4 else 0.15
    con = sqlite3.connect(db)
    ks = con.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    nth = int(argv[5]) if len(argv) > 5 else 1
    a = [k for k in ks if anchor in k[0]][-nth]
    lo, hi = a[1] - before * 1e6, a[2] + after * 1e6
    sel = [k for k in ks if lo <= k[1] <= hi]
    t0 = sel[0][1]
    for n, s, e, st, q in sel:
        d = (e - s) * 1e-6
        if d >= min_ms:
            print(f"{(s - t0) * 1e-6:9.3f} {d:8.3f}  st{st:<4} q{q:<3} {n.split('(')[0][:70]}")


if __name__ == "__main__":
    main(sys.argv[1:])
