"""Print the kernel timeline (start offset, duration, gap) of the last N kernel
dispatches in a rocprofv3 rocpd database: shows launch gaps between phases."""
import sqlite3
import sys


def main(db, n=60):
    con = sqlite3.connect(db)
    views = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    if "kernels" not in views:
        print("views:", views)
        return
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    rows = rows[-int(n):]
    t0 = rows[0][1]
    prev_end = t0
    for name, s, e in rows:
        print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f}  gap {(s - prev_end) / 1e3:7.1f}  {name.split('(')[0][:70]}")
        prev_end = e


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else 60)
