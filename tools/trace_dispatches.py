"""List individual kernel dispatches (name, grid, workgroup, LDS, duration) from
a rocprofv3 --kernel-trace database (rocpd sqlite), optionally filtered by a
name substring; used to split the NTT passes of one transform.
usage: trace_dispatches.py run_results.db [substring] [last_n]"""
import sqlite3
import sys


def main(db, sub="", last=60):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    want = [c for c in ("grid_size_x", "grid_x", "workgroup_size_x", "group_segment_size", "lds_size")
            if c in cols]
    q = "select name, start, end" + "".join(", " + c for c in want) + " from kernels order by start"
    rows = [r for r in con.execute(q) if sub in r[0]]
    print("columns:", ["name", "us"] + want)
    for r in rows[-int(last):]:
        print(f"{r[0].split('(')[0][:48]:48s} {(r[2] - r[1]) / 1e3:10.1f} " + " ".join(str(x) for x in r[3:]))


if __name__ == "__main__":
    main(*sys.argv[1:])
