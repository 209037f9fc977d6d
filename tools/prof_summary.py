"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) as a
markdown table: kernel, calls, total ms, average us, percent, and (--last K)
the average over each kernel's last K dispatches -- the launches bench.py's
roofline pass times with HIP events.
usage: prof_summary.py run_results.db [out.md] [title] [--last K]"""
import sqlite3
import sys
from collections import defaultdict


def main(argv):
    last = 0
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    db = argv[0]
    out = argv[1] if len(argv) > 1 else None
    title = argv[2] if len(argv) > 2 else "kernel stats"
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels").fetchall()
    tail = {}
    if last:
        per = defaultdict(list)
        for name, start, end in con.execute("select name, start, end from kernels order by start"):
            per[name].append(end - start)
        tail = {k: sum(v[-last:]) / len(v[-last:]) for k, v in per.items()}
    lines = [f"# {title}", "", f"source: `{db}` (rocprofv3 --kernel-trace --stats; durations in us)", ""]
    if last:
        lines += [f"| kernel | calls | total ms | avg us | % | avg us, last {last} dispatches |",
                  "|---|---|---|---|---|---|"]
    else:
        lines += ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0]
        row = f"| `{short}` | {calls} | {tot / 1e3:.3f} | {avg:.1f} | {pct:.1f} |"
        if last:
            t = tail.get(name)
            row += f" {t / 1e3:.1f} |" if t is not None else " |"  # start/end: ns
        lines.append(row)
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
