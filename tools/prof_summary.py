"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) as a
markdown table: kernel, calls, total ms, average us, percent."""
import sqlite3
import sys


def main(db, out=None, title="kernel stats"):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels").fetchall()
    lines = [f"# {title}", "", f"source: `{db}` (rocprofv3 --kernel-trace --stats; durations in us)", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0]
        lines.append(f"| `{short}` | {calls} | {tot / 1e3:.3f} | {avg:.1f} | {pct:.1f} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
