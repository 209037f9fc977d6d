"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE
--kernel-trace database (MI355X_MICROARCH.md 'DVFS give-back': effective clock
= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; within 3 % of the in-kernel
clock on dispatches of 10 ms or more).
usage: clock_probe.py run_results.db [kernel-substring ...] [--last K]"""
import sqlite3
import sys
from collections import defaultdict


def main(argv):
    last = 0
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    db, subs = argv[0], argv[1:]
    con = sqlite3.connect(db)
    cnt = {}
    for did, name, v in con.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                                    "where counter_name = 'GRBM_GUI_ACTIVE' group by dispatch_id"):
        cnt[did] = (name.split("(")[0], v)
    dur = {}
    try:
        for did, s, e in con.execute("select dispatch_id, start, end from kernels"):
            dur[did] = (e - s) * 1e-9
    except sqlite3.Error:
        pass
    per = defaultdict(list)
    for did in sorted(cnt):
        name, v = cnt[did]
        if subs and not any(x in name for x in subs):
            continue
        if did in dur and dur[did] > 0:
            per[name].append((dur[did], v / 8 / dur[did] / 1e9))
    for name, xs in per.items():
        if last:
            xs = xs[-last:]
        ms = sum(d for d, _ in xs) / len(xs) * 1e3
        ghz = sum(g for _, g in xs) / len(xs)
        print(f"{name}: dispatches {len(xs)}, avg {ms:.3f} ms, effective clock {ghz:.3f} GHz")


if __name__ == "__main__":
    main(sys.argv[1:])
