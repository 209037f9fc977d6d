"""Per-kernel averages of arbitrary rocprofv3 --pmc counters (rocpd sqlite),
plus derived VALU figures when the SQ counters are present.
usage: pmc_counters.py out.json [--workload JSON] db1 [db2 ...]   (one db per --pmc pass)
The output carries csrc_sha16, the digest of the kernel tree measured (bench.py
only uses profiles of its own tree).
SQ_* cycle counters count quad-cycles on gfx950 (MI355X_MICROARCH.md, PMC units):
  valu_busy = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (fraction of resident-wave
  time a VALU instruction issues), insts_per_wave = SQ_INSTS_VALU / SQ_WAVES."""
import json
import os
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest  # noqa: E402


def collect(db):
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, dispatch_id, counter_name, sum(value) from counters_collection "
                       "group by dispatch_id, counter_name").fetchall()
    acc = defaultdict(lambda: defaultdict(list))
    for name, _, cn, v in rows:
        acc[name.split("(")[0]][cn].append(v)
    return acc


def main(out, dbs, workload=None):
    res = defaultdict(dict)
    for db in dbs:
        for k, cs in collect(db).items():
            for cn, vs in cs.items():
                res[k][cn] = sum(vs) / len(vs)
                res[k]["dispatches"] = max(res[k].get("dispatches", 0), len(vs))
    for k, c in res.items():
        if c.get("SQ_WAVE_CYCLES") and "SQ_ACTIVE_INST_VALU" in c:
            c["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_WAVES") and "SQ_INSTS_VALU" in c:
            c["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        if c.get("SQ_BUSY_CYCLES") and "SQ_ACTIVE_INST_VALU" in c:
            c["valu_per_busy"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_BUSY_CYCLES"]
    json.dump({"source": dbs, "unit": "counter value per dispatch (average)", "csrc_sha16": csrc_digest(),
               "workload": json.loads(workload) if workload else {}, "kernels": res},
              open(out, "w"), indent=1)
    for k, c in sorted(res.items()):
        print(k[:70], json.dumps({a: round(b, 4) if isinstance(b, float) else b for a, b in c.items()}))


if __name__ == "__main__":
    a = sys.argv[2:]
    wl = None
    if a and a[0] == "--workload":
        wl, a = a[1], a[2:]
    main(sys.argv[1], a, wl)
