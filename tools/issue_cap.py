"""VALU issue costs in the chip's real cycles: the
tools/mbench_field k_mad_tp kernels -- 16 independent v_mad_u64_u32 per
iteration (mix 0), plus 32 simple 32-bit VALU ops interleaved (mix 1) -- under
rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace.
SIMD-cycles per wave-iteration = (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) /
(SQ_WAVES x iterations); the mix-1 minus mix-0 difference prices a simple op,
the rest of mix 0 a mad.  bench.py's roofline.valu divides the accumulation's
issue rate, counted the same way, by the ceiling of its mix from these costs.
usage: issue_cap.py run_results.db out.json"""
import json
import os
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest  # noqa: E402

ITERS = 2048  # the timed launches (the warm-ups run 4)
MADS = 16


def main(db, out):
    con = sqlite3.connect(db)
    per = defaultdict(dict)
    for did, name, cn, v in con.execute("select dispatch_id, kernel_name, counter_name, sum(value) from "
                                        "counters_collection group by dispatch_id, counter_name"):
        per[did][cn] = v
        per[did]["name"] = name
    dur = {}
    for did, s, e in con.execute("select dispatch_id, start, end from kernels"):
        dur[did] = (e - s) * 1e-9
    res = {}
    for mix in (0, 1):
        rows = [(did, c) for did, c in per.items() if f"k_mad_tp<{mix}>" in c["name"]]
        big = max(c["SQ_INSTS_VALU"] for _, c in rows)
        rows = [(did, c) for did, c in rows if c["SQ_INSTS_VALU"] > 0.5 * big]  # the 2048-iteration launches
        acc = defaultdict(list)
        for did, c in rows:
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            wi = c["SQ_WAVES"] * ITERS
            acc["simd_cycles_per_wave_iter"].append(cyc * 1024 / wi)
            acc["insts_per_wave_iter"].append(c["SQ_INSTS_VALU"] / wi)
            acc["insts_per_simd_cycle"].append(c["SQ_INSTS_VALU"] / (cyc * 1024))
            if did in dur:
                acc["clock_GHz"].append(cyc / dur[did] / 1e9)
        res[f"mix{mix}"] = {k: sum(v) / len(v) for k, v in acc.items()}
        res[f"mix{mix}"]["dispatches"] = len(rows)
    m0, m1 = res["mix0"], res["mix1"]
    cs = (m1["simd_cycles_per_wave_iter"] - m0["simd_cycles_per_wave_iter"]) / (
        m1["insts_per_wave_iter"] - m0["insts_per_wave_iter"])
    cm = (m0["simd_cycles_per_wave_iter"] - (m0["insts_per_wave_iter"] - MADS) * cs) / MADS
    d = {"source": db, "csrc_sha16": csrc_digest(), "kernels": res, "cycles_per_mad": cm, "cycles_per_simple": cs,
         "note": "SIMD-cycles per wave-instruction at the chip's counted clock; the ceiling of a mix with a "
                 "fraction f of mads is 1 / (f x cycles_per_mad + (1 - f) x cycles_per_simple)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps({"cycles_per_mad": cm, "cycles_per_simple": cs,
                      "cap_57pct_mad": 1 / (0.57 * cm + 0.43 * cs),
                      "clock_GHz": [m0.get("clock_GHz"), m1.get("clock_GHz")]}))


if __name__ == "__main__":
    main(*sys.argv[1:3])
