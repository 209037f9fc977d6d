"""Per-kernel HBM traffic from two separate rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; MI355X_MICROARCH.md "HBM"): average bytes per dispatch for each
kernel.  FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB; on gfx950
FETCH_SIZE counts 1/2 of the bytes of wide coalesced reads (the guide's
correction: x2).  Other access widths are uncalibrated (noted in the output).
usage: pmc_traffic.py fetch.db write.db out.json [workload-json]
(workload-json: e.g. '{"workload": "groth16", "log_n": 24, "n_gpus": 1}', the key
bench.py matches a profile on)"""
import json
import os
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_digest  # noqa: E402  (the kernel tree this profile measured)


def per_kernel(db, counter):
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, dispatch_id, sum(value) from counters_collection "
                       "where counter_name = ? group by dispatch_id", (counter,)).fetchall()
    acc = defaultdict(list)
    for name, _, v in rows:
        acc[name.split("(")[0]].append(v)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(fdb, wdb, out, workload=None):
    f = per_kernel(fdb, "FETCH_SIZE")
    w = per_kernel(wdb, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0.0, 0))
        wk = w.get(k, (0.0, 0))
        fetch_b = fk[0] * 1024.0
        write_b = wk[0] * 1024.0
        res[k] = {"dispatches": max(fk[1], wk[1]),
                  "fetch_bytes_raw": fetch_b, "fetch_bytes_x2": 2.0 * fetch_b,
                  "write_bytes": write_b, "traffic_bytes": 2.0 * fetch_b + write_b,
                  "traffic_bytes_raw": fetch_b + write_b}
    json.dump({"source": [fdb, wdb], "unit": "bytes per dispatch", "csrc_sha16": csrc_digest(),
               "workload": json.loads(workload) if workload else {},
               "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read undercount, measured for 16-B/lane "
                             "coalesced streams), WRITE_SIZE KiB x 1024; traffic_bytes_raw: no x2 (the "
                             "point gathers of the MSM accumulation are 64-B requests, outside the "
                             "calibrated case)",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda x: -x[1]["traffic_bytes"])[:15]:
        print(f"{k[:60]:60s} {v['dispatches']:5d} fetch {v['fetch_bytes_x2'] / 1e6:10.2f} MB write {v['write_bytes'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main(*sys.argv[1:5])
