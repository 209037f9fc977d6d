"""FETCH_SIZE width calibration (MI355X_MICROARCH.md "HBM": calibrate other
access widths on a known byte count): reads one rocprofv3 --pmc FETCH_SIZE pass
over tools/mbench_gather_calib and that program's stdout (known bytes per
dispatch), writes factor[width] = known bytes / (FETCH_SIZE KiB x 1024).
usage: pmc_calib.py fetch.db calib_stdout.txt out.json"""
import json
import sqlite3
import sys


def main(db, log, out):
    known, table = {}, None
    for line in open(log):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            if "table_bytes" in d:
                table = d["table_bytes"]
                continue
            known[d["kernel"]] = d["known_bytes"]
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, dispatch_id, sum(value) from counters_collection "
                       "where counter_name = 'FETCH_SIZE' group by dispatch_id").fetchall()
    fetch = {}
    for name, _, v in rows:
        for k in known:
            if name.startswith(k.replace("k_gather<", "void k_gather<")) or name.split("(")[0].endswith(k):
                fetch[k] = v * 1024.0
    widths = {"k_stream16": 16, "k_gather<64>": 64, "k_gather<96>": 96, "k_gather<128>": 128}
    res = {"source": [db, log], "table_bytes": table, "known_bytes": known, "fetch_bytes_raw": fetch,
           "factor": {str(widths[k]): known[k] / fetch[k] for k in known if k in fetch and fetch[k] > 0},
           "note": "factor = known bytes read once (table >> the 256 MiB Infinity Cache) / FETCH_SIZE bytes; "
                   "gathers include the coalesced 4-B permutation reads"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["factor"]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
