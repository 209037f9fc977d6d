#!/usr/bin/env python3
"""PlonK BLS12-381 prove timing (gnark_amd.plonk_prover) with per-stage times.
usage: bench_plonk.py log_n [reps] [projection, e.g. 8 or 2,4,8]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def heartbeat(every=20.0):
    """a line on stderr every `every` s (a silent GPU run is taken to be hung)"""
    import threading
    import time
    t0 = time.time()

    def beat():
        while True:
            time.sleep(every)
            print(f"[bench_plonk] alive {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    proj = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else ()
    r = bench.plonk_prove_bench(L, reps=reps, per_rep=True, projection=proj)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
