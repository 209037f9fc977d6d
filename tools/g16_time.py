"""Groth16 prove time on one GPU (bench.py's headline key and inputs, solution
resident in HBM), for A/B runs of environment knobs without the rest of
bench.py: prints one JSON line with every proof's host-timed ms.
usage: g16_time.py [log_n] [reps] [warmup]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))


def main():
    import bench
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    g = bench.Groth16Bench(log_n, 0, 1, None, None, host_inputs=False)
    import gc
    gc.collect()  # the setup's garbage (GB-sized buffers): not inside a timed proof
    gc.freeze()
    for _ in range(warm):
        g.prove()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        g.prove()
        torch.cuda.synchronize()
        ts.append(round(1e3 * (time.perf_counter() - a), 3))
    env = {k: v for k, v in os.environ.items() if k.startswith("GG_")}
    print(json.dumps({"log_n": log_n, "env": env, "ms": ts, "min_ms": min(ts),
                      "median_ms": sorted(ts)[len(ts) // 2]}), flush=True)
    g.close()


if __name__ == "__main__":
    main()
