"""Where one shard of the N-way Groth16 split spends its proof (BASELINE
configs[3] on N GPUs), on one GPU: the 2^log_n MiMC-shaped key split over N
shards that all live on device 0, shard `solo` rehearsed alone
(gg_groth16_mpk_set_rehearsal: the others skip their work), so a kernel trace
(rocprofv3 --kernel-trace) shows one GPU's share; tools/part_breakdown.py reads
the last proof.
usage: g16_shard_probe.py [log_n] [shards] [solo] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))


def main():
    import bench
    from gnark_amd import backend, groth16
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    shards = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    solo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    g = bench.Groth16Bench(log_n, 0, 1, None, None, host_inputs=False)
    sol = groth16.Solution(*g.host, g.shape["nw"], g.shape["ncons"])
    g.close()
    mpk = groth16.MultiGpuProvingKey(g.data, [0] * shards)
    mpk.set_rehearsal(solo)
    sd = groth16.replicate_solution(sol, [0] * shards)
    opt = backend.with_amd_acceleration()
    import gc
    gc.collect()  # the setup's garbage: not inside a timed proof
    gc.freeze()
    ts = []
    for _ in range(reps):
        # an idle gap the breakdown uses to find the last proof (PROBE_SLEEP=0 for
        # timing: the GPU clocks down in the gap, +1.3 ms on the next proof)
        time.sleep(float(os.environ.get("PROBE_SLEEP", "0.05")))
        a = time.perf_counter()
        mpk.prove(sd, opt, r=g.r, s=g.s, rehearsal_ok=True)
        ts.append(1e3 * (time.perf_counter() - a))
    st = mpk.shard_timings()[solo]
    print(json.dumps({"log_n": log_n, "shards": shards, "solo": solo, "prove_ms": ts, "shard": st,
                      "windows": [mpk.base_info(w, solo)[1:] for w in range(5)]}), flush=True)
    mpk.close()


if __name__ == "__main__":
    main()
