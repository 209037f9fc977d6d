"""Where the primary part of an N-part PlonK key spends a proof (configs[4]:
BLS12-381, 2^22, 8 x MI355X), on one GPU: the key is split over N device parts
that all live on device 0; each part is then rehearsed alone (the others skip
their work), so a kernel trace (rocprofv3 --kernel-trace) shows one part's work.
usage: plonk_part_probe.py [log_n] [parts] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))


def main():
    import json
    import random
    import numpy as np
    import bench
    from gnark_amd import fr, msm, plonk_prover as pp, DeviceBuffer
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    parts = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n = 1 << log_n

    def bls_dev(k, seed):
        a = bench.rand_scalars(k, seed)
        a[:, 3] &= np.uint64((1 << 60) - 1)
        return DeviceBuffer.from_host(np.ascontiguousarray(a).tobytes())
    gen = fr.bls_fp_mont(bench.BLS_G1_GEN[0]) + fr.bls_fp_mont(bench.BLS_G1_GEN[1])
    kzg = DeviceBuffer(96 * (n + 3))
    msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bls_dev(n + 3, 61), n + 3, scalars_on_device=True, out=kzg)
    lag = DeviceBuffer(96 * n)
    msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bls_dev(n, 62), n, scalars_on_device=True, out=lag)
    sel = [bls_dev(n, 70 + i) for i in range(8)]
    perm = np.random.default_rng(71).permutation(3 * n).astype(np.int64).tobytes()
    L, R_, O = (bls_dev(n, 80 + i) for i in range(3))
    devs = [0] * parts if parts > 1 else None
    pk = pp.ProvingKey(log_n, kzg, lag, *sel, perm, devices=devs)
    if parts > 1:
        pp.prove(pk, L, R_, O, rng=random.Random(1))
        print(json.dumps({"parts_real_proof": pk.part_timings()}), flush=True)
    # rehearse part 0 and the peers listed in PROBE_PARTS (default: every part)
    which = [int(x) for x in os.environ.get("PROBE_PARTS", ",".join(map(str, range(parts)))).split(",") if x]
    for part in which:
        if parts > 1:
            pk.set_rehearsal(True, part=part)
        for _ in range(reps):
            tim = {}
            t = time.perf_counter()
            pp.prove(pk, L, R_, O, rng=random.Random(1), timings=tim, rehearsal_ok=True)
            print(json.dumps({"part": part, "ms": 1e3 * (time.perf_counter() - t), "stage_ms": tim}), flush=True)
            time.sleep(0.03)  # an idle gap that marks proof boundaries in a kernel trace (tools/part_breakdown.py)
        if parts == 1:
            break
    pk.close()


if __name__ == "__main__":
    main()
