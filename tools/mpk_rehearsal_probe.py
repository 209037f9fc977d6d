"""Step-by-step replay of tests/test_gpu_groth16_multi.py::test_mpk_rehearsal_mode
with a line per step (a stall shows where it sits; the library's waits are
bounded by GG_WAIT_TIMEOUT_S, so a stalled wait ends in GG_ERR_TIMEOUT naming it).
usage: mpk_rehearsal_probe.py [shards] [solo ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gnark-fork_amd")):
    sys.path.insert(0, p)
T0 = time.time()


def log(*a):
    print(f"[{time.time() - T0:7.2f}s]", *a, flush=True)


def main():
    import threading
    shards = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    solos = [int(x) for x in sys.argv[2:]] or [1]

    def beat():
        while True:
            time.sleep(15)
            log("alive")
    threading.Thread(target=beat, daemon=True).start()
    from gnark_amd import backend, groth16, GnarkAmdError
    from gnark_amd._lib import lib
    from test_gpu_groth16 import synthetic_case
    log("wait timeout", lib.gg_get_wait_timeout(), "task queues", os.environ.get("GG_TASK_QUEUES", "8"))
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(12, 3000, 3, 77, k_inf_every=5)
    data = groth16.ProvingKeyData(**d)
    sol = groth16.Solution(wires, sa, sb, sc, 3000, ncons)
    mpk = groth16.MultiGpuProvingKey(data, [0] * shards)
    log("key")
    opt = backend.with_amd_acceleration()
    ref = mpk.prove(sol, opt, r=r, s=s)
    log("prove (all shards)")
    for solo in solos:
        mpk.set_rehearsal(solo)
        log("set_rehearsal", solo)
        try:
            mpk.prove(sol, opt, r=r, s=s)
        except GnarkAmdError as e:
            log("refused as expected:", e.code)
        mpk.prove(sol, opt, r=r, s=s, rehearsal_ok=True)
        log("rehearsal prove", solo)
    mpk.set_rehearsal(-1)
    log("set_rehearsal -1")
    got = mpk.prove(sol, opt, r=r, s=s)
    log("prove after rehearsal, identical:", got == ref)
    mpk.close()
    log("closed")


if __name__ == "__main__":
    main()
