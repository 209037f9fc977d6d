#!/usr/bin/env python3
"""Isolated G1 / G2 MSM timing (phase split from the HIP-event profiler).
usage: bench_msm.py G1|G2 log_n [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))
sys.path.insert(0, ROOT)
from bench import rand_scalars, g1_generator_mont, g2_generator_mont  # noqa: E402
import gnark_amd  # noqa: E402
from gnark_amd import _lib, msm, DeviceBuffer  # noqa: E402


def main():
    grp = msm.G1 if sys.argv[1].upper() == "G1" else msm.G2
    L = int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n = 1 << L
    pb = 64 if grp == msm.G1 else 128
    gen = g1_generator_mont() if grp == msm.G1 else g2_generator_mont()
    pts = DeviceBuffer(pb * n)
    msm.batch_scalar_mul(grp, gen, rand_scalars(n, 1), n, out=pts)
    base = msm.MsmBase(grp, pts.ptr, n, on_device=True)
    del pts
    npts, c, W = base.info()
    dsc = DeviceBuffer.from_host(rand_scalars(n, 2).tobytes())
    base.msm_jac(dsc, n, on_device=True)
    _lib.check(_lib.lib.gg_synchronize())
    t = time.perf_counter()
    for _ in range(reps):
        base.msm_jac(dsc, n, on_device=True)
    ms = 1e3 * (time.perf_counter() - t) / reps
    _lib.profile_enable(True)
    for _ in range(reps):
        base.msm_jac(dsc, n, on_device=True)
    ph = {}
    for name in ("msm_sort", "msm_accum", "msm_accum2", "msm_reduce"):
        tot, cnt, _ = _lib.profile_get(name)
        ph[name] = round(tot / cnt, 3) if cnt else None
    _lib.profile_enable(False)
    print(f"{sys.argv[1]} 2^{L} c={c} W={W} {ms:.3f} ms/msm {ph} {os.environ.get('TAG', '')}", flush=True)


if __name__ == "__main__":
    main()
