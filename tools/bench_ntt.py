#!/usr/bin/env python3
"""Isolated NTT / computeH timing on one GPU (not the headline bench)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd"))
sys.path.insert(0, ROOT)
from bench import rand_scalars
from gnark_amd import _lib, ntt, DeviceBuffer


def timeit(fn, reps):
    fn()
    _lib.check(_lib.lib.gg_synchronize())
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    _lib.check(_lib.lib.gg_synchronize())
    return 1e3 * (time.perf_counter() - t) / reps


def main():
    out = {}
    for L in [int(x) for x in (sys.argv[1:] or ["20", "24"])]:
        n = 1 << L
        d = ntt.Domain(L)
        bufs = [DeviceBuffer.from_host(rand_scalars(n, 7 + i).tobytes()) for i in range(4)]
        reps = 20 if L <= 20 else 5
        r = {}
        r["fft_dif"] = timeit(lambda: d.fft(bufs[0], ntt.DIF), reps)
        r["fft_dit"] = timeit(lambda: d.fft(bufs[0], ntt.DIT), reps)
        r["ifft_dif_coset"] = timeit(lambda: d.fft_inverse(bufs[0], ntt.DIF, True), reps)
        _lib.profile_enable(True)
        r["compute_h"] = timeit(lambda: d.compute_h(bufs[0], bufs[1], bufs[2], n, bufs[3], inputs_on_device=True), reps)
        ms, cnt, _ = _lib.profile_get("ntt_pass")
        _lib.profile_enable(False)
        r["ntt_pass_avg_ms"] = ms / cnt if cnt else None
        r["ntt_pass_launches"] = cnt
        bfly = n // 2 * L
        r["G_butterfly_per_s_fft"] = bfly / (r["fft_dif"] * 1e-3) / 1e9
        out[L] = r
        print(L, json.dumps(r), flush=True)
        d.close()


if __name__ == "__main__":
    main()
