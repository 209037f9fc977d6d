"""Times the G1 MSM at 2^20 on uniform vs witness-like vs 90%-ones scalars."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd")); sys.path.insert(0, ROOT)
import numpy as np
from bench import rand_scalars, g1_generator_mont
from gnark_amd import msm, DeviceBuffer, fr
n = 1 << int(os.environ.get("LOGN", "20"))
pts = DeviceBuffer(64 * n)
msm.batch_scalar_mul(msm.G1, g1_generator_mont(), rand_scalars(n, 1), n, out=pts)
base = msm.MsmBase(msm.G1, pts.ptr, n, on_device=True)
one = np.frombuffer(fr.fr_mont(1), dtype=np.uint64)
rng = np.random.default_rng(3)
out = {}
for name, frac0, frac1 in (("uniform", 0, 0), ("witness_50pct_01", 0.25, 0.25), ("ones_90pct", 0, 0.9)):
    sc = rand_scalars(n, 2)
    u = rng.random(n)
    sc[u < frac0] = 0
    sc[(u >= frac0) & (u < frac0 + frac1)] = one
    d = DeviceBuffer.from_host(sc.tobytes())
    for _ in range(2):
        base.msm_jac(d, n, on_device=True)
    t = time.perf_counter()
    for _ in range(10):
        base.msm_jac(d, n, on_device=True)
    out[name] = (time.perf_counter() - t) / 10 * 1e3
print(json.dumps({"msm_ms": out, "n": n, "window": base.info()}))
