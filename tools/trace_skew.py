import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-fork_amd")); sys.path.insert(0, ROOT)
import numpy as np
from bench import rand_scalars, g1_generator_mont
from gnark_amd import msm, DeviceBuffer, fr
n = 1 << 20
pts = DeviceBuffer(64 * n)
msm.batch_scalar_mul(msm.G1, g1_generator_mont(), rand_scalars(n, 1), n, out=pts)
base = msm.MsmBase(msm.G1, pts.ptr, n, on_device=True)
one = np.frombuffer(fr.fr_mont(1), dtype=np.uint64)
sc = rand_scalars(n, 2)
sc[np.random.default_rng(3).random(n) < 0.9] = one
d = DeviceBuffer.from_host(sc.tobytes())
for _ in range(3):
    base.msm_jac(d, n, on_device=True)
