"""MSM bases built from points already in HBM (gg_msm_base_create with
points_on_device = 1): infinity points are dropped on the device (flag / scan /
scatter, no round trip through host memory) and the MSM equals the one over
the same points uploaded from the host, for G1 / G2 (BN254) and BLS12-381 G1,
with and without infinity holes (prove.go:201-290 MultiExp semantics: an
infinity point contributes nothing)."""
import pytest

from helpers import random_fr_mont

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("group_name,n,inf_every", [("G1", 5000, 0), ("G1", 70000, 7), ("G2", 3000, 5),
                                                    ("BLS12_381_G1", 4000, 3)])
def test_device_base_matches_host_base(group_name, n, inf_every):
    from gnark_amd import DeviceBuffer, msm
    group = getattr(msm, group_name)
    aff = msm._AFF[group]
    import bench
    if group == msm.G1:
        g = bench.g1_generator_mont()
    elif group == msm.G2:
        g = bench.g2_generator_mont()
    else:
        import bls12_381_oracle as bo
        g = bo.g1_to_bytes(bo.G1_GEN)
    pts = bytearray(msm.batch_scalar_mul(group, g, random_fr_mont(n, seed=n).tobytes(), n))
    if inf_every:
        for i in range(0, n, inf_every):
            pts[aff * i:aff * (i + 1)] = bytes(aff)
    pts = bytes(pts)
    scal = random_fr_mont(n, seed=n + 1).tobytes()
    host = msm.MsmBase(group, pts, n)
    dev_pts = DeviceBuffer.from_host(pts)
    dev = msm.MsmBase(group, dev_pts, n, on_device=True)
    assert dev.info() == host.info()
    assert dev.msm(scal, n) == host.msm(scal, n)
    host.close()
    dev.close()
