"""Same-base MSM batches (gg_msm_batch: PlonK's commitToLRO / commitToQuotient,
backend/plonk/bls12-381/prove.go:425-502, 1199-1218): 1..4 scalar vectors over
one resident base in one sort, one accumulation launch, one level 2 and one
bucket reduction.  Each result must equal the single MSM of its vector (and the
C oracle / the trapdoor identity), on every group, both bucket-reduction paths,
precompute groups, and batch sizes that leave empty bucket groups (3 -> 4)."""
import pytest

import coracle
from helpers import random_fr_mont, random_g1_points, random_g2_points

pytestmark = pytest.mark.gpu


def _vectors(n, k, seed, dists):
    return [random_fr_mont(n, seed + 17 * v, dists[v % len(dists)]) for v in range(k)]


def _affine(group, jacs):
    from gnark_amd import msm
    return [msm.jac_to_affine(group, j) for j in jacs]


@pytest.mark.parametrize("n,c,k,dists", [
    (1000, 0, 3, ["uniform"]),
    (4096, 13, 4, ["witness", "uniform"]),
    (4096, 11, 1, ["uniform"]),
    (1 << 15, 16, 2, ["witness", "uniform"]),
    (1 << 16, 20, 3, ["uniform", "witness", "small"]),  # 2^19 buckets per group: the radix segment path
])
def test_batch_g1_matches_single_and_oracle(n, c, k, dists):
    from gnark_amd import msm
    pts = random_g1_points(n, 500 + n + c)
    vecs = _vectors(n, k, 900 + n, dists)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=c)
    got = _affine(msm.G1, base.msm_batch_jac(vecs, n))
    for v in range(k):
        assert got[v] == base.msm(vecs[v], n)
        if n <= 4096:
            assert got[v] == coracle.msm_g1(pts.tobytes(), vecs[v].tobytes(), n)
    base.close()


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("groups", [2, 4])
def test_batch_g1_precompute_groups(groups, seg, monkeypatch):
    """G groups per base times a batch of 3 (4 copies of the bucket space): the
    weights 2^(j c) restart for every vector."""
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_GROUPS", str(groups))
    monkeypatch.setenv("GG_MSM_SEGSUM", seg)
    n = 1 << 14
    pts = random_g1_points(n, 777)
    vecs = _vectors(n, 3, 778, ["uniform", "witness"])
    base = msm.MsmBase(msm.G1, pts, n, window_bits=18)
    assert base.layout()[0] == groups
    got = _affine(msm.G1, base.msm_batch_jac(vecs, n))
    assert got == [base.msm(v, n) for v in vecs]
    base.close()


@pytest.mark.parametrize("n,c,k", [(1000, 0, 3), (1 << 14, 18, 2)])
def test_batch_g2_matches_single(n, c, k):
    from gnark_amd import msm
    pts = random_g2_points(n, 600 + n)
    vecs = _vectors(n, k, 610 + n, ["uniform", "witness"])
    base = msm.MsmBase(msm.G2, pts, n, window_bits=c)
    got = _affine(msm.G2, base.msm_batch_jac(vecs, n))
    assert got == [base.msm(v, n) for v in vecs]
    base.close()


@pytest.mark.parametrize("n,c,k", [(4096, 13, 3), (1 << 15, 20, 3)])
def test_batch_bls12_381_g1_trapdoor(n, c, k):
    """PlonK's KZG group: every result equals sum s_i k_i G."""
    import bls12_381_oracle as bl
    from gnark_amd import msm
    from test_gpu_bls import _points, _scalars
    pts, ks = _points(n, 71000 + n, 0)
    sv = [_scalars(n, 72000 + n + v, "uniform" if v % 2 == 0 else "edge") for v in range(k)]
    base = msm.MsmBase(msm.BLS12_381_G1, pts, n, window_bits=c)
    got = _affine(msm.BLS12_381_G1, base.msm_batch_jac([x[1] for x in sv], n))
    for v in range(k):
        assert got[v] == bl.g1_to_bytes(bl.msm_g1_trapdoor(ks, sv[v][0]))
    base.close()


def test_batch_bls12_381_g2_matches_single():
    from gnark_amd import msm
    from test_gpu_bls import _scalars
    import bls12_381_oracle as bl
    n = 300
    pts = b"".join(bl.g2_to_bytes(bl.g2_mul(bl.G2_GEN, 5 + 3 * i)) for i in range(n))
    vecs = [_scalars(n, 73000 + v)[1] for v in range(2)]
    base = msm.MsmBase(msm.BLS12_381_G2, pts, n)
    got = _affine(msm.BLS12_381_G2, base.msm_batch_jac(vecs, n))
    assert got == [base.msm(v, n) for v in vecs]
    base.close()


def test_batch_device_scalars_and_errors():
    from gnark_amd import DeviceBuffer, GnarkAmdError, msm
    n = 2048
    pts = random_g1_points(n, 881)
    vecs = _vectors(n, 4, 882, ["uniform"])
    base = msm.MsmBase(msm.G1, pts, n)
    dev = [DeviceBuffer.from_host(v.tobytes()) for v in vecs]
    got = base.msm_batch_jac(dev, n, on_device=True)
    assert _affine(msm.G1, got) == [base.msm(v, n) for v in vecs]
    with pytest.raises(GnarkAmdError):
        base.msm_batch_jac(vecs + vecs[:1], n)  # 5 vectors
    with pytest.raises(GnarkAmdError):
        base.msm_batch_jac(vecs[:2], n - 1)  # shorter than the base
    base.close()
