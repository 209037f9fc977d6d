"""Bucket stripes of one MSM (gg_msm_stripe): the 2^s stripes' Jacobian results
add up to the whole MSM.  This is the split the multi-GPU Groth16 key uses for
its A, B1, K and G2 MSMs (every GPU holds the whole table and
takes the buckets b = part mod 2^s).  Checked bit-exact against the C oracle
(G1, G2) or the trapdoor (BLS12-381) and against gg_msm, over both bucket
reduction paths (quad-cooperative trees below 2^18 buckets per stripe, the
radix segment sums above), precompute groups, heavy, empty and absent buckets."""
import random

import pytest

import bls12_381_oracle as bo
import coracle
from helpers import random_fr_mont, random_g1_points, random_g2_points

pytestmark = pytest.mark.gpu


def _sum_stripes(base, group, sc, n, slog):
    from gnark_amd import msm
    acc = None
    for part in range(1 << slog):
        j = base.msm_stripe_jac(sc, n, slog, part)
        acc = j if acc is None else msm.jac_add(group, acc, j)
    return msm.jac_to_affine(group, acc)


def _scalars(n, seed, dist):
    if dist == "skew":  # half the entries in one bucket per window (heavy-bucket trees)
        sc = random_fr_mont(n, seed)
        sc[: n // 2] = sc[0]
        return sc
    return random_fr_mont(n, seed, dist)


@pytest.mark.parametrize("n,dist,c,slog", [
    (4096, "uniform", 0, 1), (4096, "uniform", 0, 3), (4096, "witness", 0, 2),
    (4096, "small", 10, 3),        # 16-bit scalars: most stripes' high windows empty
    (4096, "uniform", 20, 1),      # 2^18 buckets per stripe: radix segment sums (L = 2)
    (1 << 16, "uniform", 22, 2),   # 2^19 per stripe (L = 4), the 2^24 key's window
    (1 << 16, "skew", 22, 3),      # 2^18 per stripe with heavy buckets
    (1 << 16, "witness", 21, 3),   # 2^17 per stripe: quad path, 0/1 witness
    (257, "uniform", 8, 4),        # more stripes than most buckets hold entries
])
def test_g1_stripes_vs_oracle(n, dist, c, slog):
    from gnark_amd import msm
    pts = random_g1_points(n, 300 + n + c)
    sc = _scalars(n, 400 + n + slog, dist)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=c)
    want = coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    assert base.msm(sc, n) == want
    assert _sum_stripes(base, msm.G1, sc, n, slog) == want
    base.close()


@pytest.mark.parametrize("groups,slog", [(2, 1), (4, 2), (2, 3)])
def test_g1_stripes_precompute_groups(groups, slog, monkeypatch):
    """precompute groups G > 1: the bucket id carries the group in its top bits
    (B = j 2^(c-1) + b); a stripe keeps b mod 2^s of every group"""
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_GROUPS", str(groups))
    n = 4096
    pts = random_g1_points(n, 510 + groups)
    sc = random_fr_mont(n, 520 + slog)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=16)
    assert base.layout()[0] == groups
    want = coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    assert _sum_stripes(base, msm.G1, sc, n, slog) == want
    base.close()


@pytest.mark.parametrize("n,c,slog,dist", [(2048, 0, 2, "uniform"), (4096, 20, 1, "uniform"),
                                           (4096, 19, 3, "witness")])
def test_g2_stripes_vs_oracle(n, c, slog, dist):
    from gnark_amd import msm
    pts = random_g2_points(n, 600 + n + c)
    sc = random_fr_mont(n, 700 + slog, dist)
    base = msm.MsmBase(msm.G2, pts, n, window_bits=c)
    want = coracle.msm_g2(pts.tobytes(), sc.tobytes(), n)
    assert _sum_stripes(base, msm.G2, sc, n, slog) == want
    base.close()


@pytest.mark.parametrize("n,c,slog", [(1024, 0, 2), (2048, 20, 1)])
def test_bls12_381_stripes_trapdoor(n, c, slog):
    from gnark_amd import msm
    from test_gpu_bls import _points
    pts, ks = _points(n, 900 + n)
    rng = random.Random(950 + n)
    sv = [rng.randrange(bo.R) for _ in range(n)]
    sb = bo.fr_vec_to_bytes(sv)
    base = msm.MsmBase(msm.BLS12_381_G1, pts, n, window_bits=c)
    want = bo.g1_to_bytes(bo.msm_g1_trapdoor(ks, sv))
    assert _sum_stripes(base, msm.BLS12_381_G1, sb, n, slog) == want
    base.close()


def test_stripe_arguments():
    from gnark_amd import GnarkAmdError, msm
    n = 256
    pts = random_g1_points(n, 11)
    sc = random_fr_mont(n, 12)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=6)
    with pytest.raises(GnarkAmdError):
        base.msm_stripe_jac(sc, n, 5, 0)  # stripe_log > window_bits - 2
    with pytest.raises(GnarkAmdError):
        base.msm_stripe_jac(sc, n, 2, 4)  # part >= 2^stripe_log
    # stripe 0 of 1 is the whole MSM
    assert msm.jac_to_affine(msm.G1, base.msm_stripe_jac(sc, n, 0, 0)) == base.msm(sc, n)
    base.close()
