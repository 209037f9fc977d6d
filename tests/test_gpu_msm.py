"""GPU MSM parity (gg_msm) against the golden fixtures, the C oracle and the
trapdoor identity MSM(k_i G, s_i) = (sum s_i k_i) G."""
import numpy as np
import pytest

import bn254_oracle as o
import coracle
from helpers import b, golden, random_fr_mont, random_g1_points, random_g2_points

pytestmark = pytest.mark.gpu


def test_msm_golden():
    from gnark_amd import msm
    for c in golden()["msm"]:
        base = msm.MsmBase(c["group"], b(c["points"]), c["n"])
        got = base.msm(b(c["scalars"]), c["n"])
        assert got.hex() == c["expected"], (c["group"], c["n"])


@pytest.mark.parametrize("n,dist,c", [
    (1000, "uniform", 0), (1000, "witness", 0), (4096, "uniform", 4), (4096, "uniform", 8),
    (4096, "witness", 13), (1 << 16, "uniform", 0), (1 << 16, "witness", 0), (1 << 16, "small", 16),
    # balanced window widths: 24 windows of 10/11 bits, 13 of 19/20, 12 of 21/22
    (4096, "uniform", 11), (4096, "uniform", 20), (4096, "witness", 22),
])
def test_msm_g1_vs_oracle(n, dist, c):
    from gnark_amd import msm
    pts = random_g1_points(n, 1000 + n)
    sc = random_fr_mont(n, 2000 + n, dist)
    base = msm.MsmBase(msm.G1, pts, n, window_bits=c)
    assert base.msm(sc, n) == coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)


def test_msm_g1_2p20_config2():
    """BASELINE config 2: 2^20 random scalars/points, bit-exact vs the CPU oracle."""
    from gnark_amd import msm
    n = 1 << 20
    pts = random_g1_points(n, 4242)
    sc = random_fr_mont(n, 4343)
    base = msm.MsmBase(msm.G1, pts, n)
    exp = coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    assert base.msm(sc, n) == exp
    sw = random_fr_mont(n, 4444, "witness")
    assert base.msm(sw, n) == coracle.msm_g1(pts.tobytes(), sw.tobytes(), n)


def test_msm_trapdoor_2p18():
    from gnark_amd import msm
    n = 1 << 18
    ks = random_fr_mont(n, 77)
    ss = random_fr_mont(n, 78)
    pts = coracle.g1_batch_mul(o.g1_to_bytes(o.G1_GEN), ks.tobytes(), n)
    base = msm.MsmBase(msm.G1, bytes(pts), n)
    got = o.g1_from_bytes(base.msm(ss, n))
    kv = o.fr_vec_from_bytes(ks.tobytes())
    sv = o.fr_vec_from_bytes(ss.tobytes())
    assert got == o.g1_mul(o.G1_GEN, sum(x * y for x, y in zip(kv, sv)) % o.R)


def test_msm_edge_cases():
    from gnark_amd import msm
    n = 1 << 12
    p = o.g1_to_bytes(o.g1_mul(o.G1_GEN, 123456789))
    same = p * n  # DummySetup: every key point identical (setup.go:482-572)
    sc = random_fr_mont(n, 5)
    base = msm.MsmBase(msm.G1, same, n)
    tot = sum(o.fr_vec_from_bytes(sc.tobytes())) % o.R
    assert o.g1_from_bytes(base.msm(sc, n)) == o.g1_mul(o.g1_from_bytes(p), tot)
    # all-zero scalars -> infinity
    assert base.msm(np.zeros((n, 4), dtype=np.uint64), n) == bytes(64)
    # all scalars = 1 and = r-1 (max digit carries)
    one = np.frombuffer(o.fr_to_bytes(1) * n, dtype=np.uint64)
    rm1 = np.frombuffer(o.fr_to_bytes(o.R - 1) * n, dtype=np.uint64)
    pts = random_g1_points(n, 9)
    base2 = msm.MsmBase(msm.G1, pts, n)
    assert base2.msm(one, n) == coracle.msm_g1(pts.tobytes(), one.tobytes(), n)
    assert base2.msm(rm1, n) == coracle.msm_g1(pts.tobytes(), rm1.tobytes(), n)
    # infinity points inside the key are skipped (pk.G1.K, icicle.go:98-105)
    pts3 = pts.copy().reshape(n, 64)
    pts3[::7] = 0
    base3 = msm.MsmBase(msm.G1, pts3, n)
    assert base3.msm(sc, n) == coracle.msm_g1(pts3.tobytes(), sc.tobytes(), n)
    # P and -P with equal scalars cancel
    q = o.g1_mul(o.G1_GEN, 5)
    pq = o.g1_to_bytes(q) + o.g1_to_bytes((q[0], (-q[1]) % o.P))
    base4 = msm.MsmBase(msm.G1, pq, 2)
    s2 = o.fr_to_bytes(99) * 2
    assert base4.msm(s2, 2) == bytes(64)


@pytest.mark.parametrize("n,frac_one", [(1 << 16, 1.0), (1 << 18, 0.9)])
def test_msm_skewed_scalars(n, frac_one):
    """Real witnesses are 0/1-heavy: one bucket can hold most entries."""
    from gnark_amd import msm
    pts = random_g1_points(n, 70)
    sc = random_fr_mont(n, 71)
    one = np.frombuffer(o.fr_to_bytes(1), dtype=np.uint64)
    sel = np.random.default_rng(72).random(n) < frac_one
    sc[sel] = one
    base = msm.MsmBase(msm.G1, pts, n)
    assert base.msm(sc, n) == coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("n,c,dist", [(1 << 18, 20, "skew"), (1 << 18, 22, "witness"), (1 << 17, 19, "uniform")])
def test_msm_radix_bucket_reduction(n, c, dist, seg, monkeypatch):
    """Windows with >= 2^18 buckets take the radix-form level 2 + weighted sum
    (k_bucket_sum_r / k_bucket_runsum, the 2^24 proof's path); GG_MSM_SEGSUM=0
    the quad path: both bit-exact vs the C oracle, including heavy buckets
    (half of all scalars on one value: k_range_tree first) and empty ones."""
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_SEGSUM", seg)
    pts = random_g1_points(n, 80 + c)
    sc = random_fr_mont(n, 81 + c, "uniform" if dist == "skew" else dist)
    if dist == "skew":
        sc[: n // 2] = sc[0]
    base = msm.MsmBase(msm.G1, pts, n, window_bits=c)
    assert base.info()[1] == c
    assert base.msm(sc, n) == coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    base.close()


def test_msm_scalar_index_map():
    from gnark_amd import msm
    n, nw = 3000, 5000
    pts = random_g1_points(n, 31)
    w = random_fr_mont(nw, 32)
    idx = np.random.default_rng(3).choice(nw, size=n, replace=False).astype(np.uint32)
    base = msm.MsmBase(msm.G1, pts, n, scalar_index=idx)
    gathered = np.ascontiguousarray(w[idx])
    assert base.msm(w, nw) == coracle.msm_g1(pts.tobytes(), gathered.tobytes(), n)


def test_msm_device_scalars_and_jacobian_add():
    from gnark_amd import msm, DeviceBuffer
    n = 1 << 14
    pts = random_g1_points(n, 41)
    sc = random_fr_mont(n, 42)
    exp = coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
    # shard in two halves, combine partials (the multi-GPU reduction path)
    h = n // 2
    b0 = msm.MsmBase(msm.G1, pts[: h * 64], h)
    b1 = msm.MsmBase(msm.G1, pts[h * 64:], n - h)
    d0 = DeviceBuffer.from_host(sc[:h].tobytes())
    d1 = DeviceBuffer.from_host(sc[h:].tobytes())
    j0 = b0.msm_jac(d0, h, on_device=True)
    j1 = b1.msm_jac(d1, n - h, on_device=True)
    assert msm.jac_to_affine(msm.G1, msm.jac_add(msm.G1, j0, j1)) == exp


@pytest.mark.parametrize("n,dist", [(1000, "uniform"), (1 << 12, "witness"), (1 << 15, "uniform")])
def test_msm_g2_vs_oracle(n, dist):
    from gnark_amd import msm
    pts = random_g2_points(n, 500 + n)
    sc = random_fr_mont(n, 600 + n, dist)
    base = msm.MsmBase(msm.G2, pts, n)
    assert base.msm(sc, n) == coracle.msm_g2(pts.tobytes(), sc.tobytes(), n)


def _g2_trapdoor(ks, ss):
    e = coracle.fr_dot(ks, ss, len(ks))
    return bytes(coracle.g2_batch_mul(o.g2_to_bytes(o.G2_GEN), e, 1))


@pytest.mark.parametrize("n,dist", [(1 << 16, "uniform"), (1 << 18, "witness"), (1 << 16, "skew")])
def test_msm_g2_window20(n, dist):
    """The window choose_c picks for the 2^24 G2 base of config 4 (c = 20: 13
    windows, 2^19 Fp2 buckets, the Fp2 reduction arena), here forced on smaller
    bases; 'skew' puts half of all scalars on one value (one heavy bucket per
    window, the segmented heavy-bucket tree)."""
    from gnark_amd import msm
    ks = random_fr_mont(n, 700 + n)
    pts = coracle.g2_batch_mul(o.g2_to_bytes(o.G2_GEN), ks.tobytes(), n)
    if dist == "skew":
        ss = random_fr_mont(n, 800 + n)
        ss[: n // 2] = ss[0]
    else:
        ss = random_fr_mont(n, 800 + n, dist)
    base = msm.MsmBase(msm.G2, bytes(pts), n, window_bits=20)
    assert base.info()[1:] == (20, 13)
    assert base.msm(ss, n) == _g2_trapdoor(ks, ss)


@pytest.mark.parametrize("seg", ["1", "0"])
@pytest.mark.parametrize("n,c,dist", [(1 << 16, 20, "skew"), (1 << 17, 22, "witness"), (1 << 16, 19, "uniform")])
def test_msm_g2_radix_bucket_reduction(n, c, dist, seg, monkeypatch):
    """G2 windows with >= 2^18 buckets take the radix-form Fp2 level 2 and
    weighted sums (k_bucket_sum_r / k_bucket_runsum over Xyzz2_29, segments of
    L = 2 / 16 / 2 buckets here); GG_MSM_SEGSUM=0 the quad path.  Trapdoor-
    checked, with heavy buckets ('skew': k_range_tree_r first) and empty ones."""
    from gnark_amd import msm
    monkeypatch.setenv("GG_MSM_SEGSUM", seg)
    ks = random_fr_mont(n, 710 + c)
    pts = coracle.g2_batch_mul(o.g2_to_bytes(o.G2_GEN), ks.tobytes(), n)
    ss = random_fr_mont(n, 810 + c, "uniform" if dist == "skew" else dist)
    if dist == "skew":
        ss[: n // 2] = ss[0]
    base = msm.MsmBase(msm.G2, bytes(pts), n, window_bits=c)
    assert base.info()[1] == c
    assert base.msm(ss, n) == _g2_trapdoor(ks, ss)
    base.close()


def test_msm_g2_window20_2p20():
    """2^20 G2 points at c = 20, trapdoor-checked."""
    from gnark_amd import msm
    n = 1 << 20
    ks = random_fr_mont(n, 901)
    ss = random_fr_mont(n, 902, "witness")
    pts = msm.batch_scalar_mul(msm.G2, o.g2_to_bytes(o.G2_GEN), ks, n)
    base = msm.MsmBase(msm.G2, pts, n)
    assert base.info()[1] in (17, 18, 19, 20)
    assert base.msm(ss, n) == _g2_trapdoor(ks, ss)
    base20 = msm.MsmBase(msm.G2, pts, n, window_bits=20)
    assert base20.msm(ss, n) == _g2_trapdoor(ks, ss)
