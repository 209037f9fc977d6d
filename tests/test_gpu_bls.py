"""BLS12-381 hot ops of the PlonK prover on the GPU,
through the C ABI, bit-exact against oracle/bls12_381_oracle.py:
  * G1 MSM (KZG commitments, prove.go:336, 494, 769, 1165-1169, 1203-1213);
  * fixed-base batch scalar multiplication (key generation);
  * Fr FFT / FFTInverse in all DIF/DIT x coset variants (prove.go:995-1061, 1223-1276).
Point sets are P_i = k_i G with known k_i, so large MSMs are checked with the
trapdoor identity sum s_i P_i = (sum s_i k_i) G."""
import random

import pytest

import bls12_381_oracle as b

pytestmark = pytest.mark.gpu


def _points(n, seed, inf_every=0):
    """P_i = (k0 + i q) G by successive additions; returns (bytes, ks)."""
    rng = random.Random(seed)
    k0, q = rng.randrange(1, b.R), rng.randrange(1, b.R)
    p, Q = b.g1_mul(b.G1_GEN, k0), b.g1_mul(b.G1_GEN, q)
    out, ks = [], []
    for i in range(n):
        k = (k0 + i * q) % b.R
        if inf_every and i % inf_every == 3:
            out.append(b.g1_to_bytes(b.INF))
            ks.append(0)
        else:
            out.append(b.g1_to_bytes(p))
            ks.append(k)
        p = b.g1_add(p, Q)
    return b"".join(out), ks


def _scalars(n, seed, dist="uniform"):
    rng = random.Random(seed)
    if dist == "uniform":
        v = [rng.randrange(b.R) for _ in range(n)]
    elif dist == "small":
        v = [rng.randrange(4) for _ in range(n)]
    else:  # edge values
        v = [rng.choice([0, 1, 2, b.R - 1, b.R - 2, (b.R - 1) // 2, rng.randrange(b.R)]) for _ in range(n)]
    return v, b.fr_vec_to_bytes(v)


@pytest.mark.parametrize("n,dist,c,inf_every", [
    (1, "uniform", 0, 0), (7, "edge", 0, 0), (100, "uniform", 0, 5), (4096, "uniform", 0, 0),
    (4096, "small", 8, 0), (4096, "edge", 13, 0), (4096, "uniform", 17, 11), (1 << 16, "uniform", 0, 0),
])
def test_bls_msm_vs_oracle(n, dist, c, inf_every):
    from gnark_amd import msm
    pts, ks = _points(n, 100 + n, inf_every)
    sv, sb = _scalars(n, 200 + n, dist)
    base = msm.MsmBase(msm.BLS12_381_G1, pts, n, window_bits=c)
    got = base.msm(sb, n)
    assert got == b.g1_to_bytes(b.msm_g1_trapdoor(ks, sv))


def test_bls_msm_small_naive():
    """independent of the trapdoor: naive sum of scalar multiples"""
    from gnark_amd import msm
    pts, ks = _points(9, 7)
    pl = [b.g1_from_bytes(pts[i * 96:(i + 1) * 96]) for i in range(9)]
    sv, sb = _scalars(9, 8)
    got = msm.MsmBase(msm.BLS12_381_G1, pts, 9).msm(sb, 9)
    assert got == b.g1_to_bytes(b.msm_g1(pl, sv))


def test_bls_batch_scalar_mul():
    from gnark_amd import msm
    sv, sb = _scalars(64, 9, "edge")
    out = msm.batch_scalar_mul(msm.BLS12_381_G1, b.g1_to_bytes(b.G1_GEN), sb, 64)
    for i, s in enumerate(sv):
        assert out[i * 96:(i + 1) * 96] == b.g1_to_bytes(b.g1_mul(b.G1_GEN, s))


def _dom(log_n):
    from gnark_amd import fr, ntt
    w = fr.bls_domain_generator(log_n)
    d = ntt.Domain(log_n, fr.bls_fr_mont(w), fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN),
                   curve=ntt.GG_CURVE_BLS12_381)
    return d, b.Domain(1 << log_n, w)


@pytest.mark.parametrize("log_n", [0, 1, 2, 5, 10, 12])
@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("dec", ["DIF", "DIT"])
@pytest.mark.parametrize("coset", [False, True])
def test_bls_ntt_variants_vs_oracle(log_n, inverse, dec, coset):
    from gnark_amd import ntt, DeviceBuffer
    d, od = _dom(log_n)
    n = 1 << log_n
    rng = random.Random(log_n * 31 + inverse * 7 + (dec == "DIT") * 3 + coset)
    a = [rng.randrange(b.R) for _ in range(n)]
    buf = DeviceBuffer.from_host(b.fr_vec_to_bytes(a))
    gdec = ntt.DIF if dec == "DIF" else ntt.DIT
    if inverse:
        d.fft_inverse(buf, gdec, coset)
        exp = b.fft_inverse(od, list(a), dec, coset)
    else:
        d.fft(buf, gdec, coset)
        exp = b.fft(od, list(a), dec, coset)
    assert b.fr_vec_from_bytes(buf.to_host()) == exp


@pytest.mark.parametrize("log_n", [16, 20])
def test_bls_ntt_roundtrip_large(log_n):
    import numpy as np
    from gnark_amd import ntt, DeviceBuffer
    d, _ = _dom(log_n)
    rng = np.random.default_rng(log_n)
    raw = rng.integers(0, 2**63, size=(1 << log_n, 4), dtype=np.uint64)
    raw[:, 3] &= np.uint64((1 << 60) - 1)  # < r (Montgomery bytes of some canonical value)
    x = raw.tobytes()
    buf = DeviceBuffer.from_host(x)
    for coset in (False, True):
        d.fft(buf, ntt.DIF, coset)
        d.fft_inverse(buf, ntt.DIT, coset)
        assert buf.to_host() == x


# ---------------------------------------------------------------- PlonK quotient kernels
def _rand_fr(rng, k):
    return [rng.randrange(b.R) for _ in range(k)]


@pytest.mark.parametrize("log_n,rho,nb_bsb", [(0, 4, 0), (3, 4, 1), (10, 4, 2), (8, 2, 0)])
def test_plonk_numerator_coset(log_n, rho, nb_bsb):
    from gnark_amd import plonk, DeviceBuffer
    rng = random.Random(log_n * 7 + rho + nb_bsb)
    n = 1 << log_n
    nx = 15 + 2 * nb_bsb
    xs = [_rand_fr(rng, n) for _ in range(nx)]
    bco = [_rand_fr(rng, 2), _rand_fr(rng, 2), _rand_fr(rng, 2), _rand_fr(rng, 3)]
    w = pow(b.FR_GEN, (b.R - 1) >> log_n, b.R)
    tw0 = [pow(w, j, b.R) for j in range(n)]
    beta, gamma, alpha = _rand_fr(rng, 3)
    cs = b.FR_GEN
    xb = [DeviceBuffer.from_host(b.fr_vec_to_bytes(v)) for v in xs]
    twb = DeviceBuffer.from_host(b.fr_vec_to_bytes(tw0))
    cres = DeviceBuffer(rho * n * 32)
    exp = [0] * (rho * n)
    got = None
    for coset in range(rho):
        plonk.numerator_coset(xb, [[b.fr_to_bytes(c) for c in q] for q in bco], twb,
                              b.fr_to_bytes(beta), b.fr_to_bytes(gamma), b.fr_to_bytes(alpha),
                              b.fr_to_bytes(cs), n, rho, coset, cres)
        b.numerator_coset(xs, bco, tw0, beta, gamma, alpha, cs, n, rho, coset, exp)
    got = b.fr_vec_from_bytes(cres.to_host())
    assert got == exp


@pytest.mark.parametrize("log_n,rho", [(2, 4), (6, 4), (9, 2)])
def test_plonk_divide_by_xn_minus_one(log_n, rho):
    from gnark_amd import fr, ntt, plonk, DeviceBuffer
    rng = random.Random(log_n + 100 * rho)
    n = 1 << log_n
    lb = (n * rho).bit_length() - 1
    wb = fr.bls_domain_generator(lb)
    big = ntt.Domain(lb, fr.bls_fr_mont(wb), fr.bls_fr_mont(fr.BLS_FR_MULTIPLICATIVE_GEN),
                     curve=ntt.GG_CURVE_BLS12_381)
    a = _rand_fr(rng, n * rho)
    buf = DeviceBuffer.from_host(b.fr_vec_to_bytes(a))
    plonk.divide_by_xn_minus_one(big, n, buf)
    exp = b.divide_by_xn_minus_one(list(a), n, b.Domain(n * rho, wb))
    assert b.fr_vec_from_bytes(buf.to_host()) == exp


@pytest.mark.parametrize("n", [1, 5, 1000, 1 << 17])
def test_bls_batch_invert(n):
    from gnark_amd import plonk, DeviceBuffer
    rng = random.Random(n)
    a = [rng.randrange(b.R) if rng.random() > 0.05 else 0 for _ in range(n)]
    buf = DeviceBuffer.from_host(b.fr_vec_to_bytes(a))
    plonk.batch_invert(buf, n)
    got = b.fr_vec_from_bytes(buf.to_host())
    if n <= 1000:
        assert got == b.batch_invert(a)
    else:  # x * x^-1 == 1 (and zeros stay zero), checked on a sample
        for i in rng.sample(range(n), 2000):
            assert (a[i] * got[i] % b.R) == (1 if a[i] else 0)
