"""PlonK BLS12-381 row a21 kernels on the GPU through the C ABI, bit-exact
against oracle/bls12_381_oracle.py: the copy-constraint ratio Z
(iop.BuildRatioCopyConstraint, prove.go:610-621), the running product behind
it, Horner evaluation and the KZG opening quotient (kzg.Open, prove.go:646,
823-830), foldH (prove.go:670-705) and computeLinearizedPolynomial
(prove.go:1289-1389).  Large sizes (several scan levels) are checked through
size-independent properties on sampled indices."""
import random

import numpy as np
import pytest

import bls12_381_oracle as bo
from test_oracle_bls import _copy_witness

pytestmark = pytest.mark.gpu


def dev(v):
    from gnark_amd import DeviceBuffer
    return DeviceBuffer.from_host(bo.fr_vec_to_bytes(v))


def host(buf, k=None):
    return bo.fr_vec_from_bytes(buf.to_host(None if k is None else 32 * k))


def rand_vec(n, seed):
    rnd = random.Random(seed)
    return [rnd.randrange(bo.R) for _ in range(n)]


def rand_mont_bytes(n, seed):
    """n uniform fr < 2^254 (Montgomery bytes = the integer's image, any value < r is valid)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    a[:, 3] &= np.uint64((1 << 60) - 1)
    return a.tobytes()


@pytest.mark.parametrize("n", [2, 4, 16, 256, 2048, 4096])
def test_ratio_copy_constraint_vs_oracle(n):
    from gnark_amd import plonk, fr, DeviceBuffer
    dom = bo.Domain(n)
    perm, f = _copy_witness(n, 10 + n)
    beta, gamma = rand_vec(2, n)
    exp = bo.ratio_copy_constraint(f, perm, beta, gamma, dom)
    z = DeviceBuffer(32 * n)
    pd = DeviceBuffer.from_host(np.asarray(perm, dtype=np.int64).tobytes())
    plonk.ratio_copy_constraint(dev(f[0]), dev(f[1]), dev(f[2]), pd, n, bo.fr_to_bytes(beta),
                                bo.fr_to_bytes(gamma), bo.fr_to_bytes(dom.generator),
                                bo.fr_to_bytes(dom.gen), z)
    assert host(z) == exp
    # a random (unsatisfied) witness also matches the restatement
    g = [rand_vec(n, 77 + j) for j in range(3)]
    exp2 = bo.ratio_copy_constraint(g, perm, beta, gamma, dom)
    plonk.ratio_copy_constraint(dev(g[0]), dev(g[1]), dev(g[2]), pd, n, bo.fr_to_bytes(beta),
                                bo.fr_to_bytes(gamma), bo.fr_to_bytes(dom.generator),
                                bo.fr_to_bytes(dom.gen), z)
    assert host(z) == exp2


def test_ratio_copy_constraint_closes_2p20():
    """Size-independent property at 2^20: Z[0] = 1 and, for a satisfied
    permutation, Z[n-1] * num_(n-1) / den_(n-1) = 1; sampled Z[i+1]/Z[i] equal
    the i-th ratio."""
    from gnark_amd import plonk, DeviceBuffer
    n = 1 << 20
    dom = bo.Domain(n)
    perm, f = _copy_witness(n, 99)
    beta, gamma = rand_vec(2, 5)
    z = DeviceBuffer(32 * n)
    pd = DeviceBuffer.from_host(np.asarray(perm, dtype=np.int64).tobytes())
    plonk.ratio_copy_constraint(dev(f[0]), dev(f[1]), dev(f[2]), pd, n, bo.fr_to_bytes(beta),
                                bo.fr_to_bytes(gamma), bo.fr_to_bytes(dom.generator),
                                bo.fr_to_bytes(dom.gen), z)
    zb = z.to_host()
    Z = lambda i: bo.fr_from_bytes(zb[32 * i:32 * i + 32])  # noqa: E731
    w, u = dom.generator, dom.gen

    def ratio(i):
        num = den = 1
        for j in range(3):
            idv = pow(u, j, bo.R) * pow(w, i, bo.R)
            s = perm[j * n + i]
            sg = pow(u, s // n, bo.R) * pow(w, s % n, bo.R)
            num = num * (f[j][i] + beta * idv + gamma) % bo.R
            den = den * (f[j][i] + beta * sg + gamma) % bo.R
        return num * pow(den, -1, bo.R) % bo.R

    assert Z(0) == 1
    assert Z(n - 1) * ratio(n - 1) % bo.R == 1
    rnd = random.Random(3)
    for i in [0, 2046, 2047, 2048, n - 2] + [rnd.randrange(n - 1) for _ in range(40)]:
        assert Z(i + 1) == Z(i) * ratio(i) % bo.R, i


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 2047, 2048, 2049, 5000, 4096 * 2048 + 3])
def test_prefix_product(n):
    from gnark_amd import plonk, DeviceBuffer
    data = rand_mont_bytes(n, n)
    buf = DeviceBuffer.from_host(data)
    plonk.prefix_product(buf, n)
    out = buf.to_host()
    x = lambda i: bo.fr_from_bytes(data[32 * i:32 * i + 32])  # noqa: E731
    y = lambda i: bo.fr_from_bytes(out[32 * i:32 * i + 32])  # noqa: E731
    if n <= 5000:
        acc = 1
        for i in range(n):
            acc = acc * x(i) % bo.R
            assert y(i) == acc, i
    else:  # three scan levels: sampled y[i] = y[i-1] x[i], incl. block and level edges
        rnd = random.Random(1)
        assert y(0) == x(0)
        for i in [1, 2047, 2048, 2049, 4096 * 2048 - 1, 4096 * 2048, n - 1] + \
                [rnd.randrange(1, n) for _ in range(60)]:
            assert y(i) == y(i - 1) * x(i) % bo.R, i


@pytest.mark.parametrize("n", [1, 2, 3, 8, 100, 2048, 2049, 6000])
def test_horner_and_kzg_quotient_vs_oracle(n):
    from gnark_amd import plonk, DeviceBuffer
    f = rand_vec(n, 200 + n)
    a = rand_vec(1, n)[0]
    q = DeviceBuffer(32 * max(n - 1, 1))
    val = plonk.evaluate(dev(f), n, bo.fr_to_bytes(a), q_out=q)
    fa = bo.evaluate(f, a)
    assert bo.fr_from_bytes(val) == fa
    if n > 1:
        assert host(q, n - 1) == bo.divide_by_x_minus_a(f, fa, a)


@pytest.mark.parametrize("lens", [[1], [3, 1, 2], [100, 0, 2049], [300000, 262144, 262145, 7, 262143]])
def test_evaluate_many_vs_oracle(lens):
    """gg_fr_evaluate_many (the batched evaluations at zeta of prove.go:640-660 and
    the batch opening's claimed values): every f_k(a) equals Horner's (oracle),
    lengths around the 2^18-lane grid edge, an empty polynomial gives 0."""
    from gnark_amd import plonk, DeviceBuffer
    fs = [rand_vec(n, 500 + i + n) for i, n in enumerate(lens)]
    a = rand_vec(1, sum(lens))[0]
    bufs = [dev(f) if f else DeviceBuffer(32) for f in fs]
    got = plonk.evaluate_many(bufs, lens, bo.fr_to_bytes(a))
    assert [bo.fr_from_bytes(g) for g in got] == [bo.evaluate(f, a) if f else 0 for f in fs]


def test_evaluate_many_bn254_and_2p22():
    """BN254 fr (backend/plonk/bn254) against a Python Horner, and at 2^22 + 3
    the batched value equals the scan-based evaluation (gg_bls12_381_fr_horner)."""
    from gnark_amd import plonk, DeviceBuffer
    from gnark_amd._lib import GG_CURVE_BN254
    import bn254_oracle as o
    rnd = random.Random(12)
    f = [rnd.randrange(o.R) for _ in range(5000)]
    a = rnd.randrange(o.R)
    d = DeviceBuffer.from_host(b"".join(o.fr_to_bytes(x) for x in f))
    got = plonk.evaluate_many([d], [5000], o.fr_to_bytes(a), curve=GG_CURVE_BN254)[0]
    acc = 0
    for c in reversed(f):
        acc = (acc * a + c) % o.R
    assert o.fr_from_bytes(got) == acc
    n = (1 << 22) + 3
    big = DeviceBuffer.from_host(rand_mont_bytes(n, 8))
    x = rand_vec(1, 10)[0]
    v = plonk.evaluate_many([big, big], [n, n - 3], bo.fr_to_bytes(x))
    assert v[0] == plonk.evaluate(big, n, bo.fr_to_bytes(x))
    assert v[1] == plonk.evaluate(big, n - 3, bo.fr_to_bytes(x))


def test_horner_quotient_property_2p22():
    """At 2^22 + 3 (three scan levels): q(x)(x - a) + f(a) = f(x) at a random x."""
    from gnark_amd import plonk, DeviceBuffer
    n = (1 << 22) + 3
    f = DeviceBuffer.from_host(rand_mont_bytes(n, 8))
    a, x = rand_vec(2, 9)
    q = DeviceBuffer(32 * (n - 1))
    fa = bo.fr_from_bytes(plonk.evaluate(f, n, bo.fr_to_bytes(a), q_out=q))
    fx = bo.fr_from_bytes(plonk.evaluate(f, n, bo.fr_to_bytes(x)))
    qx = bo.fr_from_bytes(plonk.evaluate(q, n - 1, bo.fr_to_bytes(x)))
    assert (qx * (x - a) + fa - fx) % bo.R == 0
    # evaluation at 1 is the plain sum of the coefficients
    data = f.to_host()
    s = sum(int.from_bytes(data[i:i + 32], "little") for i in range(0, len(data), 32))
    s = s * pow(bo.FR_MONT, -1, bo.R) % bo.R
    assert bo.fr_from_bytes(plonk.evaluate(f, n, bo.fr_to_bytes(1))) == s


@pytest.mark.parametrize("n", [4, 64, 4096])
def test_fold_h_vs_oracle(n):
    from gnark_amd import plonk, DeviceBuffer
    h = rand_vec(3 * (n + 2), n)
    zeta = rand_vec(1, n + 1)[0]
    out = DeviceBuffer(32 * (n + 2))
    plonk.fold_h(dev(h), n, bo.fr_to_bytes(pow(zeta, n + 2, bo.R)), out)
    assert host(out) == bo.fold_h(h, n, zeta)


@pytest.mark.parametrize("n,ncmt", [(8, 0), (64, 1), (1024, 2)])
def test_linearized_vs_oracle(n, ncmt):
    from gnark_amd import plonk
    rnd = random.Random(n + ncmt)
    nz = n + 3  # blinded Z has n + deg(Bz) + 1 coefficients
    bz = rand_vec(nz, 1)
    s3 = rand_vec(n, 2)
    qs = [rand_vec(n, 3 + k) for k in range(5)]
    pi2 = [rand_vec(n, 10 + j) for j in range(ncmt)]
    qcp = rand_vec(ncmt, 20)
    l, r, o, alpha, beta, gamma, zeta, zu, s1z, s2z = (rnd.randrange(bo.R) for _ in range(10))
    sc = plonk.linearized_scalars(l, r, o, alpha, beta, gamma, zeta, zu, s1z, s2z, bo.FR_GEN, n)
    zb = dev(bz)
    plonk.linearized(zb, nz, dev(s3), n, [dev(q) for q in qs], n, sc,
                     pi2=[dev(p) for p in pi2], qcp_zeta=qcp)
    exp = bo.linearized(bz, s3, qs[0], qs[1], qs[2], qs[3], qs[4], pi2, qcp, sc[0], sc[1], sc[2],
                        sc[3], sc[4], sc[6], sc[7])
    assert host(zb) == exp


def test_undersized_buffers_refused_before_launch():
    from gnark_amd import plonk, DeviceBuffer
    n = 64
    h = DeviceBuffer(3 * (n + 2) * 32)
    with pytest.raises(ValueError):
        plonk.fold_h(h, n, bo.fr_to_bytes(3), DeviceBuffer(32 * n))
    with pytest.raises(ValueError):
        plonk.evaluate(DeviceBuffer(32 * (n - 1)), n, bo.fr_to_bytes(3))
