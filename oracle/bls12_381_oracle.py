"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Pure-Python big-integer restatement of the BLS12-381 arithmetic on the PlonK
hot path of the reference (tumberger/gnark-fork, backend/plonk/bls12-381):
KZG commitments are G1 MSMs (prove.go:336, 494, 769, 1165-1169, 1203-1213) and
the quotient work is Fr FFTs on the small/big domains (prove.go:995-1061,
1223-1276).  Only ``tests/`` may import this module, as the *checker*; the
product path (``gnark-fork_amd``) never imports it.

Parity pins (tests/test_oracle_bls.py):
  * p, r: std/math/emulated/emparams/emparams.go:145-171 (hex and decimal);
  * curve y^2 = x^3 + 4 and the order-r subgroup: every compressed G1 point of
    the BLS12-381 verifying keys in backend/groth16/bellman_test.go:19-132
    decompresses onto the curve and satisfies r * P = O.
The arithmetic of gnark-crypto ecc/bls12-381 (go.mod:8, absent here) is
restated from its published algorithm: Montgomery form (R = 2^384 for fp,
2^256 for fr), little-endian u64 limbs; G1 affine {X, Y}, infinity = (0, 0).
The FFT root of unity (7^((r-1)/n), gnark-crypto's FrMultiplicativeGen = 7) has
no fixture in the reference: NTT values are "parity unpinned" and the device
API takes omega / the coset generator from pk.Domain.
"""
from __future__ import annotations

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
B = 4
FP_BYTES, FR_BYTES = 48, 32
FP_MONT, FR_MONT = 1 << 384, 1 << 256
FR_GEN = 7
FR_TWO_ADICITY = 32

# standard BLS12-381 G1 generator (validated by the pins: on curve, order r)
G1_GEN = (0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
          0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1)
INF = None


# ---------------------------------------------------------------- encodings
def fp_to_bytes(x: int) -> bytes:
    return (x % P * FP_MONT % P).to_bytes(FP_BYTES, "little")


def fp_from_bytes(b: bytes) -> int:
    return int.from_bytes(b, "little") * pow(FP_MONT, -1, P) % P


def fr_to_bytes(x: int) -> bytes:
    return (x % R * FR_MONT % R).to_bytes(FR_BYTES, "little")


def fr_from_bytes(b: bytes) -> int:
    return int.from_bytes(b, "little") * pow(FR_MONT, -1, R) % R


def fr_vec_to_bytes(v) -> bytes:
    return b"".join(fr_to_bytes(x) for x in v)


def fr_vec_from_bytes(b: bytes):
    return [fr_from_bytes(b[i:i + FR_BYTES]) for i in range(0, len(b), FR_BYTES)]


def g1_to_bytes(p) -> bytes:
    """gnark bls12381.G1Affine in memory; infinity = (0, 0)."""
    if p is INF:
        return bytes(2 * FP_BYTES)
    return fp_to_bytes(p[0]) + fp_to_bytes(p[1])


def g1_from_bytes(b: bytes):
    if b == bytes(2 * FP_BYTES):
        return INF
    return (fp_from_bytes(b[:FP_BYTES]), fp_from_bytes(b[FP_BYTES:]))


# ---------------------------------------------------------------- G1 (affine, exact)
def on_curve(p) -> bool:
    return p is INF or (p[1] * p[1] - p[0] ** 3 - B) % P == 0


def g1_add(p, q):
    if p is INF:
        return q
    if q is INF:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % P == 0:
            return INF
        lam = 3 * p[0] * p[0] * pow(2 * p[1], -1, P) % P
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], -1, P) % P
    x = (lam * lam - p[0] - q[0]) % P
    return (x, (lam * (p[0] - x) - p[1]) % P)


def g1_neg(p):
    return INF if p is INF else (p[0], (-p[1]) % P)


def g1_mul(p, k: int):
    k %= R
    acc, base = INF, p
    while k:
        if k & 1:
            acc = g1_add(acc, base)
        base = g1_add(base, base)
        k >>= 1
    return acc


def g1_mul_raw(p, k: int):
    """k * p without reducing k mod r (subgroup check)."""
    acc, base = INF, p
    while k:
        if k & 1:
            acc = g1_add(acc, base)
        base = g1_add(base, base)
        k >>= 1
    return acc


def msm_g1(points, scalars):
    """sum_i s_i P_i (naive; small n)."""
    acc = INF
    for p, s in zip(points, scalars):
        acc = g1_add(acc, g1_mul(p, s))
    return acc


def msm_g1_trapdoor(ks, scalars):
    """MSM over P_i = k_i G: (sum_i s_i k_i) G -- O(n) field work, any n."""
    t = 0
    for k, s in zip(ks, scalars):
        t = (t + k * s) % R
    return g1_mul(G1_GEN, t)


def g1_decompress_zcash(b: bytes):
    """Zcash/bellman compressed G1 (48 B big-endian; flags: 0x80 compressed,
    0x40 infinity, 0x20 y is the larger root)."""
    assert len(b) == 48 and b[0] & 0x80
    if b[0] & 0x40:
        return INF
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    y = pow((x ** 3 + B) % P, (P + 1) // 4, P)  # p = 3 mod 4
    if (y * y - x ** 3 - B) % P:
        raise ValueError("not on curve")
    if bool(b[0] & 0x20) != (y > P - y):
        y = P - y
    return (x, y)


# ---------------------------------------------------------------- Fp2 / G2 (exact, affine)
# Fp2 = Fp[u] / (u^2 + 1), elements (a0, a1); G2: y^2 = x^3 + 4 (1 + u) (the M-twist
# of gnark-crypto ecc/bls12-381), pinned by the compressed G2 points of
# backend/groth16/bellman_test.go (on the curve, order r).
B2 = (4, 4)
G2_GEN = ((0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
           0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
          (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
           0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE))


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2_inv(a):
    t = pow((a[0] * a[0] + a[1] * a[1]) % P, -1, P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_pow(a, e):
    r, b = (1, 0), a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_mul(b, b)
        e >>= 1
    return r


def f2_sqrt(a):
    """sqrt in Fp2 for p = 3 mod 4 (Adj-Rodriguez-Henriquez, algorithm 9); None if a is a non-square."""
    a1 = f2_pow(a, (P - 3) // 4)
    alpha = f2_mul(a1, f2_mul(a1, a))
    a0 = f2_mul((alpha[0], (-alpha[1]) % P), alpha)  # alpha^p * alpha
    if a0 == (P - 1, 0):
        return None
    x0 = f2_mul(a1, a)
    if alpha == (P - 1, 0):
        x = f2_mul((0, 1), x0)
    else:
        x = f2_mul(f2_pow(f2_add((1, 0), alpha), (P - 1) // 2), x0)
    return x if f2_mul(x, x) == (a[0] % P, a[1] % P) else None


def g2_on_curve(p) -> bool:
    if p is INF:
        return True
    x, y = p
    return f2_sub(f2_mul(y, y), f2_add(f2_mul(f2_mul(x, x), x), B2)) == (0, 0)


def g2_add(p, q):
    if p is INF:
        return q
    if q is INF:
        return p
    if p[0] == q[0]:
        if f2_add(p[1], q[1]) == (0, 0):
            return INF
        xx = f2_mul(p[0], p[0])
        lam = f2_mul(f2_add(f2_add(xx, xx), xx), f2_inv(f2_add(p[1], p[1])))
    else:
        lam = f2_mul(f2_sub(q[1], p[1]), f2_inv(f2_sub(q[0], p[0])))
    x = f2_sub(f2_sub(f2_mul(lam, lam), p[0]), q[0])
    return (x, f2_sub(f2_mul(lam, f2_sub(p[0], x)), p[1]))


def g2_mul(p, k: int, reduce=True):
    if reduce:
        k %= R
    acc, base = INF, p
    while k:
        if k & 1:
            acc = g2_add(acc, base)
        base = g2_add(base, base)
        k >>= 1
    return acc


def f2_lex_largest(y) -> bool:
    """E2.LexicographicallyLargest: compare A1 first, A0 if A1 = 0."""
    if y[1]:
        return y[1] > P - y[1]
    return y[0] > P - y[0]


def g2_decompress_zcash(b: bytes):
    """Zcash/bellman compressed G2 (96 B: X.A1 | X.A0 big-endian; flags on the first byte)."""
    assert len(b) == 96 and b[0] & 0x80
    if b[0] & 0x40:
        return INF
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_mul(x, x), x), B2))
    if y is None:
        raise ValueError("not on curve")
    if bool(b[0] & 0x20) != f2_lex_largest(y):
        y = ((-y[0]) % P, (-y[1]) % P)
    return (x, y)


def g2_compress(p) -> bytes:
    if p is INF:
        return bytes([0xC0]) + bytes(95)
    b = bytearray(p[0][1].to_bytes(48, "big") + p[0][0].to_bytes(48, "big"))
    b[0] |= 0xA0 if f2_lex_largest(p[1]) else 0x80
    return bytes(b)


def g2_to_bytes(p) -> bytes:
    """gnark bls12381.G2Affine in memory {X.A0, X.A1, Y.A0, Y.A1}; infinity = zeros."""
    if p is INF:
        return bytes(192)
    return b"".join(fp_to_bytes(v) for v in (p[0][0], p[0][1], p[1][0], p[1][1]))


def g2_from_bytes(b: bytes):
    if b == bytes(192):
        return INF
    v = [fp_from_bytes(b[i:i + 48]) for i in range(0, 192, 48)]
    return ((v[0], v[1]), (v[2], v[3]))


# ---------------------------------------------------------------- Groth16 over BLS12-381
def groth16_setup_scalars(constraints, nb_wires, nb_public, log_n, t, alpha, beta, delta):
    """Discrete logs of a backend/groth16/bls12-381 proving key (setup.go:85-337
    with given toxic waste): per-wire u_i(t), v_i(t), w_i(t) by the Lagrange
    recurrence of setup.go:352-434, then pk.G1.A/B (filtered), K, Z (bit-reversed,
    n - 1) and the infinity masks.  constraints: [(L, R, O)], each [(wire, coeff)]."""
    n = 1 << log_n
    w = pow(FR_GEN, (R - 1) >> log_n, R)
    A, B, C = [0] * nb_wires, [0] * nb_wires, [0] * nb_wires
    tv = []
    wi = 1
    for _ in range(len(constraints) + 1):
        tv.append((t - wi) % R)
        wi = wi * w % R
    L = (pow(t, n, R) - 1) * pow(tv[0], -1, R) % R * pow(n, -1, R) % R
    for j, (lc, rc, oc) in enumerate(constraints):
        for wid, k in lc:
            A[wid] = (A[wid] + k * L) % R
        for wid, k in rc:
            B[wid] = (B[wid] + k * L) % R
        for wid, k in oc:
            C[wid] = (C[wid] + k * L) % R
        L = L * w % R * tv[j] % R * pow(tv[j + 1], -1, R) % R
    dinv = pow(delta, -1, R)
    K = [(A[i] * beta + B[i] * alpha + C[i]) * dinv % R for i in range(nb_public, nb_wires)]
    zt = (pow(t, n, R) - 1) * dinv % R
    Z = [zt * pow(t, i, R) % R for i in range(n)]
    Z = [Z[bitrev(i, log_n)] for i in range(n)][: n - 1]
    return {"A": [a for a in A if a], "B": [b for b in B if b], "K": K, "Z": Z,
            "infA": [int(a == 0) for a in A], "infB": [int(b == 0) for b in B], "u": A, "v": B, "w": C}


def groth16_expected_scalars(constraints, wires, nb_public, log_n, ks, t, alpha, beta, delta, r, s):
    """Discrete logs (a, b, c) of the proof Ar, Bs, Krs of prove.go:63-322 for a
    satisfied instance: h(t) Z(t) = A(t) B(t) - C(t) with A(t) = sum_j A_j L_j(t)
    over the constraint rows -- no FFT needed."""
    n = 1 << log_n
    u, v, wv = ks["u"], ks["v"], ks["w"]
    a = (alpha + sum(x * y for x, y in zip(wires, u)) + r * delta) % R
    b = (beta + sum(x * y for x, y in zip(wires, v)) + s * delta) % R
    ct = sum(x * y for x, y in zip(wires, wv)) % R
    # A(t) B(t) - C(t) = a' b' - c' with a' = sum w_i u_i(t) etc. (u_i(t) already Lagrange-summed)
    at = sum(x * y for x, y in zip(wires, u)) % R
    bt = sum(x * y for x, y in zip(wires, v)) % R
    hz = (at * bt - ct) % R
    priv = sum(wires[i] * ((u[i] * beta + v[i] * alpha + wv[i]) % R) for i in range(nb_public, len(wires))) % R
    c = ((priv + hz) * pow(delta, -1, R) + s * a + r * b - r * s * delta) % R
    return a, b, c


# ---------------------------------------------------------------- FFT (gnark conventions)
def bitrev(i: int, logn: int) -> int:
    return int(format(i, f"0{logn}b")[::-1], 2) if logn else 0


class Domain:
    """gnark-crypto fft.NewDomain for bls12-381 fr (omega_n = 7^((r-1)/n); unpinned)."""

    def __init__(self, n: int, omega: int = None, gen: int = FR_GEN):
        assert n & (n - 1) == 0
        self.cardinality = n
        self.log_n = n.bit_length() - 1
        assert self.log_n <= FR_TWO_ADICITY
        self.generator = omega if omega is not None else pow(FR_GEN, (R - 1) >> self.log_n, R)
        self.generator_inv = pow(self.generator, -1, R)
        self.cardinality_inv = pow(n, -1, R)
        self.gen = gen
        self.gen_inv = pow(gen, -1, R)


def _dif(a, w):
    n = len(a)
    m = n >> 1
    while m >= 1:
        wm = pow(w, n // (2 * m), R)
        for start in range(0, n, 2 * m):
            t = 1
            for j in range(m):
                u, v = a[start + j], a[start + j + m]
                a[start + j] = (u + v) % R
                a[start + j + m] = (u - v) * t % R
                t = t * wm % R
        m >>= 1
    return a


def _dit(a, w):
    n = len(a)
    m = 1
    while m < n:
        wm = pow(w, n // (2 * m), R)
        for start in range(0, n, 2 * m):
            t = 1
            for j in range(m):
                u = a[start + j]
                v = a[start + j + m] * t % R
                a[start + j] = (u + v) % R
                a[start + j + m] = (u - v) % R
                t = t * wm % R
        m <<= 1
    return a


DIF, DIT = "DIF", "DIT"


def fft(dom: Domain, a, decimation, coset=False):
    """domain.FFT(a, decimation, [OnCoset()])."""
    n, logn = dom.cardinality, dom.log_n
    if coset:
        for i in range(n):
            e = bitrev(i, logn) if decimation == DIT else i
            a[i] = a[i] * pow(dom.gen, e, R) % R
    return _dif(a, dom.generator) if decimation == DIF else _dit(a, dom.generator)


def fft_inverse(dom: Domain, a, decimation, coset=False):
    """domain.FFTInverse(a, decimation, [OnCoset()])."""
    n, logn = dom.cardinality, dom.log_n
    if decimation == DIF:
        _dif(a, dom.generator_inv)
    else:
        _dit(a, dom.generator_inv)
    for i in range(n):
        x = a[i] * dom.cardinality_inv % R
        if coset:
            e = i if decimation == DIT else bitrev(i, logn)
            x = x * pow(dom.gen_inv, e, R) % R
        a[i] = x
    return a


def batch_invert(v):
    """fr.BatchInvert (prove.go:1273): zeros map to zero."""
    return [pow(x, -1, R) if x else 0 for x in v]


# ---------------------------------------------------------------- PlonK quotient path
# s.x ids (backend/plonk/bls12-381/prove.go:60-77)
ID_L, ID_R, ID_O, ID_Z, ID_ZS, ID_QL, ID_QR, ID_QM, ID_QO, ID_QK, ID_S1, ID_S2, ID_S3, \
    ID_ID, ID_LONE, ID_QCI = range(16)


def _horner(coeffs, x):
    r = 0
    for c in reversed(coeffs):
        r = (r * x + c) % R
    return r


def numerator_coset(x, bcoef, tw0, beta, gamma, alpha, cs, n, rho, coset, cres):
    """allConstraints (prove.go:912-934, with gateConstraint :852-868,
    orderingConstraint :874-892, ratioLocalConstraint :894-902) at every point j
    of one coset, scattered to cres[bitrev(rho*j + coset)] (prove.go:1030-1041)."""
    css = cs * cs % R
    nb_bsb = (len(x) - ID_QCI + 1) >> 1
    lb = (rho * n).bit_length() - 1
    for j in range(n):
        u = [p[j] for p in x]
        u[ID_S1] = u[ID_S1] * beta % R
        u[ID_S2] = u[ID_S2] * beta % R
        u[ID_S3] = u[ID_S3] * beta % R
        u[ID_L] = (u[ID_L] + _horner(bcoef[0], tw0[j])) % R
        u[ID_R] = (u[ID_R] + _horner(bcoef[1], tw0[j])) % R
        u[ID_O] = (u[ID_O] + _horner(bcoef[2], tw0[j])) % R
        u[ID_Z] = (u[ID_Z] + _horner(bcoef[3], tw0[j])) % R
        u[ID_ZS] = (u[ID_ZS] + _horner(bcoef[3], tw0[(j + 1) % n])) % R
        ic = (u[ID_QL] * u[ID_L] + u[ID_QR] * u[ID_R] + u[ID_QM] * u[ID_L] * u[ID_R]
              + u[ID_QO] * u[ID_O] + u[ID_QK]) % R
        for i in range(nb_bsb):
            ic = (ic + u[ID_QCI + 2 * i] * u[ID_QCI + 2 * i + 1]) % R
        a = (gamma + u[ID_L] + u[ID_ID]) % R
        b = (u[ID_ID] * cs + u[ID_R] + gamma) % R
        c = (u[ID_ID] * css + u[ID_O] + gamma) % R
        r = a * b * c * u[ID_Z] % R
        a = (u[ID_S1] + u[ID_L] + gamma) % R
        b = (u[ID_S2] + u[ID_R] + gamma) % R
        c = (u[ID_S3] + u[ID_O] + gamma) % R
        l = (a * b * c * u[ID_ZS] - r) % R
        rl = (u[ID_Z] - 1) * u[ID_LONE] % R
        res = ((rl * alpha + l) * alpha + ic) % R
        cres[bitrev(rho * j + coset, lb)] = res
    return cres


def xn_minus_one_inv_big_coset(n_small, big: Domain):
    """evaluateXnMinusOneDomainBigCoset (prove.go:1253-1276)."""
    rho = big.cardinality // n_small
    res = [pow(big.gen, n_small, R)]
    t = pow(big.generator, n_small, R)
    for _ in range(1, rho):
        res.append(res[-1] * t % R)
    return batch_invert([(v - 1) % R for v in res])


def divide_by_xn_minus_one(a, n_small, big: Domain):
    """divideByXMinusOne (prove.go:1223-1250): a is LagrangeCoset / BitReverse;
    result Canonical / Regular (FFTInverse DIT on the coset)."""
    f = xn_minus_one_inv_big_coset(n_small, big)
    rho = len(f)
    lb = big.log_n
    a = [v * f[bitrev(i, lb) % rho] % R for i, v in enumerate(a)]
    return fft_inverse(big, a, DIT, coset=True)


# ---------------------------------------------------------------- row a21
def support_permutation(n: int, dom: Domain):
    """getSupportPermutation (setup.go:391-407): <w> || u<w> || u^2<w>, u = FrMultiplicativeGen."""
    w, u = dom.generator, dom.gen
    res = []
    for blk in range(3):
        f = pow(u, blk, R)
        for i in range(n):
            res.append(f * pow(w, i, R) % R)
    return res


def ratio_copy_constraint(entries, perm, beta, gamma, dom: Domain):
    """iop.BuildRatioCopyConstraint (gnark-crypto [ext], called at prove.go:610-621),
    restated from its published algorithm with the reference's own permutation
    support (setup.go:391-407): Lagrange/Regular entries, result Lagrange/Regular."""
    n = dom.cardinality
    ids = support_permutation(n, dom)
    z = [1] * n
    num = [1] * n
    den = [1] * n
    for i in range(n - 1):
        b = d = 1
        for j, f in enumerate(entries):
            b = b * ((f[i] + beta * ids[j * n + i] + gamma) % R) % R
            d = d * ((f[i] + beta * ids[perm[j * n + i]] + gamma) % R) % R
        num[i + 1], den[i + 1] = b, d
    den = batch_invert(den)
    for i in range(1, n):
        z[i] = z[i - 1] * num[i] % R * den[i] % R
    return z


def evaluate(coeffs, x):
    """iop.Polynomial.Evaluate on canonical regular coefficients (Horner)."""
    return _horner(coeffs, x)


def divide_by_x_minus_a(f, fa, a):
    """kzg dividePolyByXminusA (gnark-crypto [ext], kzg.Open at prove.go:646,
    823-830): f - f(a) divided by X - a by synthetic division; returns n - 1 coefficients."""
    f = list(f)
    f[0] = (f[0] - fa) % R
    for i in range(len(f) - 2, -1, -1):
        f[i] = (f[i] + f[i + 1] * a) % R
    return f[1:]


def fold_h(h, n_small, zeta):
    """foldH (prove.go:670-705): H0 + zeta^(n+2) H1 + zeta^(2(n+2)) H2."""
    m = n_small + 2
    z = pow(zeta, m, R)
    return [((h[2 * m + i] * z + h[m + i]) * z + h[i]) % R for i in range(m)]


def linearized(blinded_z, s3, ql, qr, qm, qo, qk, pi2, qcp, s1, s2, alpha, l, r, o, lag):
    """Inner loop of computeLinearizedPolynomial (prove.go:1347-1386), verbatim."""
    rl = r * l % R
    out = []
    for i, zi in enumerate(blinded_z):
        t = zi * s2 % R
        if i < len(s3):
            t = (t + s3[i] * s1) % R
        t = t * alpha % R
        if i < len(qm):
            t = (t + ql[i] * l + qm[i] * rl + qr[i] * r + qo[i] * o + qk[i]) % R
            for j in range(len(qcp)):
                t = (t + pi2[j][i] * qcp[j]) % R
        out.append((t + zi * lag) % R)
    return out


# ---------------------------------------------------------------- PlonK verifier (trapdoor)
def g1_raw_bytes(p) -> bytes:
    """G1Affine.RawBytes = Marshal (deriveRandomness verify.go:342-360, bindPublicData
    :296-340, kzg deriveGamma, the BSB22 hash prove.go:341): X | Y big-endian,
    infinity = 0x40 | zeros (gnark-crypto mUncompressedInfinity)."""
    if p is INF:
        return bytes([0x40]) + bytes(95)
    return p[0].to_bytes(48, "big") + p[1].to_bytes(48, "big")


g1_marshal = g1_raw_bytes  # round-1 name


def g1_compress(p) -> bytes:
    """G1Affine.Bytes (compressed): X big-endian with the zcash flags 0x80 (y
    smallest) / 0xA0 (y largest) / 0xC0 (infinity); inverse of g1_decompress_zcash,
    which the bellman_test.go keys pin.  (Marshal is NOT this: it is RawBytes.)"""
    if p is INF:
        return bytes([0xC0]) + bytes(47)
    b = bytearray(p[0].to_bytes(48, "big"))
    b[0] |= 0xA0 if p[1] > P - p[1] else 0x80
    return bytes(b)


def expand_message_xmd(msg: bytes, dst: bytes, n: int) -> bytes:
    """RFC 9380 section 5.3.1 with SHA-256 (gnark-crypto ecc/hash.ExpandMsgXmd [ext])."""
    import hashlib
    b_in, r_in = 64, 32
    ell = (n + r_in - 1) // r_in
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    b0 = hashlib.sha256(bytes(b_in) + msg + n.to_bytes(2, "big") + b"\x00" + dst_prime).digest()
    out, bi = b"", b"\x00" * r_in
    for i in range(1, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:n]


def hash_to_field(msg: bytes, dst: bytes = b"BSB22-Plonk") -> int:
    """gnark-crypto bls12-381 fr.Hash(msg, dst, 1) (hash_to_field.New, the default
    HashToFieldFn of the PlonK prover/verifier: prove.go:232-234, verify.go:127-129):
    L = 16 + 32 bytes of expand_message_xmd, big-endian, mod r.  Parity unpinned
    (gnark-crypto is absent); prover and verifier here share it."""
    return int.from_bytes(expand_message_xmd(msg, dst, 48), "big") % R


class Transcript:
    """gnark-crypto fiat-shamir (restated): challenge i = H(name_i | value_(i-1) | bindings_i)."""

    def __init__(self, *names, h=None):
        import hashlib
        self.h = h or hashlib.sha256
        self.order, self.data, self.values = list(names), {n: [] for n in names}, {}

    def bind(self, name, b):
        self.data[name].append(bytes(b))

    def challenge(self, name) -> int:
        i = self.order.index(name)
        h = self.h()
        h.update(name.encode())
        if i:
            h.update(self.values[self.order[i - 1]])
        for d in self.data[name]:
            h.update(d)
        self.values[name] = h.digest()
        return int.from_bytes(self.values[name], "big") % R


def _derive(fs, name, *points):
    for p in points:
        fs.bind(name, g1_raw_bytes(p))
    return fs.challenge(name)


def _kzg_check_trapdoor(digest, proof_h, point, value, tau) -> bool:
    """KZG opening check with the SRS secret instead of the pairing:
    [w(tau)] (tau - z) == C - [y] G  <=>  e(W, [tau - z]_2) == e(C - [y]G, G2)."""
    lhs = g1_mul(proof_h, (tau - point) % R)
    rhs = g1_add(digest, g1_neg(g1_mul(G1_GEN, value)))
    return lhs == rhs


def plonk_verify_trapdoor(proof, vk, tau, public=(), challenge_hash=None, folding_hash=None) -> bool:
    """backend/plonk/bls12-381 Verify (verify.go:45-290) with public inputs and
    BSB22 commitments; the two KZG batch checks use the SRS trapdoor tau.
    proof / vk: plain dicts of affine points (x, y ints) and fr ints:
      proof: LRO[3], Z, H[3], batched_H, claimed[7 + ncmt], zs_H, zu, bsb22[ncmt]
      vk: n, omega, u (coset shift), S[3], Ql, Qr, Qm, Qo, Qk, Qcp[ncmt],
          nb_public, cmt_idx[ncmt]."""
    n, u = vk["n"], vk["u"]
    qcp = vk.get("Qcp", [])
    bsb = proof.get("bsb22", [])
    if len(bsb) != len(qcp) or len(public) != vk.get("nb_public", 0):
        return False
    fs = Transcript("gamma", "beta", "alpha", "zeta", h=challenge_hash)
    # G1Affine.Marshal() = the uncompressed RawBytes: groth16/bls12-381/verify.go:80-82 copies
    # Marshal() and continues at SizeOfG1AffineUncompressed; plonk/bn254/solidity.go binds X | Y
    for p in list(vk["S"]) + [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"]] + list(qcp):
        fs.bind("gamma", g1_raw_bytes(p))
    for x in public:
        fs.bind("gamma", (x % R).to_bytes(32, "big"))
    gamma = _derive(fs, "gamma", *proof["LRO"])
    beta = _derive(fs, "beta")
    alpha = _derive(fs, "alpha", *bsb, proof["Z"])
    zeta = _derive(fs, "zeta", *proof["H"])
    zn = pow(zeta, n, R)
    lag1 = (zn - 1) * pow(zeta - 1, -1, R) % R * pow(n, -1, R) % R
    # PI(zeta) = sum_i L_i(zeta) w_i + hashed BSB22 commitments at their rows (verify.go:102-155)
    w = vk["omega"]
    pi = 0
    for i, x in enumerate(public):
        wi = pow(w, i, R)
        li = wi * (zn - 1) % R * pow(n * (zeta - wi), -1, R) % R
        pi = (pi + li * x) % R
    for j, c in enumerate(bsb):
        hc = hash_to_field(g1_raw_bytes(c))
        wi = pow(w, vk["nb_public"] + vk["cmt_idx"][j], R)
        li = wi * (zn - 1) % R * pow(n * (zeta - wi), -1, R) % R
        pi = (pi + li * hc) % R
    zu = proof["zu"]
    cl = proof["claimed"]
    hq, lin, l, r, o, s1, s2 = cl[:7]
    qcz = cl[7:]
    # quotient identity (verify.go:158-195)
    t = (s1 * beta + l + gamma) * (s2 * beta + r + gamma) % R * (o + gamma) % R * alpha % R * zu % R
    rhs = (lin + pi + t - lag1 * alpha % R * alpha) % R * pow((zn - 1) % R, -1, R) % R
    if hq != rhs:
        return False
    # folded H digest and linearized digest (verify.go:197-250)
    zp = pow(zeta, n + 2, R)
    fh = g1_add(g1_add(proof["H"][0], g1_mul(proof["H"][1], zp)), g1_mul(proof["H"][2], zp * zp % R))
    a1 = zu * beta % R * ((beta * s1 + l + gamma) % R) % R * ((beta * s2 + r + gamma) % R) % R * alpha % R
    a2 = (beta * zeta + l + gamma) * ((beta * zeta * u + r + gamma) % R) % R * \
        ((beta * zeta * u * u + o + gamma) % R) % R
    a2 = ((-a2) * alpha + lag1 * alpha % R * alpha) % R
    pts = list(bsb) + [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"], vk["S"][2], proof["Z"]]
    scs = list(qcz) + [l, r, l * r % R, o, 1, a1, a2]
    lin_d = INF
    for p, s in zip(pts, scs):
        lin_d = g1_add(lin_d, g1_mul(p, s))
    # kzg.FoldProof + BatchVerifyMultiPoints (verify.go:252-290), trapdoor checks
    digests = [fh, lin_d, proof["LRO"][0], proof["LRO"][1], proof["LRO"][2], vk["S"][0], vk["S"][1]] + list(qcp)
    fsg = Transcript("gamma", h=folding_hash)
    fsg.bind("gamma", (zeta % R).to_bytes(32, "big"))
    for d in digests:
        fsg.bind("gamma", g1_raw_bytes(d))
    for c in cl:
        fsg.bind("gamma", (c % R).to_bytes(32, "big"))
    fsg.bind("gamma", (zu % R).to_bytes(32, "big"))
    gf = fsg.challenge("gamma")
    fd, fy, gp = INF, 0, 1
    for d, y in zip(digests, cl):
        fd = g1_add(fd, g1_mul(d, gp))
        fy = (fy + gp * y) % R
        gp = gp * gf % R
    if not _kzg_check_trapdoor(fd, proof["batched_H"], zeta, fy, tau):
        return False
    return _kzg_check_trapdoor(proof["Z"], proof["zs_H"], zeta * vk["omega"] % R, zu, tau)
