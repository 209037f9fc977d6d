"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Pure-Python big-integer restatement of the reference's Groth16/BN254 prover hot
path (tumberger/gnark-fork, gnark v0.10.0-alpha).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the *checker*.  The product path (``gnark-fork_amd``)
never imports it.

Parity pins (see DESIGN.md "Oracle"):
  * p, r: backend/groth16/bn254/solidity.go:41-42
  * omega_n = 5^((r-1)/n): std/commitments/fri/fri_test.go:35 gives omega_256^-1,
    checked in tests/test_oracle_pins.py
  * witness binary encoding KAT: backend/witness/witness.go:33-36
  * filterHeap KATs: backend/groth16/bn254/utils_test.go:17-38
  * cubic circuit (X=3, Y=35): examples/cubic/cubic.go:29-33, cubic_test.go
  * Groth16 verification equation: backend/groth16/bn254/verify.go:43-140
    (restated with a from-spec optimal-ate pairing below).
MSM / NTT output *values* have no reference golden vectors;
they are pinned through the verification equation and mathematical identities.

The arithmetic of gnark-crypto v0.12.2-0.20231117165148-e77308824822 (go.mod:8,
not present in the container) is restated from its published algorithm:
Montgomery form with R = 2^256, little-endian u64 limbs, DIF/DIT radix-2 FFT
with the conventions used at backend/groth16/bn254/prove.go:369-393.
"""
from __future__ import annotations

import hashlib
import struct

# --------------------------------------------------------------------------
# Fields  (backend/groth16/bn254/solidity.go:41-42)
# --------------------------------------------------------------------------
P = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
MONT = 1 << 256
FR_BYTES = 32
FP_BYTES = 32

# gnark-crypto fft.Domain: FrMultiplicativeGen = 5, 2-adicity 28 [ext; pinned by
# std/commitments/fri/fri_test.go:35 -> tests/test_oracle_pins.py]
FR_GEN = 5
FR_TWO_ADICITY = 28


def inv(x: int, m: int) -> int:
    return pow(x, -1, m)


def to_mont(x: int, m: int) -> int:
    return (x * MONT) % m


def from_mont(x: int, m: int) -> int:
    return (x * inv(MONT, m)) % m


def fr_to_bytes(x: int) -> bytes:
    """gnark fr.Element in memory: Montgomery form, [4]uint64 little-endian."""
    return to_mont(x % R, R).to_bytes(32, "little")


def fr_from_bytes(b: bytes) -> int:
    return from_mont(int.from_bytes(b[:32], "little"), R)


def fp_to_bytes(x: int) -> bytes:
    return to_mont(x % P, P).to_bytes(32, "little")


def fp_from_bytes(b: bytes) -> int:
    return from_mont(int.from_bytes(b[:32], "little"), P)


def fr_vec_to_bytes(v) -> bytes:
    return b"".join(fr_to_bytes(x) for x in v)


def fr_vec_from_bytes(b: bytes):
    return [fr_from_bytes(b[i:i + 32]) for i in range(0, len(b), 32)]


# --------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2+1)
# --------------------------------------------------------------------------
class Fp2:
    __slots__ = ("a0", "a1")

    def __init__(self, a0=0, a1=0):
        self.a0 = a0 % P
        self.a1 = a1 % P

    def __add__(self, o):
        return Fp2(self.a0 + o.a0, self.a1 + o.a1)

    def __sub__(self, o):
        return Fp2(self.a0 - o.a0, self.a1 - o.a1)

    def __neg__(self):
        return Fp2(-self.a0, -self.a1)

    def __mul__(self, o):
        if isinstance(o, int):
            return Fp2(self.a0 * o, self.a1 * o)
        return Fp2(self.a0 * o.a0 - self.a1 * o.a1, self.a0 * o.a1 + self.a1 * o.a0)

    __rmul__ = __mul__

    def __eq__(self, o):
        if isinstance(o, int):
            return self.a0 == o % P and self.a1 == 0
        return self.a0 == o.a0 and self.a1 == o.a1

    def __hash__(self):
        return hash((self.a0, self.a1))

    def is_zero(self):
        return self.a0 == 0 and self.a1 == 0

    def inv(self):
        d = inv((self.a0 * self.a0 + self.a1 * self.a1) % P, P)
        return Fp2(self.a0 * d, -self.a1 * d)

    def __pow__(self, e):
        res, b = Fp2(1, 0), self
        while e:
            if e & 1:
                res = res * b
            b = b * b
            e >>= 1
        return res

    def conj(self):
        return Fp2(self.a0, -self.a1)

    def __repr__(self):
        return f"Fp2({self.a0:#x}, {self.a1:#x})"


class _FpOps:
    """int-valued field ops for G1."""
    zero, one = 0, 1

    @staticmethod
    def add(a, b): return (a + b) % P
    @staticmethod
    def sub(a, b): return (a - b) % P
    @staticmethod
    def mul(a, b): return (a * b) % P
    @staticmethod
    def neg(a): return (-a) % P
    @staticmethod
    def inv(a): return inv(a, P)
    @staticmethod
    def is_zero(a): return a % P == 0


class _Fp2Ops:
    zero, one = Fp2(0, 0), Fp2(1, 0)

    @staticmethod
    def add(a, b): return a + b
    @staticmethod
    def sub(a, b): return a - b
    @staticmethod
    def mul(a, b): return a * b
    @staticmethod
    def neg(a): return -a
    @staticmethod
    def inv(a): return a.inv()
    @staticmethod
    def is_zero(a): return a.is_zero()


# curve constants: y^2 = x^3 + 3 (std/algebra/emulated/sw_emulated/params.go:49);
# twist b' = 3/(9+u) [ext: gnark-crypto bn254 bTwistCurveCoeff]
B1 = 3
B2 = Fp2(3, 0) * Fp2(9, 1).inv()

# Generators [ext: gnark-crypto bn254 Generators(); G1=(1,2), G2 = EIP-197 generator].
G1_GEN = (1, 2)
G2_GEN = (
    Fp2(10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
    Fp2(8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


# --------------------------------------------------------------------------
# Curve arithmetic: affine points are tuples (x, y) or None (infinity).
# Jacobian (X, Y, Z): x = X/Z^2, y = Y/Z^3 (gnark G1Jac convention).
# --------------------------------------------------------------------------
def jac_from_affine(F, p):
    if p is None:
        return (F.one, F.one, F.zero)
    return (p[0], p[1], F.one)


def jac_is_inf(F, p):
    return F.is_zero(p[2])


def jac_double(F, p):
    X, Y, Z = p
    if F.is_zero(Z):
        return p
    A = F.mul(X, X)
    Bq = F.mul(Y, Y)
    C = F.mul(Bq, Bq)
    t = F.add(X, Bq)
    D = F.sub(F.sub(F.mul(t, t), A), C)
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fv = F.mul(E, E)
    X3 = F.sub(Fv, F.add(D, D))
    C8 = F.add(C, C); C8 = F.add(C8, C8); C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    YZ = F.mul(Y, Z)
    Z3 = F.add(YZ, YZ)
    return (X3, Y3, Z3)


def jac_add(F, p, q):
    if F.is_zero(p[2]):
        return q
    if F.is_zero(q[2]):
        return p
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    Z1Z1 = F.mul(Z1, Z1)
    Z2Z2 = F.mul(Z2, Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    if U1 == U2:
        if S1 == S2:
            return jac_double(F, p)
        return (F.one, F.one, F.zero)
    H = F.sub(U2, U1)
    Rr = F.sub(S2, S1)
    HH = F.mul(H, H)
    HHH = F.mul(H, HH)
    V = F.mul(U1, HH)
    X3 = F.sub(F.sub(F.mul(Rr, Rr), HHH), F.add(V, V))
    Y3 = F.sub(F.mul(Rr, F.sub(V, X3)), F.mul(S1, HHH))
    Z3 = F.mul(F.mul(Z1, Z2), H)
    return (X3, Y3, Z3)


def jac_neg(F, p):
    return (p[0], F.neg(p[1]), p[2])


def jac_to_affine(F, p):
    if F.is_zero(p[2]):
        return None
    zi = F.inv(p[2])
    zi2 = F.mul(zi, zi)
    return (F.mul(p[0], zi2), F.mul(p[1], F.mul(zi2, zi)))


def jac_mul(F, p, k: int):
    k %= R
    acc = (F.one, F.one, F.zero)
    for bit in bin(k)[2:] if k else "":
        acc = jac_double(F, acc)
        if bit == "1":
            acc = jac_add(F, acc, p)
    return acc


def aff_mul(F, p, k):
    return jac_to_affine(F, jac_mul(F, jac_from_affine(F, p), k))


def aff_add(F, p, q):
    return jac_to_affine(F, jac_add(F, jac_from_affine(F, p), jac_from_affine(F, q)))


def g1_mul(p, k):
    return aff_mul(_FpOps, p, k)


def g2_mul(p, k):
    return aff_mul(_Fp2Ops, p, k)


def g1_add(p, q):
    return aff_add(_FpOps, p, q)


def g2_add(p, q):
    return aff_add(_Fp2Ops, p, q)


def on_curve_g1(p):
    if p is None:
        return True
    x, y = p
    return (y * y - x * x * x - B1) % P == 0


def on_curve_g2(p):
    if p is None:
        return True
    x, y = p
    return (y * y - x * x * x - B2).is_zero()


def msm(F, points, scalars, c: int = 0):
    """Pippenger bucket MSM (unsigned windows) over affine points.

    Restates gnark-crypto ``G1Jac.MultiExp`` semantics [ext]: result =
    sum_i scalars[i]*points[i]; affine infinity (None) contributes nothing.
    """
    n = len(points)
    assert n == len(scalars)
    if n == 0:
        return None
    if c == 0:
        c = max(2, min(16, n.bit_length() - 2))
    nw = (256 + c - 1) // c
    ks = [s % R for s in scalars]
    total = (F.one, F.one, F.zero)
    for w in reversed(range(nw)):
        for _ in range(c):
            total = jac_double(F, total)
        buckets = [None] * (1 << c)
        for p, k in zip(points, ks):
            if p is None:
                continue
            d = (k >> (w * c)) & ((1 << c) - 1)
            if d:
                q = jac_from_affine(F, p)
                buckets[d] = q if buckets[d] is None else jac_add(F, buckets[d], q)
        run = (F.one, F.one, F.zero)
        acc = (F.one, F.one, F.zero)
        for d in range((1 << c) - 1, 0, -1):
            if buckets[d] is not None:
                run = jac_add(F, run, buckets[d])
            acc = jac_add(F, acc, run)
        total = jac_add(F, total, acc)
    return jac_to_affine(F, total)


def msm_g1(points, scalars, c=0):
    return msm(_FpOps, points, scalars, c)


def msm_g2(points, scalars, c=0):
    return msm(_Fp2Ops, points, scalars, c)


# --------------------------------------------------------------------------
# Point byte layouts (gnark-crypto memory layout: Montgomery limbs LE)
# G1Affine {X, Y fp.Element} = 64 B, infinity = all-zero (icicle.go:98-105).
# G2Affine {X, Y E2{A0, A1}} = 128 B.
# --------------------------------------------------------------------------
def g1_to_bytes(p) -> bytes:
    if p is None:
        return bytes(64)
    return fp_to_bytes(p[0]) + fp_to_bytes(p[1])


def g1_from_bytes(b: bytes):
    if b[:64] == bytes(64):
        return None
    return (fp_from_bytes(b[0:32]), fp_from_bytes(b[32:64]))


def g2_to_bytes(p) -> bytes:
    if p is None:
        return bytes(128)
    x, y = p
    return fp_to_bytes(x.a0) + fp_to_bytes(x.a1) + fp_to_bytes(y.a0) + fp_to_bytes(y.a1)


def g2_from_bytes(b: bytes):
    if b[:128] == bytes(128):
        return None
    return (Fp2(fp_from_bytes(b[0:32]), fp_from_bytes(b[32:64])),
            Fp2(fp_from_bytes(b[64:96]), fp_from_bytes(b[96:128])))


def g1_raw_encode(p) -> bytes:
    """gnark RawEncoding of G1Affine: X|Y big-endian, infinity flag 0b01<<6 [ext]."""
    if p is None:
        b = bytearray(64)
        b[0] |= 0x40
        return bytes(b)
    return p[0].to_bytes(32, "big") + p[1].to_bytes(32, "big")


def g2_raw_encode(p) -> bytes:
    """X.A1|X.A0|Y.A1|Y.A0 big-endian (test/assert_solidity.go:60-69)."""
    if p is None:
        b = bytearray(128)
        b[0] |= 0x40
        return bytes(b)
    x, y = p
    return b"".join(v.to_bytes(32, "big") for v in (x.a1, x.a0, y.a1, y.a0))


# --------------------------------------------------------------------------
# FFT domain + gnark FFT conventions (prove.go:369-393; gnark-crypto fft [ext])
# --------------------------------------------------------------------------
def bitrev(i: int, logn: int) -> int:
    return int(format(i, f"0{logn}b")[::-1], 2) if logn else 0


class Domain:
    """Restates gnark-crypto ``fft.NewDomain`` (setup.go:111 call site)."""

    def __init__(self, m: int):
        n = 1
        while n < m:
            n <<= 1
        self.cardinality = n
        self.log_n = n.bit_length() - 1
        assert self.log_n <= FR_TWO_ADICITY
        self.generator = pow(FR_GEN, (R - 1) >> self.log_n, R)  # omega_n
        self.generator_inv = inv(self.generator, R)
        self.cardinality_inv = inv(n, R)
        self.fr_mul_gen = FR_GEN
        self.fr_mul_gen_inv = inv(FR_GEN, R)

    def coset_table(self):
        g, t, x = self.fr_mul_gen, [], 1
        for _ in range(self.cardinality):
            t.append(x)
            x = x * g % R
        return t

    def coset_table_inv(self):
        g, t, x = self.fr_mul_gen_inv, [], 1
        for _ in range(self.cardinality):
            t.append(x)
            x = x * g % R
        return t


def _dif(a, w):
    """Decimation in frequency: natural in, bit-reversed out (unscaled)."""
    n = len(a)
    m = n >> 1
    while m >= 1:
        # omega for this stage has order 2m
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
    """Decimation in time: bit-reversed in, natural out (unscaled)."""
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
    """domain.FFT(a, decimation, [OnCoset()]) -- in place, returns a."""
    n = dom.cardinality
    logn = dom.log_n
    assert len(a) == n
    if coset:
        ct = dom.coset_table()
        if decimation == DIT:
            for i in range(n):
                a[i] = a[i] * ct[bitrev(i, logn)] % R
        else:
            for i in range(n):
                a[i] = a[i] * ct[i] % R
    if decimation == DIF:
        _dif(a, dom.generator)
    else:
        _dit(a, dom.generator)
    return a


def fft_inverse(dom: Domain, a, decimation, coset=False):
    """domain.FFTInverse(a, decimation, [OnCoset()])."""
    n = dom.cardinality
    logn = dom.log_n
    assert len(a) == n
    if decimation == DIF:
        _dif(a, dom.generator_inv)
    else:
        _dit(a, dom.generator_inv)
    ninv = dom.cardinality_inv
    if not coset:
        for i in range(n):
            a[i] = a[i] * ninv % R
        return a
    cti = dom.coset_table_inv()
    if decimation == DIT:
        for i in range(n):
            a[i] = a[i] * cti[i] % R * ninv % R
    else:
        for i in range(n):
            a[i] = a[i] * cti[bitrev(i, logn)] % R * ninv % R
    return a


def compute_h(a, b, c, dom: Domain):
    """Restates computeH, backend/groth16/bn254/prove.go:353-396.

    Returns h (length n) in bit-reversed coefficient order."""
    n = dom.cardinality
    a = list(a) + [0] * (n - len(a))
    b = list(b) + [0] * (n - len(b))
    c = list(c) + [0] * (n - len(c))
    fft_inverse(dom, a, DIF)
    fft_inverse(dom, b, DIF)
    fft_inverse(dom, c, DIF)
    fft(dom, a, DIT, coset=True)
    fft(dom, b, DIT, coset=True)
    fft(dom, c, DIT, coset=True)
    den = inv((pow(dom.fr_mul_gen, n, R) - 1) % R, R)
    for i in range(n):
        a[i] = (a[i] * b[i] - c[i]) % R * den % R
    fft_inverse(dom, a, DIF, coset=True)
    return a


# --------------------------------------------------------------------------
# R1CS (minimal restatement of constraint/bn254 R1C + solver output)
# Each constraint: (L, R, O), each a list of (wire_id, coeff).
# --------------------------------------------------------------------------
class R1CS:
    def __init__(self, nb_public, nb_secret, nb_internal, constraints):
        self.nb_public = nb_public      # includes the ONE wire
        self.nb_secret = nb_secret
        self.nb_internal = nb_internal
        self.constraints = constraints

    @property
    def nb_wires(self):
        return self.nb_public + self.nb_secret + self.nb_internal

    def solution(self, w):
        """A, B, C vectors (constraint/bn254/solver.go:532-560)."""
        def ev(le):
            return sum(w[i] * k for i, k in le) % R
        A, B, C = [], [], []
        for L, Rr, O in self.constraints:
            A.append(ev(L)); B.append(ev(Rr)); C.append(ev(O))
        for x, y, z in zip(A, B, C):
            if (x * y - z) % R:
                raise ValueError("constraint not satisfied")
        return A, B, C


def cubic_r1cs():
    """examples/cubic/cubic.go:29-33 compiled per frontend/cs/r1cs/api.go:198-232,
    api_assertions.go:30-35, builder.go:177-194.
    wires: 0=ONE, 1=Y (public), 2=X (secret), 3=X*X, 4=X^3."""
    cons = [
        ([(2, 1)], [(2, 1)], [(3, 1)]),
        ([(3, 1)], [(2, 1)], [(4, 1)]),
        ([(0, 1)], [(1, 1)], [(4, 1), (2, 1), (0, 5)]),
    ]
    return R1CS(2, 1, 2, cons)


def cubic_witness(x=3, y=35):
    return [1, y, x, x * x % R, x * x * x % R]


def mimc_chain_r1cs(nb_chains: int, rounds: int):
    """Synthetic x^5 chains (BASELINE config 4 shape; std/hash/mimc pow5):
    per round: t=x*x, u=t*t, x'=u*x + k  (3 constraints / round).
    Wires: ONE, then nb_chains secret inputs, then internal wires."""
    nb_public = 1
    nb_secret = nb_chains
    cons = []
    wid = nb_public + nb_secret
    for ch in range(nb_chains):
        x = nb_public + ch
        for rd in range(rounds):
            k = (rd * 7 + 3) % R
            t, u, xn = wid, wid + 1, wid + 2
            wid += 3
            cons.append(([(x, 1)], [(x, 1)], [(t, 1)]))
            cons.append(([(t, 1)], [(t, 1)], [(u, 1)]))
            # u * x = xn - k  ->  O = xn + (-k)*ONE
            cons.append(([(u, 1)], [(x, 1)], [(xn, 1), (0, (-k) % R)]))
            x = xn
    return R1CS(nb_public, nb_secret, wid - nb_public - nb_secret, cons)


def mimc_chain_witness(rcs: R1CS, inputs):
    w = [0] * rcs.nb_wires
    w[0] = 1
    for i, v in enumerate(inputs):
        w[1 + i] = v % R
    for L, Rr, O in rcs.constraints:
        a = sum(w[i] * k for i, k in L) % R
        b = sum(w[i] * k for i, k in Rr) % R
        out_wire, _ = O[0]
        rest = sum(w[i] * k for i, k in O[1:]) % R
        w[out_wire] = (a * b - rest) % R
    return w


# --------------------------------------------------------------------------
# Groth16 setup / prove (setup.go:85-337, prove.go:63-322)
# --------------------------------------------------------------------------
class ToxicWaste:
    def __init__(self, t, alpha, beta, gamma, delta):
        self.t, self.alpha, self.beta, self.gamma, self.delta = t, alpha, beta, gamma, delta
        self.gamma_inv = inv(gamma, R)
        self.delta_inv = inv(delta, R)


def setup_abc(rcs: R1CS, dom: Domain, tw: ToxicWaste):
    """setup.go:352-434."""
    nw = rcs.nb_wires
    A, B, C = [0] * nw, [0] * nw, [0] * nw
    w = dom.generator
    n = dom.cardinality
    tvals = []
    wi = 1
    for _ in range(len(rcs.constraints) + 1):
        tvals.append((tw.t - wi) % R)
        wi = wi * w % R
    tinv = [inv(x, R) for x in tvals]
    L = (pow(tw.t, n, R) - 1) * tinv[0] % R * dom.cardinality_inv % R
    for j, (Lc, Rc, Oc) in enumerate(rcs.constraints):
        for wid, k in Lc:
            A[wid] = (A[wid] + k * L) % R
        for wid, k in Rc:
            B[wid] = (B[wid] + k * L) % R
        for wid, k in Oc:
            C[wid] = (C[wid] + k * L) % R
        L = L * w % R * tvals[j] % R * tinv[j + 1] % R
    return A, B, C


class ProvingKey:
    pass


class VerifyingKey:
    pass


def setup(rcs: R1CS, tw: ToxicWaste):
    """Groth16 Setup without commitments (setup.go:85-337). Returns (pk, vk)."""
    nw = rcs.nb_wires
    nb_public = rcs.nb_public
    nb_private = rcs.nb_secret + rcs.nb_internal
    dom = Domain(len(rcs.constraints))
    A, B, C = setup_abc(rcs, dom, tw)
    pkK, vkK = [], []
    for i in range(nw):
        t1 = (A[i] * tw.beta + B[i] * tw.alpha + C[i]) % R
        if i < nb_public:
            vkK.append(t1 * tw.gamma_inv % R)
        else:
            pkK.append(t1 * tw.delta_inv % R)
    n = dom.cardinality
    zdt = (pow(tw.t, n, R) - 1) * tw.delta_inv % R
    Z = []
    for _ in range(n):
        Z.append(zdt)
        zdt = zdt * tw.t % R
    infA = [a == 0 for a in A]
    infB = [b == 0 for b in B]
    Af = [a for a in A if a]
    Bf = [b for b in B if b]
    pk = ProvingKey()
    vk = VerifyingKey()
    pk.domain = dom
    pk.scalars = dict(A=Af, B=Bf, K=pkK, Z=Z, alpha=tw.alpha, beta=tw.beta, delta=tw.delta)
    pk.g1_alpha = g1_mul(G1_GEN, tw.alpha)
    pk.g1_beta = g1_mul(G1_GEN, tw.beta)
    pk.g1_delta = g1_mul(G1_GEN, tw.delta)
    pk.g1_A = [g1_mul(G1_GEN, s) for s in Af]
    pk.g1_B = [g1_mul(G1_GEN, s) for s in Bf]
    zpts = [g1_mul(G1_GEN, s) for s in Z]
    logn = dom.log_n
    zpts = [zpts[bitrev(i, logn)] for i in range(n)]  # setup.go:265 bitReverse
    pk.g1_Z = zpts[: n - 1]
    pk.g1_K = [g1_mul(G1_GEN, s) for s in pkK]
    pk.g2_B = [g2_mul(G2_GEN, s) for s in Bf]
    pk.g2_beta = g2_mul(G2_GEN, tw.beta)
    pk.g2_delta = g2_mul(G2_GEN, tw.delta)
    pk.infinity_A, pk.infinity_B = infA, infB
    pk.nb_infinity_A = sum(infA)
    pk.nb_infinity_B = sum(infB)
    vk.g1_alpha = pk.g1_alpha
    vk.g1_K = [g1_mul(G1_GEN, s) for s in vkK]
    vk.g2_beta = pk.g2_beta
    vk.g2_delta = pk.g2_delta
    vk.g2_gamma = g2_mul(G2_GEN, tw.gamma)
    return pk, vk


def filter_heap(slice_, slice_first_index, to_remove):
    """prove.go:328-351 (KATs: utils_test.go:17-38)."""
    if not to_remove:
        return list(slice_)
    rm = set(to_remove)
    return [v for i, v in enumerate(slice_) if i + slice_first_index not in rm]


class Proof:
    def __init__(self, ar, bs, krs):
        self.Ar, self.Bs, self.Krs = ar, bs, krs

    def raw_bytes(self):
        """WriteRawTo prefix Ar|Bs|Krs (marshal.go:41-66), no commitments:
        followed by u32 len(Commitments)=0 and CommitmentPok (infinity)."""
        return g1_raw_encode(self.Ar) + g2_raw_encode(self.Bs) + g1_raw_encode(self.Krs)


def prove(rcs: R1CS, pk, w, r: int, s: int, return_h=False):
    """Groth16 Prove with injected r, s (prove.go:63-322)."""
    A, B, C = rcs.solution(w)
    dom = pk.domain
    h = compute_h(A, B, C, dom)
    wA = [w[i] for i in range(len(w)) if not pk.infinity_A[i]]
    wB = [w[i] for i in range(len(w)) if not pk.infinity_B[i]]
    kr = (-(r * s)) % R
    d_r = g1_mul(pk.g1_delta, r)
    d_s = g1_mul(pk.g1_delta, s)
    d_kr = g1_mul(pk.g1_delta, kr)
    bs1 = msm_g1(pk.g1_B, wB)
    bs1 = g1_add(g1_add(bs1, pk.g1_beta), d_s)
    ar = msm_g1(pk.g1_A, wA)
    ar = g1_add(g1_add(ar, pk.g1_alpha), d_r)
    n = dom.cardinality
    krs2 = msm_g1(pk.g1_Z, h[: n - 1])
    priv = filter_heap(w[rcs.nb_public:], rcs.nb_public, [])
    krs = msm_g1(pk.g1_K, priv)
    krs = g1_add(krs, d_kr)
    krs = g1_add(krs, krs2)
    krs = g1_add(krs, g1_mul(ar, s))
    krs = g1_add(krs, g1_mul(bs1, r))
    bs = msm_g2(pk.g2_B, wB)
    bs = g2_add(bs, g2_mul(pk.g2_delta, s))
    bs = g2_add(bs, pk.g2_beta)
    pr = Proof(ar, bs, krs)
    if return_h:
        return pr, h
    return pr


def expected_proof_scalars(rcs: R1CS, tw: ToxicWaste, w, r, s):
    """Trapdoor check: discrete logs of (Ar, Bs, Krs) w.r.t. the generators.

    A = alpha + sum w_i u_i(t) + r delta; B = beta + sum w_i v_i(t) + s delta;
    C = (sum_priv w_i (beta u_i + alpha v_i + w_i(t)) + h(t) Z(t)) / delta
        + s A + r B - r s delta."""
    dom = Domain(len(rcs.constraints))
    Au, Bv, Cw = setup_abc(rcs, dom, tw)
    a = (tw.alpha + sum(wi * x for wi, x in zip(w, Au)) + r * tw.delta) % R
    b = (tw.beta + sum(wi * x for wi, x in zip(w, Bv)) + s * tw.delta) % R
    A, B, C = rcs.solution(w)
    h = compute_h(A, B, C, dom)
    n = dom.cardinality
    # h is bit-reversed coefficients: h(t) = sum_i h[i] t^{bitrev(i)}
    ht = sum(h[i] * pow(tw.t, bitrev(i, dom.log_n), R) for i in range(n)) % R
    zt = (pow(tw.t, n, R) - 1) % R
    priv = sum(w[i] * ((Au[i] * tw.beta + Bv[i] * tw.alpha + Cw[i]) % R)
               for i in range(rcs.nb_public, rcs.nb_wires)) % R
    c = ((priv + ht * zt) * tw.delta_inv + s * a + r * b - r * s * tw.delta) % R
    return a, b, c


# --------------------------------------------------------------------------
# Optimal-ate pairing on BN254 (from-spec restatement, used to run the
# reference's own correctness signal -- groth16 Verify, verify.go:43-140).
# Fp12 = Fp2[w]/(w^6 - xi), xi = 9 + u.
# --------------------------------------------------------------------------
BN_X = 4965661367192848881
XI = Fp2(9, 1)


class Fp12:
    """Elements as 6 Fp2 coefficients of w (w^6 = xi)."""
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = c

    @staticmethod
    def one():
        return Fp12([Fp2(1, 0)] + [Fp2(0, 0)] * 5)

    def __mul__(self, o):
        r = [Fp2(0, 0)] * 11
        for i, x in enumerate(self.c):
            if x.is_zero():
                continue
            for j, y in enumerate(o.c):
                if y.is_zero():
                    continue
                r[i + j] = r[i + j] + x * y
        out = r[:6]
        for k in range(6, 11):
            out[k - 6] = out[k - 6] + r[k] * XI
        return Fp12(out)

    def __eq__(self, o):
        return all(a == b for a, b in zip(self.c, o.c))

    def __pow__(self, e):
        res, b = Fp12.one(), self
        while e:
            if e & 1:
                res = res * b
            b = b * b
            e >>= 1
        return res

    def frob(self):
        # (sum c_i w^i)^p = sum conj(c_i) w^{ip}; w^p = w * xi^((p-1)/6)
        g = XI ** ((P - 1) // 6)
        out, gi = [], Fp2(1, 0)
        for i in range(6):
            out.append(self.c[i].conj() * gi)
            gi = gi * g
        return Fp12(out)

    def inv(self):
        # via norm to Fp6 is verbose; use exponentiation in the multiplicative group
        return self ** (P ** 12 - 2)


def _line(T, Q, Pt):
    """Evaluate line through T,Q (affine in twisted coords) at P (G1), embedded in Fp12.
    Untwist: (x, y) -> (x w^2, y w^3)."""
    (x1, y1), (x2, y2) = T, Q
    xp, yp = Pt
    if x1 == x2 and y1 == y2:
        lam = (x1 * x1 * 3) * (y1 * 2).inv()
    elif x1 == x2:
        # vertical line x - x1 : x_P - x1 w^2
        c = [Fp2(0, 0)] * 6
        c[0] = Fp2(xp, 0)
        c[2] = -x1
        return Fp12(c)
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    # l(P) = y_P - y1 w^3 - lam (x_P w - x1 w^3)   with lam scaled by w (untwist)
    c = [Fp2(0, 0)] * 6
    c[0] = Fp2(yp, 0)
    c[1] = -(lam * xp)
    c[3] = lam * x1 - y1
    return Fp12(c)


def _ate_loop_count():
    return 6 * BN_X + 2


def miller_loop(Pt, Q):
    if Pt is None or Q is None:
        return Fp12.one()
    T = Q
    f = Fp12.one()
    bits = bin(_ate_loop_count())[2:]
    for b in bits[1:]:
        f = f * f * _line(T, T, Pt)
        T = g2_add(T, T)
        if b == "1":
            f = f * _line(T, Q, Pt)
            T = g2_add(T, Q)
    # Frobenius twists: Q1 = pi(Q), Q2 = -pi^2(Q)
    gx = XI ** ((P - 1) // 3)
    gy = XI ** ((P - 1) // 2)
    Q1 = (Q[0].conj() * gx, Q[1].conj() * gy)
    gx2 = XI ** ((P * P - 1) // 3)
    gy2 = XI ** ((P * P - 1) // 2)
    Q2 = (Q[0] * gx2, -(Q[1] * gy2))
    f = f * _line(T, Q1, Pt)
    T = g2_add(T, Q1)
    f = f * _line(T, Q2, Pt)
    return f


def final_exp(f):
    return f ** ((P ** 12 - 1) // R)


def pairing(Pt, Q):
    return final_exp(miller_loop(Pt, Q))


def pairing_check(pairs):
    """prod e(P_i, Q_i) == 1."""
    f = Fp12.one()
    for Pt, Q in pairs:
        f = f * miller_loop(Pt, Q)
    return final_exp(f) == Fp12.one()


def verify(proof: Proof, vk, public_witness):
    """verify.go:43-140 without commitments:
    e(Krs, -delta) e(Ar, Bs) e(sum x_i K_i, -gamma) == e(alpha, beta)."""
    ksum = vk.g1_K[0]
    for x, k in zip(public_witness, vk.g1_K[1:]):
        ksum = g1_add(ksum, g1_mul(k, x))
    neg = lambda q: (q[0], -q[1])
    na = (vk.g1_alpha[0], (-vk.g1_alpha[1]) % P)
    return pairing_check([
        (proof.Krs, neg(vk.g2_delta)),
        (proof.Ar, proof.Bs),
        (ksum, neg(vk.g2_gamma)),
        (na, vk.g2_beta),
    ])


# --------------------------------------------------------------------------
# Witness binary encoding (backend/witness/witness.go:15-36)
# --------------------------------------------------------------------------
def witness_encode(public, secret) -> bytes:
    vals = list(public) + list(secret)
    out = struct.pack(">III", len(public), len(secret), len(vals))
    for v in vals:
        out += (v % R).to_bytes(32, "big")
    return out


# --------------------------------------------------------------------------
# Deterministic PRNG for fixtures (splitmix64; SURVEY 8d seed "groth")
# --------------------------------------------------------------------------
class SplitMix64:
    def __init__(self, seed=0x67726F7468):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def fr(self):
        while True:
            v = 0
            for k in range(4):
                v |= self.next() << (64 * k)
            v &= (1 << 254) - 1
            if v < R:
                return v


def sha_digest(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
