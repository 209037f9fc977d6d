"""Pins the BLS12-381 oracle (oracle/bls12_381_oracle.py) against the fixtures
the reference holds for this curve: the moduli (emparams.go) and the compressed
G1 points of backend/groth16/bellman_test.go (tests/golden/bls12_381_pins.json,
extracted by tests/golden/make_golden_bls.py)."""
import json
import os
import random

import bls12_381_oracle as b
import bls12_381_oracle as bo

HERE = os.path.dirname(os.path.abspath(__file__))
PINS = json.load(open(os.path.join(HERE, "golden", "bls12_381_pins.json")))


def test_moduli_match_reference_emparams():
    # std/math/emulated/emparams/emparams.go:145-171 (hex; decimal checked too)
    assert b.P == int(PINS["p_hex"], 16)
    assert b.R == int(PINS["r_hex"], 16)
    assert b.P == 4002409555221667393417789825735904156556882819939007885332058136124031650490837864442687629129015664037894272559787
    assert b.R == 52435875175126190479447740508185965837690552500527637822603658699938581184513


def test_bellman_points_on_curve_and_in_subgroup():
    # every G1 point of the reference's BLS12-381 Groth16 KATs: y^2 = x^3 + 4, r*P = O
    pts = [b.g1_decompress_zcash(bytes.fromhex(h)) for h in PINS["g1_compressed"]]
    assert len(pts) >= 10
    for p in pts:
        assert b.on_curve(p)
        assert b.g1_mul_raw(p, b.R) is b.INF
    assert b.on_curve(b.G1_GEN) and b.g1_mul_raw(b.G1_GEN, b.R) is b.INF


def test_msm_trapdoor_identity():
    rng = random.Random(3)
    ks = [rng.randrange(b.R) for _ in range(6)]
    ss = [rng.randrange(b.R) for _ in range(6)]
    pts = [b.g1_mul(b.G1_GEN, k) for k in ks]
    assert b.msm_g1(pts, ss) == b.msm_g1_trapdoor(ks, ss)


def test_fft_roundtrip_and_evaluation():
    rng = random.Random(5)
    n = 16
    d = b.Domain(n)
    assert pow(d.generator, n, b.R) == 1 and pow(d.generator, n // 2, b.R) != 1
    a = [rng.randrange(b.R) for _ in range(n)]
    # DIF: natural -> bit-reversed evaluations at omega^i
    ev = b.fft(d, list(a), b.DIF)
    for i in range(n):
        x = pow(d.generator, i, b.R)
        assert ev[b.bitrev(i, d.log_n)] == sum(c * pow(x, j, b.R) for j, c in enumerate(a)) % b.R
    # coset variants: round trips
    for dec, back in ((b.DIF, b.DIT), (b.DIT, b.DIF)):
        for coset in (False, True):
            src = list(a) if dec == b.DIF else [a[b.bitrev(i, d.log_n)] for i in range(n)]
            y = b.fft(d, list(src), dec, coset)
            z = b.fft_inverse(d, y, back, coset)
            assert z == src


def test_encodings_roundtrip():
    x = 123456789
    assert b.fp_from_bytes(b.fp_to_bytes(x)) == x
    assert b.fr_from_bytes(b.fr_to_bytes(x)) == x
    g = b.G1_GEN
    assert b.g1_from_bytes(b.g1_to_bytes(g)) == g
    assert b.g1_to_bytes(b.INF) == bytes(96)


# ---- row a21 restatements: internal consistency (no GPU)
def _copy_witness(n, seed):
    """A random permutation of the 3n wire slots made of cycles, and L/R/O values
    constant on each cycle (a witness that satisfies the copy constraints)."""
    import random
    rnd = random.Random(seed)
    slots = list(range(3 * n))
    rnd.shuffle(slots)
    perm = [0] * (3 * n)
    vals = [0] * (3 * n)
    i = 0
    while i < 3 * n:
        k = min(rnd.randint(1, 5), 3 * n - i)
        cyc = slots[i:i + k]
        v = rnd.randrange(bo.R)
        for a, b_ in zip(cyc, cyc[1:] + cyc[:1]):
            perm[a] = b_
            vals[a] = v
        i += k
    return perm, [vals[:n], vals[n:2 * n], vals[2 * n:]]


def test_ratio_copy_constraint_wraps_to_one():
    """For a satisfied permutation Z(w^n) = Z(1) = 1: the last ratio step closes the cycle."""
    n = 16
    dom = bo.Domain(n)
    perm, f = _copy_witness(n, 3)
    beta, gamma = 12345678910, 987654321
    z = bo.ratio_copy_constraint(f, perm, beta, gamma, dom)
    ids = bo.support_permutation(n, dom)
    i = n - 1
    num = den = 1
    for j in range(3):
        num = num * (f[j][i] + beta * ids[j * n + i] + gamma) % bo.R
        den = den * (f[j][i] + beta * ids[perm[j * n + i]] + gamma) % bo.R
    assert z[0] == 1
    assert z[n - 1] * num * pow(den, -1, bo.R) % bo.R == 1
    # a broken copy constraint does not close
    f[0][3] = (f[0][3] + 1) % bo.R
    z2 = bo.ratio_copy_constraint(f, perm, beta, gamma, dom)
    assert z2 != z


def test_divide_by_x_minus_a_identity():
    import random
    rnd = random.Random(5)
    f = [rnd.randrange(bo.R) for _ in range(33)]
    a = rnd.randrange(bo.R)
    fa = bo.evaluate(f, a)
    q = bo.divide_by_x_minus_a(f, fa, a)
    x = rnd.randrange(bo.R)
    assert (bo.evaluate(q, x) * (x - a) + fa - bo.evaluate(f, x)) % bo.R == 0


def test_fold_h_is_evaluation_split():
    import random
    rnd = random.Random(6)
    n = 8
    h = [rnd.randrange(bo.R) for _ in range(3 * (n + 2))]
    zeta = rnd.randrange(bo.R)
    folded = bo.fold_h(h, n, zeta)
    # sum_k zeta^(k(n+2)) H_k(X) evaluated at X = zeta equals h(zeta)
    assert bo.evaluate(folded, zeta) == bo.evaluate(h, zeta)


def test_g1_encodings():
    """G1Affine.Bytes (compressed) re-creates the reference's own compressed keys
    byte for byte (backend/groth16/bellman_test.go:19-132); G1Affine.Marshal, the
    encoding bindPublicData / kzg deriveGamma / the BSB22 hash bind, is RawBytes
    (uncompressed X | Y): groth16/bls12-381/verify.go:80-82 copies Marshal() and
    continues at SizeOfG1AffineUncompressed, and plonk/bn254/solidity.go:407-460
    binds X | Y words where verify.go:296-340 binds Marshal().  Both keep the
    gnark-crypto infinity flags."""
    for h in PINS["g1_compressed"]:
        raw = bytes.fromhex(h)
        assert b.g1_compress(b.g1_decompress_zcash(raw)) == raw
    assert b.g1_compress(b.INF) == bytes([0xC0]) + bytes(47)
    assert b.g1_raw_bytes(b.INF) == bytes([0x40]) + bytes(95)
    p = b.g1_mul(b.G1_GEN, 12345)
    assert b.g1_raw_bytes(p) == p[0].to_bytes(48, "big") + p[1].to_bytes(48, "big")


def test_expand_message_xmd_rfc9380_vectors():
    """expand_message_xmd(SHA-256) against RFC 9380 appendix K.1
    (DST QUUX-V01-CS02-with-expander-SHA256-128): the hash_to_field of the BSB22
    commitment value (prove.go:341-348) builds on it."""
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    assert b.expand_message_xmd(b"", dst, 0x20).hex() == \
        "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"
    assert b.expand_message_xmd(b"abc", dst, 0x20).hex() == \
        "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"


def test_bellman_g2_points_decompress_recompress():
    """The compressed G2 points of the reference's BLS12-381 Groth16 KATs
    (bellman_test.go: vk beta/gamma/delta_g2, proof B) decompress onto
    y^2 = x^3 + 4(1 + u), lie in the order-r subgroup and re-encode byte for
    byte; the standard generator G2_GEN used by the tests is on the same curve."""
    assert len(PINS["g2_compressed"]) >= 10
    for h in PINS["g2_compressed"][:12]:
        raw = bytes.fromhex(h)
        p = b.g2_decompress_zcash(raw)
        assert b.g2_on_curve(p)
        assert b.g2_compress(p) == raw
        assert b.g2_mul(p, b.R, reduce=False) is b.INF
    assert b.g2_on_curve(b.G2_GEN) and b.g2_mul(b.G2_GEN, b.R, reduce=False) is b.INF
    q = b.g2_mul(b.G2_GEN, 7)
    assert b.g2_add(q, b.g2_mul(b.G2_GEN, 5)) == b.g2_mul(b.G2_GEN, 12)
    assert b.g2_from_bytes(b.g2_to_bytes(q)) == q


def test_groth16_bls_oracle_scalars_cubic():
    """groth16_expected_scalars on the cubic circuit (examples/cubic, x^3 + x + 5 = y)
    over BLS12-381: the h(t) Z(t) = A(t) B(t) - C(t) shortcut agrees with an explicit
    interpolation of A, B, C over the domain."""
    R = b.R
    cons = [([(2, 1)], [(2, 1)], [(3, 1)]), ([(3, 1)], [(2, 1)], [(4, 1)]),
            ([(0, 1)], [(1, 1)], [(4, 1), (2, 1), (0, 5)])]
    w = [1, 35, 3, 9, 27]
    ks = b.groth16_setup_scalars(cons, 5, 2, 2, 123456789, 11, 13, 17)
    a, bb, c = b.groth16_expected_scalars(cons, w, 2, 2, ks, 123456789, 11, 13, 17, 3, 4)
    # A(t) = sum_j A_j L_j(t), by direct Lagrange interpolation over the 4-point domain
    n, t = 4, 123456789
    om = pow(b.FR_GEN, (R - 1) >> 2, R)
    pts = [pow(om, j, R) for j in range(n)]

    def lag(j):
        num, den = 1, 1
        for k in range(n):
            if k != j:
                num = num * (t - pts[k]) % R
                den = den * (pts[j] - pts[k]) % R
        return num * pow(den, -1, R) % R
    ev = [sum(w[i] * k for i, k in row) % R for row in (r[0] for r in cons)]
    At = sum(ev[j] * lag(j) for j in range(3)) % R
    assert a == (11 + At + 3 * 17) % R
