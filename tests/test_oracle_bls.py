"""Pins the BLS12-381 oracle (oracle/bls12_381_oracle.py) against the fixtures
the reference holds for this curve: the moduli (emparams.go) and the compressed
G1 points of backend/groth16/bellman_test.go (tests/golden/bls12_381_pins.json,
extracted by tests/golden/make_golden_bls.py)."""
import json
import os
import random

import bls12_381_oracle as b

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
