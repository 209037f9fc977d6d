"""The C restatement (large-size checker / cpu_baseline) agrees with the pinned
Python oracle and with the committed golden fixtures."""
import numpy as np
import pytest

import bn254_oracle as o
import coracle
from helpers import b, golden


def test_c_oracle_msm_matches_golden():
    for case in golden()["msm"]:
        f = coracle.msm_g1 if case["group"] == 1 else coracle.msm_g2
        assert f(b(case["points"]), b(case["scalars"]), case["n"]).hex() == case["expected"]


def test_c_oracle_ntt_matches_golden():
    for case in golden()["ntt"]:
        got = coracle.ntt(b(case["input"]), case["log_n"], case["inverse"], case["dif"], case["coset"])
        assert got.hex() == case["expected"], case


def test_c_oracle_groth16_matches_golden():
    for g in golden()["groth16"]:
        infA, infB = b(g["infA"]), b(g["infB"])
        nw = len(infA)
        ar, bs, krs, h = coracle.groth16_prove(
            g["log_n"], b(g["g1_A"]), len(b(g["g1_A"])) // 64, b(g["g1_B"]), len(b(g["g1_B"])) // 64,
            b(g["g1_Z"]), b(g["g1_K"]), len(b(g["g1_K"])) // 64, b(g["alpha1"]), b(g["beta1"]),
            b(g["delta1"]), b(g["g2_B"]), b(g["beta2"]), b(g["delta2"]), infA, infB, b(g["wires"]),
            nw, g["nb_public"], b(g["solA"]), b(g["solB"]), b(g["solC"]), len(b(g["solA"])) // 32,
            b(g["r"]), b(g["s"]), want_h=True)
        assert h.hex() == g["h"]
        assert ar.hex() == g["Ar"] and bs.hex() == g["Bs"] and krs.hex() == g["Krs"]


def test_golden_regenerates_from_python_oracle():
    """Fixtures are exactly what the pinned Python oracle produces."""
    g = golden()["groth16"][0]
    rcs = o.cubic_r1cs()
    tw = o.ToxicWaste(1234567, 891011, 121314, 151617, 181920)
    pk, vk = o.setup(rcs, tw)
    pr = o.prove(rcs, pk, o.cubic_witness(3, 35), 4242, 5353)
    assert o.g1_to_bytes(pr.Ar).hex() == g["Ar"]
    assert o.g2_to_bytes(pr.Bs).hex() == g["Bs"]
    assert o.g1_to_bytes(pr.Krs).hex() == g["Krs"]
    assert pr.raw_bytes().hex() == g["raw_prefix"]


@pytest.mark.parametrize("n", [1000, 4096])
def test_c_oracle_msm_trapdoor(n):
    from helpers import random_fr_mont
    ks = random_fr_mont(n, 11)
    ss = random_fr_mont(n, 12, "witness")
    pts = coracle.g1_batch_mul(o.g1_to_bytes(o.G1_GEN), ks.tobytes(), n)
    got = o.g1_from_bytes(coracle.msm_g1(bytes(pts), ss.tobytes(), n))
    kv = o.fr_vec_from_bytes(ks.tobytes())
    sv = o.fr_vec_from_bytes(ss.tobytes())
    assert got == o.g1_mul(o.G1_GEN, sum(x * y for x, y in zip(kv, sv)))


def test_c_oracle_ntt_roundtrip_2p16():
    from helpers import random_fr_mont
    v = random_fr_mont(1 << 16, 5).tobytes()
    f = coracle.ntt(v, 16, 0, 1, 1)
    back = coracle.ntt(f, 16, 1, 0, 1)  # DIF out is bit-reversed, DIT inverse takes it back
    assert back == v


# ---- O(n) R1CS / setup / expected-proof checker (oracle/c/oracle_r1cs.c), the
# checker of the full-size (2^24) Groth16 parity test
def _fr(v):
    return o.fr_to_bytes(v % o.R)


def _frs(vals):
    return b"".join(_fr(v) for v in vals)


@pytest.mark.parametrize("chains,rounds", [(2, 3), (5, 4)])
def test_c_mimc_r1cs_matches_python_oracle(chains, rounds):
    rcs = o.mimc_chain_r1cs(chains, rounds)
    inputs = [7 + 3 * i for i in range(chains)]
    w = o.mimc_chain_witness(rcs, inputs)
    cr = coracle.MimcR1CS(chains, rounds)
    assert (cr.ncons, cr.nw, cr.nb_public) == (len(rcs.constraints), rcs.nb_wires, rcs.nb_public)
    wc = cr.solve(_frs(inputs))
    assert bytes(wc) == _frs(w)
    A, B, C, bad = cr.abc(wc)
    assert bad == 0
    pa, pb, pc = rcs.solution(w)
    assert bytes(A) == _frs(pa) and bytes(B) == _frs(pb) and bytes(C) == _frs(pc)
    # key discrete logs vs the pinned Python setup
    tw = o.ToxicWaste(1234567, 891011, 121314, 151617, 181920)
    pk, _ = o.setup(rcs, tw)
    log_n = pk.domain.log_n
    ks = cr.key_scalars(log_n, _fr(tw.t), _fr(tw.alpha), _fr(tw.beta), _fr(tw.delta))
    assert ks["infA"] == bytes(int(x) for x in pk.infinity_A)
    assert ks["infB"] == bytes(int(x) for x in pk.infinity_B)
    assert ks["A"] == _frs(pk.scalars["A"]) and ks["B"] == _frs(pk.scalars["B"])
    assert ks["K"] == _frs(pk.scalars["K"])
    n = pk.domain.cardinality
    zb = [pk.scalars["Z"][o.bitrev(i, log_n)] for i in range(n)][: n - 1]
    assert ks["Z"] == _frs(zb)
    # proof discrete logs vs the big-int restatement (which runs computeH)
    r, s = 4242, 5353
    exp = o.expected_proof_scalars(rcs, tw, w, r, s)
    got = cr.expected(log_n, _fr(tw.t), _fr(tw.alpha), _fr(tw.beta), _fr(tw.delta), wc, _fr(r), _fr(s))
    assert got == tuple(_fr(x) for x in exp)
    # and vs the C oracle's full prove (MSMs + NTT computeH) on the key points
    g1 = o.g1_to_bytes(o.G1_GEN)
    g2 = o.g2_to_bytes(o.G2_GEN)

    def pts1(sc):
        k = len(sc) // 32
        return bytes(coracle.g1_batch_mul(g1, sc, k)) if k else b""

    def pts2(sc):
        k = len(sc) // 32
        return bytes(coracle.g2_batch_mul(g2, sc, k)) if k else b""
    ar, bs, krs, _ = coracle.groth16_prove(
        log_n, pts1(ks["A"]), len(ks["A"]) // 32, pts1(ks["B"]), len(ks["B"]) // 32, pts1(ks["Z"]),
        pts1(ks["K"]), len(ks["K"]) // 32, pts1(_fr(tw.alpha)), pts1(_fr(tw.beta)), pts1(_fr(tw.delta)),
        pts2(ks["B"]), pts2(_fr(tw.beta)), pts2(_fr(tw.delta)), ks["infA"], ks["infB"], bytes(wc), cr.nw,
        cr.nb_public, bytes(A), bytes(B), bytes(C), cr.ncons, _fr(r), _fr(s))
    assert ar == pts1(got[0]) and bs == pts2(got[1]) and krs == pts1(got[2])
    cr.close()


def test_c_eval_identities():
    """h (X^n - 1) = A B - C at a random point, with the O(n) evaluators."""
    chains, rounds, log_n = 3, 5, 6
    cr = coracle.MimcR1CS(chains, rounds, 1)
    assert cr.nb_public == 2
    w = cr.solve(_frs([11, 12, 13]))
    A, B, C, bad = cr.abc(w)
    assert bad == 0
    h = coracle.compute_h(bytes(A), bytes(B), bytes(C), cr.ncons, log_n)
    z = 0x1234567890ABCDEF
    hz = o.fr_from_bytes(coracle.eval_bitrev(h, log_n, _fr(z)))
    ev = [o.fr_from_bytes(coracle.eval_lagrange(bytes(v), cr.ncons, log_n, _fr(z))) for v in (A, B, C)]
    assert hz * (pow(z, 1 << log_n, o.R) - 1) % o.R == (ev[0] * ev[1] - ev[2]) % o.R
    # Lagrange evaluation = the iFFT coefficients evaluated (natural order)
    coef = o.fr_vec_from_bytes(coracle.ntt(bytes(A) + bytes(32 * ((1 << log_n) - cr.ncons)), log_n, 1, 1, 0))
    # DIF inverse: natural evaluations -> bit-reversed coefficients
    val = sum(coef[i] * pow(z, o.bitrev(i, log_n), o.R) for i in range(1 << log_n)) % o.R
    assert val == ev[0]


def test_c_fr_dot():
    from helpers import random_fr_mont
    a, b_ = random_fr_mont(777, 1), random_fr_mont(777, 2)
    av, bv = o.fr_vec_from_bytes(a.tobytes()), o.fr_vec_from_bytes(b_.tobytes())
    assert coracle.fr_dot(a, b_, 777) == o.fr_to_bytes(sum(x * y for x, y in zip(av, bv)) % o.R)
