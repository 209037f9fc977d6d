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
