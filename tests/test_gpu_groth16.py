"""Full Groth16 prove on the GPU (gg_groth16_prove) vs the oracle: bit-exact
proof bytes with injected r, s; the cubic proof also passes the pairing Verify."""
import numpy as np
import pytest

import bn254_oracle as o
import coracle
from helpers import b, golden, random_fr_mont, random_g1_points, random_g2_points

pytestmark = pytest.mark.gpu


def _pk_from_golden(g):
    from gnark_amd import groth16
    return groth16.ProvingKeyData(
        log_n=g["log_n"], g1_A=b(g["g1_A"]), g1_B=b(g["g1_B"]), g1_Z=b(g["g1_Z"]),
        g1_K=b(g["g1_K"]), alpha1=b(g["alpha1"]), beta1=b(g["beta1"]), delta1=b(g["delta1"]),
        g2_B=b(g["g2_B"]), beta2=b(g["beta2"]), delta2=b(g["delta2"]),
        infinity_A=b(g["infA"]), infinity_B=b(g["infB"]), nb_public=g["nb_public"])


@pytest.mark.parametrize("idx", [0, 1])
def test_groth16_golden(idx):
    from gnark_amd import backend, groth16, DeviceBuffer
    g = golden()["groth16"][idx]
    pk = groth16.ProvingKey(_pk_from_golden(g))
    nw = len(b(g["infA"]))
    ncons = len(b(g["solA"])) // 32
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]), nw, ncons)
    h = DeviceBuffer(32 << g["log_n"])
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=b(g["r"]), s=b(g["s"]), h_out=h)
    assert h.to_host().hex() == g["h"]
    assert pr.Ar.hex() == g["Ar"]
    assert pr.Bs.hex() == g["Bs"]
    assert pr.Krs.hex() == g["Krs"]
    assert pr.write_raw()[:256].hex() == g["raw_prefix"]


def test_groth16_cubic_gpu_proof_verifies():
    from gnark_amd import backend, groth16
    rcs = o.cubic_r1cs()
    tw = o.ToxicWaste(1234567, 891011, 121314, 151617, 181920)
    pko, vk = o.setup(rcs, tw)
    g = golden()["groth16"][0]
    pk = groth16.ProvingKey(_pk_from_golden(g))
    w = o.cubic_witness()
    A, B, C = rcs.solution(w)
    sol = groth16.Solution(o.fr_vec_to_bytes(w), o.fr_vec_to_bytes(A), o.fr_vec_to_bytes(B),
                           o.fr_vec_to_bytes(C), len(w), len(A))
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration())  # random r, s
    proof = o.Proof(o.g1_from_bytes(pr.Ar), o.g2_from_bytes(pr.Bs), o.g1_from_bytes(pr.Krs))
    assert o.verify(proof, vk, [35])
    assert not o.verify(proof, vk, [34])


def test_groth16_requires_accelerator_option():
    from gnark_amd import groth16
    g = golden()["groth16"][0]
    pk = groth16.ProvingKey(_pk_from_golden(g))
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]), 5, 3)
    with pytest.raises(RuntimeError):
        groth16.prove(pk, sol)


def synthetic_case(log_n, n_wires, nb_public, seed, inf_frac=0.1, k_inf_every=0):
    rng = np.random.default_rng(seed)
    n = 1 << log_n
    infA = (rng.random(n_wires) < inf_frac).astype(np.uint8)
    infB = (rng.random(n_wires) < 3 * inf_frac).astype(np.uint8)
    nA, nB, nK = int((infA == 0).sum()), int((infB == 0).sum()), n_wires - nb_public
    pts = random_g1_points(nA + nB + nK + n - 1 + 3, seed)
    off = 0

    def take(k):
        nonlocal off
        r = pts[off * 64:(off + k) * 64].tobytes()
        off += k
        return r

    d = dict(log_n=log_n, g1_A=take(nA), g1_B=take(nB), g1_K=take(nK), g1_Z=take(n - 1),
             alpha1=take(1), beta1=take(1), delta1=take(1))
    if k_inf_every:  # pk.G1.K may hold infinity points (setup.go:212-237; icicle.go:343-347)
        k = bytearray(d["g1_K"])
        for i in range(0, nK, k_inf_every):
            k[i * 64:(i + 1) * 64] = bytes(64)
        d["g1_K"] = bytes(k)
    g2 = random_g2_points(nB + 2, seed + 1).tobytes()
    d.update(g2_B=g2[:nB * 128], beta2=g2[nB * 128:(nB + 1) * 128], delta2=g2[(nB + 1) * 128:],
             infinity_A=infA.tobytes(), infinity_B=infB.tobytes(), nb_public=nb_public)
    ncons = n - 3
    wires = random_fr_mont(n_wires, seed + 2, "witness").tobytes()
    sa, sb, sc = (random_fr_mont(ncons, seed + 3 + i).tobytes() for i in range(3))
    r, s = o.fr_to_bytes(seed * 7919 + 1), o.fr_to_bytes(seed * 104729 + 3)
    return d, wires, sa, sb, sc, ncons, r, s


@pytest.mark.parametrize("log_n,n_wires,k_inf_every", [(6, 50, 0), (12, 3000, 0), (12, 3000, 7),
                                                       (15, 30000, 0)])
def test_groth16_synthetic_vs_oracle(log_n, n_wires, k_inf_every):
    from gnark_amd import backend, groth16, DeviceBuffer
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(log_n, n_wires, 3, 10 + log_n,
                                                       k_inf_every=k_inf_every)
    pk = groth16.ProvingKey(groth16.ProvingKeyData(**d))
    nw = n_wires
    exp = coracle.groth16_prove(
        log_n, d["g1_A"], len(d["g1_A"]) // 64, d["g1_B"], len(d["g1_B"]) // 64, d["g1_Z"],
        d["g1_K"], len(d["g1_K"]) // 64, d["alpha1"], d["beta1"], d["delta1"], d["g2_B"],
        d["beta2"], d["delta2"], d["infinity_A"], d["infinity_B"], wires, nw, 3, sa, sb, sc,
        ncons, r, s)
    sol = groth16.Solution(wires, sa, sb, sc, nw, ncons)
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=r, s=s)
    assert (pr.Ar, pr.Bs, pr.Krs) == exp[:3]
    # inputs resident on the device give the same proof
    dsol = groth16.Solution(*(DeviceBuffer.from_host(x) for x in (wires, sa, sb, sc)), nw, ncons,
                            on_device=True)
    pr2 = groth16.prove(pk, dsol, backend.with_amd_acceleration(), r=r, s=s)
    assert (pr2.Ar, pr2.Bs, pr2.Krs) == exp[:3]


# ---- multi-GPU key shards, rehearsed with all shards on one GPU
@pytest.mark.parametrize("idx,world", [(0, 2), (1, 2), (1, 3), (1, 8)])
def test_groth16_sharded_golden(idx, world):
    from gnark_amd import groth16
    g = golden()["groth16"][idx]
    data = _pk_from_golden(g)
    sol = groth16.Solution(b(g["wires"]), b(g["solA"]), b(g["solB"]), b(g["solC"]),
                           len(b(g["infA"])), len(b(g["solA"])) // 32)
    parts = []
    for rk in range(world):
        sh = groth16.ProvingKeyShard(data, rk, world)
        parts.append(groth16.prove_partial(sh, sol))
        sh.close()
    pr = groth16.finalize(data, groth16.add_partials(parts), b(g["r"]), b(g["s"]))
    assert (pr.Ar.hex(), pr.Bs.hex(), pr.Krs.hex()) == (g["Ar"], g["Bs"], g["Krs"])


@pytest.mark.parametrize("log_n,n_wires,k_inf_every,world", [(12, 3000, 7, 3), (15, 30000, 0, 4)])
def test_groth16_sharded_vs_oracle(log_n, n_wires, k_inf_every, world):
    from gnark_amd import groth16
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(log_n, n_wires, 3, 10 + log_n,
                                                       k_inf_every=k_inf_every)
    data = groth16.ProvingKeyData(**d)
    exp = coracle.groth16_prove(
        log_n, d["g1_A"], len(d["g1_A"]) // 64, d["g1_B"], len(d["g1_B"]) // 64, d["g1_Z"],
        d["g1_K"], len(d["g1_K"]) // 64, d["alpha1"], d["beta1"], d["delta1"], d["g2_B"],
        d["beta2"], d["delta2"], d["infinity_A"], d["infinity_B"], wires, n_wires, 3, sa, sb, sc,
        ncons, r, s)
    sol = groth16.Solution(wires, sa, sb, sc, n_wires, ncons)
    shards = [groth16.ProvingKeyShard(data, rk, world) for rk in range(world)]
    parts = [groth16.prove_partial(sh, sol) for sh in shards]
    pr = groth16.finalize(data, groth16.add_partials(parts), r, s)
    assert (pr.Ar, pr.Bs, pr.Krs) == exp[:3]
    # a shard is not a whole key: the single-GPU entry point refuses it
    with pytest.raises(Exception):
        groth16.prove(shards[0], sol, __import__("gnark_amd").backend.with_amd_acceleration(), r=r, s=s)
