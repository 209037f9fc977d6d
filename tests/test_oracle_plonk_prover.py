"""The oracle's PlonK prover restatement (oracle/plonk_prover_oracle.py,
prove.go:116-1391) against the oracle's verifier restatement (verify.go:45-290,
SRS trapdoor instead of the pairing): its proofs of satisfied circuits with
public inputs and BSB22 commitments verify, tampered ones do not.  CPU only;
the GPU prover is compared with it byte for byte in test_gpu_plonk_prove.py."""
import random

import pytest

import bls12_381_oracle as bo
import plonk_prover_oracle as po
from plonk_circuits import Circuit, MINV

R = bo.R


def ints(b, F=None):
    """Montgomery bytes -> ints of the circuit's field (BLS12-381 by default)."""
    R_, minv = (F.R, F.MINV) if F is not None else (R, MINV)
    return [int.from_bytes(b[i:i + 32], "little") * minv % R_ for i in range(0, len(b), 32)]


def oracle_key(circ, tau):
    F = circ.F
    sel, qcp = circ.selectors()
    perm = circ.permutation()
    s123 = circ.s_polys(perm, F.cv.omega(circ.n), F.cv.fr_gen)
    return po.setup(F.cv, circ.log_n, *[ints(x, F) for x in sel], *[ints(x, F) for x in s123],
                    [ints(x, F) for x in qcp], perm.tolist(), circ.nb_public, circ.cmt_idx, tau)


def oracle_solve(circ, key, seed):
    F = circ.F

    def commit(vals):
        return F.g1_to_bytes(po.commit_lagrange(key, ints(vals, F)))
    L, Rv, O, pub, cmts = circ.solve(None, seed, commit=commit)
    return ints(L, F), ints(Rv, F), ints(O, F), pub, [(ints(v, F), F.g1_from_bytes(d), h) for v, d, h in cmts]


def blinding(seed, R_=R):
    rnd = random.Random(seed)  # the order of gnark_amd.plonk_prover.prove: Bl, Br, Bo (2 each), Bz (3)
    return [rnd.randrange(R_) for _ in range(9)]


def to_verifier(key, pr):
    vk = key["vk"]
    return pr, {"n": key["n"], "omega": key["omega"], "u": key["u"], "S": vk["S"], "Ql": vk["Ql"], "Qr": vk["Qr"],
                "Qm": vk["Qm"], "Qo": vk["Qo"], "Qk": vk["Qk"], "Qcp": vk["Qcp"], "nb_public": key["nb_public"],
                "cmt_idx": key["cmt_idx"]}


@pytest.mark.parametrize("log_n,nb_public,n_cmt", [(3, 0, 0), (4, 1, 0), (5, 2, 1), (5, 0, 2)])
def test_oracle_prover_verifies(log_n, nb_public, n_cmt):
    circ = Circuit(log_n, 50 + log_n, nb_public=nb_public, n_cmt=n_cmt)
    tau = random.Random(log_n).randrange(2, R)
    key = oracle_key(circ, tau)
    L, Rv, O, pub, cmts = oracle_solve(circ, key, 7)
    pr = po.prove(key, L, Rv, O, pub, cmts, blinding(3))
    proof, vk = to_verifier(key, pr)
    assert bo.plonk_verify_trapdoor(proof, vk, tau, public=pub)
    bad = dict(proof)
    bad["claimed"] = list(proof["claimed"])
    bad["claimed"][1] = (bad["claimed"][1] + 1) % R
    assert not bo.plonk_verify_trapdoor(bad, vk, tau, public=pub)
    if nb_public:
        assert not bo.plonk_verify_trapdoor(proof, vk, tau, public=[(pub[0] + 1) % R] + list(pub[1:]))
    # another blinding: another proof, still valid (blinding is free)
    pr2 = po.prove(key, L, Rv, O, pub, cmts, blinding(4))
    assert pr2["LRO"] != pr["LRO"]
    assert bo.plonk_verify_trapdoor(*to_verifier(key, pr2), tau, public=pub)


@pytest.mark.parametrize("curve,log_n,nb_public,n_cmt", [("bls12-381", 4, 1, 1), ("bn254", 3, 0, 0),
                                                         ("bn254", 4, 1, 0), ("bn254", 5, 2, 1),
                                                         ("bn254", 5, 0, 2)])
def test_oracle_prover_generic_verifier(curve, log_n, nb_public, n_cmt):
    """backend/plonk/bn254 is the same prover over BN254: the oracle prover's BN254
    proofs pass the curve-generic verifier restatement (transcript = the Solidity
    verifier's, plonk/bn254/solidity.go:407-536, 961-1024); on BLS12-381 that
    verifier agrees with the reference-pinned one above."""
    circ = Circuit(log_n, 60 + log_n, nb_public=nb_public, n_cmt=n_cmt, curve=curve)
    F = circ.F
    tau = random.Random(log_n + 1).randrange(2, F.R)
    key = oracle_key(circ, tau)
    L, Rv, O, pub, cmts = oracle_solve(circ, key, 11)
    pr = po.prove(key, L, Rv, O, pub, cmts, blinding(6, F.R))
    assert po.verify_trapdoor(key, pr, pub)
    bad = dict(pr)
    bad["zu"] = (pr["zu"] + 1) % F.R
    assert not po.verify_trapdoor(key, bad, pub)
    if curve == "bls12-381":
        assert bo.plonk_verify_trapdoor(*to_verifier(key, pr), tau, public=pub)
