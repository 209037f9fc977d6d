"""End-to-end PlonK BLS12-381 prove (gnark_amd.plonk_prover, prove.go:116-1079
over the device kernels) on small synthetic sparse-R1CS circuits, checked by the
PlonK verifier equations (verify.go:45-290) restated in the oracle with the SRS
trapdoor in place of the pairing.  A witness that breaks a gate or a copy
constraint must not verify."""
import random

import numpy as np
import pytest

import bls12_381_oracle as bo

pytestmark = pytest.mark.gpu
R = bo.R


def build_circuit(log_n, seed, break_gate=False, break_copy=False):
    """n gates; gate i is c = a * b or c = a + b; a_(i+1) is wired to c_i (copy
    constraint); b slots are fresh variables except every 4th, wired to b_0."""
    rnd = random.Random(seed)
    n = 1 << log_n
    var_of = {}  # slot -> variable id
    val = {}
    nxt = [0]

    def new(v):
        vid = nxt[0]
        nxt[0] += 1
        val[vid] = v % R
        return vid

    ql, qr, qm, qo, qk = ([0] * n for _ in range(5))
    a_var = new(rnd.randrange(R))
    b0 = None
    for i in range(n):
        if i % 4 == 3 and b0 is not None:
            b_var = b0
        else:
            b_var = new(rnd.randrange(R))
            if b0 is None:
                b0 = b_var
        a, b = val[a_var], val[b_var]
        if rnd.random() < 0.5:
            qm[i], qo[i] = 1, R - 1
            c = a * b % R
        else:
            ql[i], qr[i], qo[i] = 1, 1, R - 1
            c = (a + b) % R
        c_var = new(c)
        var_of[0 * n + i], var_of[1 * n + i], var_of[2 * n + i] = a_var, b_var, c_var
        a_var = c_var
    L = [val[var_of[i]] for i in range(n)]
    Rv = [val[var_of[n + i]] for i in range(n)]
    O = [val[var_of[2 * n + i]] for i in range(n)]
    # permutation: cycles over the slots of each variable
    groups = {}
    for s in range(3 * n):
        groups.setdefault(var_of[s], []).append(s)
    perm = [0] * (3 * n)
    for slots in groups.values():
        for k, s in enumerate(slots):
            perm[s] = slots[(k + 1) % len(slots)]
    if break_gate:
        O[n // 2] = (O[n // 2] + 1) % R
        # keep the copy constraint of the wire it feeds consistent
        if n // 2 + 1 < n:
            L[n // 2 + 1] = O[n // 2]
    if break_copy:
        # b_3 is wired to b_0: change b_3 and make gate 3 still hold
        Rv[3] = (Rv[3] + 5) % R
        O[3] = (L[3] * Rv[3] if qm[3] else L[3] + Rv[3]) % R
        if 4 < n:
            L[4] = O[3]
            O[4] = (L[4] * Rv[4] if qm[4] else L[4] + Rv[4]) % R
            for i in range(5, n):
                L[i] = O[i - 1]
                O[i] = (L[i] * Rv[i] if qm[i] else L[i] + Rv[i]) % R
    return n, (ql, qr, qm, qo, qk), perm, (L, Rv, O)


def srs(log_n, tau):
    from gnark_amd import msm, fr
    n = 1 << log_n
    w = fr.bls_domain_generator(log_n)
    gen = bo.g1_to_bytes(bo.G1_GEN)
    pw = b"".join(bo.fr_to_bytes(pow(tau, i, R)) for i in range(n + 3))
    kzg = msm.batch_scalar_mul(msm.BLS12_381_G1, gen, pw, n + 3)
    zn = (pow(tau, n, R) - 1) % R
    lag = [pow(w, i, R) * zn % R * pow(n * (tau - pow(w, i, R)), -1, R) % R for i in range(n)]
    return kzg, msm.batch_scalar_mul(msm.BLS12_381_G1, gen, bo.fr_vec_to_bytes(lag), n)


def make_key(log_n, sel, perm, tau, shard=None, reduce=None, key_srs=None):
    from gnark_amd import msm, plonk_prover as pp, fr
    n = 1 << log_n
    w = fr.bls_domain_generator(log_n)
    u = fr.BLS_FR_MULTIPLICATIVE_GEN
    kzg, kzg_lag = key_srs if key_srs is not None else srs(log_n, tau)
    ids = [pow(u, s // n, R) * pow(w, s % n, R) % R for s in range(3 * n)]
    s123 = [[ids[perm[j * n + i]] for i in range(n)] for j in range(3)]
    pk = pp.ProvingKey(log_n, kzg, kzg_lag, *[bo.fr_vec_to_bytes(q) for q in sel],
                       *[bo.fr_vec_to_bytes(s) for s in s123], np.asarray(perm, np.int64).tobytes(),
                       shard=shard, reduce=reduce)
    return pk


def to_oracle(pk, proof):
    g = bo.g1_from_bytes
    vk = {"n": pk.n, "omega": pk.omega, "u": pk.g, "S": [g(s) for s in pk.vk.S], "Ql": g(pk.vk.Ql),
          "Qr": g(pk.vk.Qr), "Qm": g(pk.vk.Qm), "Qo": g(pk.vk.Qo), "Qk": g(pk.vk.Qk)}
    pr = {"LRO": [g(x) for x in proof.LRO], "Z": g(proof.Z), "H": [g(x) for x in proof.H],
          "batched_H": g(proof.batched_H), "claimed": list(proof.claimed_values),
          "zs_H": g(proof.z_shifted_H), "zu": proof.z_shifted_value}
    return pr, vk


@pytest.mark.parametrize("log_n", [3, 5, 8])
def test_plonk_prove_verifies(log_n):
    from gnark_amd import plonk_prover as pp
    n, sel, perm, (L, Rv, O) = build_circuit(log_n, 11 + log_n)
    tau = random.Random(log_n).randrange(2, R)
    pk = make_key(log_n, sel, perm, tau)
    # the witness satisfies every gate and copy constraint
    for i in range(n):
        assert (sel[0][i] * L[i] + sel[1][i] * Rv[i] + sel[2][i] * L[i] * Rv[i] + sel[3][i] * O[i]
                + sel[4][i]) % R == 0
    proof = pp.prove(pk, bo.fr_vec_to_bytes(L), bo.fr_vec_to_bytes(Rv), bo.fr_vec_to_bytes(O),
                     rng=random.Random(99))
    pr, vk = to_oracle(pk, proof)
    assert bo.plonk_verify_trapdoor(pr, vk, tau)
    # a tampered claimed value or commitment is rejected
    bad = dict(pr)
    bad["claimed"] = list(pr["claimed"])
    bad["claimed"][2] = (bad["claimed"][2] + 1) % R
    assert not bo.plonk_verify_trapdoor(bad, vk, tau)
    bad = dict(pr)
    bad["Z"] = bo.g1_add(pr["Z"], bo.G1_GEN)
    assert not bo.plonk_verify_trapdoor(bad, vk, tau)


@pytest.mark.parametrize("which", ["gate", "copy"])
def test_plonk_prove_rejects_bad_witness(which):
    from gnark_amd import plonk_prover as pp
    log_n = 5
    n, sel, perm, (L, Rv, O) = build_circuit(log_n, 7, break_gate=(which == "gate"),
                                             break_copy=(which == "copy"))
    tau = random.Random(3).randrange(2, R)
    pk = make_key(log_n, sel, perm, tau)
    proof = pp.prove(pk, bo.fr_vec_to_bytes(L), bo.fr_vec_to_bytes(Rv), bo.fr_vec_to_bytes(O),
                     rng=random.Random(5))
    pr, vk = to_oracle(pk, proof)
    assert not bo.plonk_verify_trapdoor(pr, vk, tau)


@pytest.mark.parametrize("world", [2, 3])
def test_plonk_prove_sharded_kzg_matches(world):
    """Multi-GPU layout rehearsed on one GPU: `world` key shards (a KZG-base slice
    each, one thread per rank, partial commitments summed through an in-process
    all-gather) produce exactly the single-key proof."""
    import threading
    from gnark_amd import msm, plonk_prover as pp
    log_n = 6
    n, sel, perm, (L, Rv, O) = build_circuit(log_n, 21)
    tau = random.Random(8).randrange(2, R)
    key_srs = srs(log_n, tau)
    wit = [bo.fr_vec_to_bytes(v) for v in (L, Rv, O)]
    pk0 = make_key(log_n, sel, perm, tau, key_srs=key_srs)
    ref = pp.prove(pk0, *wit, rng=random.Random(42))
    slots = [None] * world
    bar = threading.Barrier(world)

    def reducer(r):
        def red(jac):
            slots[r] = jac
            bar.wait()
            acc = slots[0]
            for j in slots[1:]:
                acc = msm.jac_add(msm.BLS12_381_G1, acc, j)
            bar.wait()
            return acc
        return red

    keys, proofs, errs = [None] * world, [None] * world, []

    def run(r):
        try:
            keys[r] = make_key(log_n, sel, perm, tau, shard=(r, world), reduce=reducer(r), key_srs=key_srs)
            proofs[r] = pp.prove(keys[r], *wit, rng=random.Random(42))
        except Exception as e:  # pragma: no cover
            errs.append(e)
            bar.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not errs, errs
    for p in proofs:
        assert p == ref
    pr, vk = to_oracle(pk0, proofs[0])
    assert bo.plonk_verify_trapdoor(pr, vk, tau)
