"""BLS12-381 G2 MSM and the Groth16 prover over BLS12-381
(backend/groth16/bls12-381/prove.go:63-396: the BN254 prover's code over another
curve), through the C ABI.

* G2 MSM (GG_BLS12_381_G2) vs the trapdoor identity MSM(k_i G2, s_i) =
  (sum s_i k_i) G2, checked by the oracle's exact G2 arithmetic (pinned by the
  reference's bellman_test.go G2 points), including window 20 and skewed scalars.
* Groth16 over BLS12-381: a satisfied MiMC-chain R1CS, key from seeded toxic
  waste (setup.go layout: infinity flags, filtered A/B, K, bit-reversed Z); the
  proof must equal (a G1, b G2, c G1) with (a, b, c) the proof's discrete logs
  (bls12_381_oracle.groth16_expected_scalars), from host and device inputs; a
  broken witness must not give it.
"""
import random

import pytest

import bls12_381_oracle as bo

pytestmark = pytest.mark.gpu
R = bo.R
MONT = (1 << 256) % R


def frb(x):
    return (x % R * MONT % R).to_bytes(32, "little")


def frv(xs):
    return b"".join(frb(x) for x in xs)


G1B = bo.g1_to_bytes(bo.G1_GEN)
G2B = bo.g2_to_bytes(bo.G2_GEN)


def test_bls_g2_host_helpers_and_batch_mul():
    from gnark_amd import msm
    G2 = msm.BLS12_381_G2
    ks = [1, 2, 7, R - 1, 123456789123456789]
    pts = msm.batch_scalar_mul(G2, G2B, frv(ks), len(ks))
    for i, k in enumerate(ks):
        assert bo.g2_from_bytes(pts[192 * i:192 * (i + 1)]) == bo.g2_mul(bo.G2_GEN, k)
    j = msm.scalar_mul(G2, pts[:192], frb(5))
    assert bo.g2_from_bytes(msm.jac_to_affine(G2, j)) == bo.g2_mul(bo.G2_GEN, 5)
    j2 = msm.jac_add(G2, j, msm.scalar_mul(G2, pts[192:384], frb(3)))
    assert bo.g2_from_bytes(msm.jac_to_affine(G2, j2)) == bo.g2_mul(bo.G2_GEN, 11)
    # zero scalar -> infinity
    z = msm.batch_scalar_mul(G2, G2B, frv([0]), 1)
    assert z == bytes(192)


@pytest.mark.parametrize("n,dist,window", [(1, "uniform", 0), (7, "uniform", 0), (1000, "uniform", 0),
                                           (1000, "witness", 0), (1 << 14, "uniform", 0),
                                           (1 << 16, "witness", 20), (1 << 16, "skew", 0)])
def test_bls_g2_msm_trapdoor(n, dist, window):
    from gnark_amd import msm
    G2 = msm.BLS12_381_G2
    rnd = random.Random(n + window)
    ks = [rnd.randrange(1, R) for _ in range(n)]
    if dist == "uniform":
        sc = [rnd.randrange(R) for _ in range(n)]
    elif dist == "witness":  # half 0/1, as real witnesses
        sc = [rnd.choice((0, 1)) if rnd.random() < 0.5 else rnd.randrange(R) for _ in range(n)]
    else:  # one value everywhere: every entry in one bucket per window
        sc = [123456789] * n
    pts = msm.batch_scalar_mul(G2, G2B, frv(ks), n)
    base = msm.MsmBase(G2, pts, n, window_bits=window)
    got = bo.g2_from_bytes(base.msm(frv(sc), n))
    want = bo.g2_mul(bo.G2_GEN, sum(k * s for k, s in zip(ks, sc)) % R)
    assert got == want
    base.close()


def mimc_bls(chains, rounds):
    """x^5-style chains over BLS12-381 fr (the BN254 test's R1CS shape):
    per round t = x x, u = t t, x' = u x + k (3 constraints)."""
    cons, wid = [], 1 + chains
    for ch in range(chains):
        x = 1 + ch
        for rd in range(rounds):
            k = (rd * 7 + 3) % R
            t, u, xn = wid, wid + 1, wid + 2
            wid += 3
            cons.append(([(x, 1)], [(x, 1)], [(t, 1)]))
            cons.append(([(t, 1)], [(t, 1)], [(u, 1)]))
            cons.append(([(u, 1)], [(x, 1)], [(xn, 1), (0, (-k) % R)]))
            x = xn
    return cons, wid


def solve(cons, nw, inputs):
    w = [0] * nw
    w[0] = 1
    for i, v in enumerate(inputs):
        w[1 + i] = v % R
    for L, Rr, O in cons:
        a = sum(w[i] * k for i, k in L) % R
        b = sum(w[i] * k for i, k in Rr) % R
        out, _ = O[0]
        w[out] = (a * b - sum(w[i] * k for i, k in O[1:])) % R
    return w


def abc(cons, w):
    ev = [[sum(w[i] * k for i, k in part) % R for part in row] for row in cons]
    return [e[0] for e in ev], [e[1] for e in ev], [e[2] for e in ev]


@pytest.mark.parametrize("log_n", [6, 12, 16])
def test_groth16_bls12_381_bit_exact(log_n):
    from gnark_amd import backend, groth16, msm, DeviceBuffer
    rounds = 5 if log_n < 10 else 85
    chains = max(1, ((1 << log_n) - 1) // (3 * rounds))
    cons, nw = mimc_bls(chains, rounds)
    assert (1 << (log_n - 1)) < len(cons) <= (1 << log_n)
    rnd = random.Random(log_n)
    w = solve(cons, nw, [rnd.randrange(R) for _ in range(chains)])
    A, B, C = abc(cons, w)
    t, al, be, de = 0x1DEA5EED1234567 + log_n, 0xA1FA0001, 0xBE7A0002, 0xDE17A0003
    ks = bo.groth16_setup_scalars(cons, nw, 1, log_n, t, al, be, de)
    G1, G2 = msm.BLS12_381_G1, msm.BLS12_381_G2

    def p1(xs):
        return msm.batch_scalar_mul(G1, G1B, frv(xs), len(xs)) if xs else b""

    def p2(xs):
        return msm.batch_scalar_mul(G2, G2B, frv(xs), len(xs)) if xs else b""
    data = groth16.ProvingKeyData(
        log_n=log_n, g1_A=p1(ks["A"]), g1_B=p1(ks["B"]), g1_Z=p1(ks["Z"]), g1_K=p1(ks["K"]),
        alpha1=p1([al]), beta1=p1([be]), delta1=p1([de]), g2_B=p2(ks["B"]), beta2=p2([be]),
        delta2=p2([de]), infinity_A=bytes(ks["infA"]), infinity_B=bytes(ks["infB"]), nb_public=1,
        curve="bls12-381")
    pk = groth16.ProvingKey(data)
    r, s = 0x5EED0001, 0x5EED0002
    ea, eb, ec = bo.groth16_expected_scalars(cons, w, 1, log_n, ks, t, al, be, de, r, s)
    want = (bo.g1_mul(bo.G1_GEN, ea), bo.g2_mul(bo.G2_GEN, eb), bo.g1_mul(bo.G1_GEN, ec))
    opt = backend.with_amd_acceleration()
    sol = groth16.Solution(frv(w), frv(A), frv(B), frv(C), nw, len(cons))
    pr = groth16.prove(pk, sol, opt, r=frb(r), s=frb(s))
    got = (bo.g1_from_bytes(pr.Ar), bo.g2_from_bytes(pr.Bs), bo.g1_from_bytes(pr.Krs))
    assert got == want
    dev = [DeviceBuffer.from_host(frv(x)) for x in (w, A, B, C)]
    pr2 = groth16.prove(pk, groth16.Solution(*dev, nw, len(cons), on_device=True), opt, r=frb(r), s=frb(s))
    assert (pr2.Ar, pr2.Bs, pr2.Krs) == (pr.Ar, pr.Bs, pr.Krs)
    # the same witness solved on the GPU over BLS12-381 fr (gg_r1cs_create_ex), proved from HBM
    from gnark_amd import solver
    sys_ = solver.R1CS.from_terms(1, chains, nw, cons, curve="bls12-381")
    gsol = sys_.solve(w[1:1 + chains])
    pr4 = groth16.prove(pk, gsol, opt, r=frb(r), s=frb(s))
    assert (pr4.Ar, pr4.Bs, pr4.Krs) == (pr.Ar, pr.Bs, pr.Krs)
    # one-process multi-GPU key (gg_groth16_mpk_create_ex over BLS12-381): shards
    # on device 0 rehearse the N-GPU layout; host, replicated and GPU-solved inputs
    world = {6: 2, 12: 3, 16: 8}[log_n]
    mpk = groth16.MultiGpuProvingKey(data, [0] * world)
    assert mpk.info() == (world, world & (world - 1) == 0)  # distributed computeH (power-of-two worlds)
    prm = mpk.prove(sol, opt, r=frb(r), s=frb(s))
    assert (prm.Ar, prm.Bs, prm.Krs) == (pr.Ar, pr.Bs, pr.Krs)
    prd = mpk.prove(groth16.replicate_solution(sol, [0] * world), opt, r=frb(r), s=frb(s))
    assert (prd.Ar, prd.Bs, prd.Krs) == (pr.Ar, pr.Bs, pr.Krs)
    prg = mpk.prove(sys_.solve(w[1:1 + chains]), opt, r=frb(r), s=frb(s))
    assert (prg.Ar, prg.Bs, prg.Krs) == (pr.Ar, pr.Bs, pr.Krs)
    mpk.close()
    if world & (world - 1) == 0:  # bucket stripes over BLS12-381 G1 / G2 tables
        import os
        os.environ["GG_MPK_SPLIT"] = "stripes"
        try:
            mps = groth16.MultiGpuProvingKey(data, [0] * world)
        finally:
            del os.environ["GG_MPK_SPLIT"]
        assert mps.split() == "stripes"
        prs = mps.prove(sol, opt, r=frb(r), s=frb(s))
        assert (prs.Ar, prs.Bs, prs.Krs) == (pr.Ar, pr.Bs, pr.Krs)
        mps.close()
    sys_.close()
    bad = list(w)
    bad[-1] = (bad[-1] + 1) % R
    pr3 = groth16.prove(pk, groth16.Solution(frv(bad), frv(A), frv(B), frv(C), nw, len(cons)), opt,
                        r=frb(r), s=frb(s))
    assert bo.g1_from_bytes(pr3.Krs) != want[2]
    pk.close()
