"""TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker, never by the
product path): Groth16 BN254 with BSB22 commitments, restated in Python.

    setup_bsb22   setup.go:99-295      K split into pkK / vkK / ckK (committed
                                       private wires get gamma^-1 and go into the
                                       Pedersen bases), pedersen.Setup
    commit        prove.go:83-110      pedersen ProvingKey.Commit + the hint's
    commitment_hash                    hash_to_field of SerializeCommitment
                                       (constraint/commitment.go:76-88)
    prove_bsb22   prove.go:63-322      K MSM over filterHeap(wires, private
                                       committed + commitment wires) (238-248),
                                       pok = pedersen.BatchProve (prove.go:128-136)
    verify_bsb22  verify.go:43-140     commitment hashes appended to the public
                                       witness, FoldCommitments + pedersen Verify,
                                       commitments added into the K sum

gnark-crypto (v0.12.2-0.20231117165148-e77308824822, go.mod:10) is absent from
/root/reference, so pedersen.Setup / Commit / BatchProve / FoldCommitments /
Verify and hash_to_field are restated from their published algorithm:
  basisExpSigma = sigma * basis, GRootSigmaNeg = -(1/sigma) G;
  Verify(C, pok): e(C, G) e(pok, GRootSigmaNeg) == 1;
  several keys: r = SHA-256("r" | commitmentsSerialized) mod r (fiat-shamir
  transcript, one binding), fold = sum r^i C_i, pok = sum r^i sigma C_i;
  hash_to_field: RFC 9380 expand_message_xmd(SHA-256, DST "bsb22-commitment",
  48 B) mod r.
These byte-level details are "parity unpinned" (no fixture in the reference);
the pairing check pins the algebra.
"""
from __future__ import annotations

import hashlib

from bn254_oracle import (R, G1_GEN, G2_GEN, Domain, Proof, filter_heap, g1_add, g1_mul, g2_add, g2_mul,
                          g1_raw_encode, compute_h, inv, msm_g1, msm_g2, pairing_check, setup_abc, bitrev)

COMMITMENT_DST = b"bsb22-commitment"  # constraint/commitment.go:7


class Commitment:
    """constraint.Groth16Commitment: private committed wires, public committed
    wires (absolute ids < nb_public), the commitment (hint output) wire."""

    def __init__(self, private_committed, public_committed, commitment_index):
        self.private_committed = list(private_committed)
        self.public_committed = list(public_committed)
        self.commitment_index = commitment_index


def expand_message_xmd(msg: bytes, dst: bytes, n: int) -> bytes:
    """RFC 9380 5.3.1, SHA-256."""
    ell = (n + 31) // 32
    dst_prime = dst + bytes([len(dst)])
    b0 = hashlib.sha256(bytes(64) + msg + n.to_bytes(2, "big") + b"\x00" + dst_prime).digest()
    out, bi = b"", bytes(32)
    for i in range(1, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:n]


def hash_to_field(msg: bytes, dst: bytes = COMMITMENT_DST) -> int:
    """fr.Hash(msg, dst, 1): 48 bytes of expand_message_xmd, big-endian, mod r."""
    return int.from_bytes(expand_message_xmd(msg, dst, 48), "big") % R


def commitment_hash(commitment_point, public_values) -> int:
    """The BSB22 hint's output (prove.go:99-108): H(Marshal(C) | public committed
    values, 32 B big-endian each) -> fr."""
    msg = g1_raw_encode(commitment_point) + b"".join((v % R).to_bytes(32, "big") for v in public_values)
    return hash_to_field(msg)


def fold_challenge(commitments_serialized: bytes) -> int:
    """pedersen getChallenge: fiat-shamir transcript over SHA-256 with one
    challenge "r" and one binding."""
    return int.from_bytes(hashlib.sha256(b"r" + commitments_serialized).digest(), "big") % R


class PedersenKey:
    def __init__(self, basis, basis_exp_sigma):
        self.basis, self.basis_exp_sigma = basis, basis_exp_sigma


class PedersenVK:
    def __init__(self, g, g_root_sigma_neg):
        self.g, self.g_root_sigma_neg = g, g_root_sigma_neg


def pedersen_setup(bases, sigma: int, g_scalar: int):
    """pedersen.Setup(bases...) with sigma and G = g_scalar * G2 injected."""
    g = g2_mul(G2_GEN, g_scalar)
    sneg = (-inv(sigma, R)) % R
    vk = PedersenVK(g, g2_mul(g, sneg))
    pks = [PedersenKey(list(b), [g1_mul(p, sigma) for p in b]) for b in bases]
    return pks, vk


def pedersen_commit(pk: PedersenKey, values):
    return msm_g1(pk.basis, list(values))


def batch_prove(pks, values, commitments_serialized: bytes):
    if len(pks) == 1:
        return msm_g1(pks[0].basis_exp_sigma, list(values[0]))
    r = fold_challenge(commitments_serialized)
    basis, scaled, ri = [], [], 1
    for pk, v in zip(pks, values):
        basis += pk.basis_exp_sigma
        scaled += [x * ri % R for x in v]
        ri = ri * r % R
    return msm_g1(basis, scaled)


def fold_commitments(commitments, commitments_serialized: bytes):
    if len(commitments) == 1:
        return commitments[0]
    r = fold_challenge(commitments_serialized)
    acc, ri = None, 1
    for c in commitments:
        acc = g1_add(acc, g1_mul(c, ri))
        ri = ri * r % R
    return acc


def pedersen_verify(vk: PedersenVK, commitment, pok) -> bool:
    return pairing_check([(commitment, vk.g), (pok, vk.g_root_sigma_neg)])


class ProvingKeyBsb22:
    pass


class VerifyingKeyBsb22:
    pass


def k_remove(cinfo):
    """prove.go:238-241: private committed wires and the commitment wires."""
    rm = []
    for c in cinfo:
        rm += c.private_committed
    rm += [c.commitment_index for c in cinfo]
    return rm


def setup_bsb22(rcs, tw, cinfo, sigma: int, g_scalar: int):
    """setup.go:99-295 with commitments.  Returns (pk, vk); pk.k_wire_index is
    the absolute wire id of each pk.G1.K point (the filterHeap order)."""
    nw, nb_public = rcs.nb_wires, rcs.nb_public
    dom = Domain(len(rcs.constraints))
    A, B, C = setup_abc(rcs, dom, tw)
    cw = {c.commitment_index for c in cinfo}
    owner = {}
    for j, c in enumerate(cinfo):
        for wdx in c.private_committed:
            owner[wdx] = j
    pkK, vkK, ckK, kidx = [], [], [[] for _ in cinfo], []
    for i in range(nw):
        t1 = (A[i] * tw.beta + B[i] * tw.alpha + C[i]) % R
        if i < nb_public or i in cw:
            vkK.append(t1 * tw.gamma_inv % R)
        elif i in owner:
            ckK[owner[i]].append(t1 * tw.gamma_inv % R)
        else:
            pkK.append(t1 * tw.delta_inv % R)
            kidx.append(i)
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
    pk, vk = ProvingKeyBsb22(), VerifyingKeyBsb22()
    pk.domain = dom
    pk.g1_alpha, pk.g1_beta, pk.g1_delta = (g1_mul(G1_GEN, x) for x in (tw.alpha, tw.beta, tw.delta))
    pk.g1_A = [g1_mul(G1_GEN, s) for s in Af]
    pk.g1_B = [g1_mul(G1_GEN, s) for s in Bf]
    zpts = [g1_mul(G1_GEN, s) for s in Z]
    zpts = [zpts[bitrev(i, dom.log_n)] for i in range(n)]  # setup.go:265
    pk.g1_Z = zpts[: n - 1]
    pk.g1_K = [g1_mul(G1_GEN, s) for s in pkK]
    pk.k_wire_index = kidx
    pk.g2_B = [g2_mul(G2_GEN, s) for s in Bf]
    pk.g2_beta, pk.g2_delta = g2_mul(G2_GEN, tw.beta), g2_mul(G2_GEN, tw.delta)
    pk.infinity_A, pk.infinity_B = infA, infB
    bases = [[g1_mul(G1_GEN, s) for s in ck] for ck in ckK]
    pk.commitment_keys, vk.commitment_key = pedersen_setup(bases, sigma, g_scalar)
    pk.cinfo = cinfo
    vk.g1_alpha, vk.g2_beta, vk.g2_delta = pk.g1_alpha, pk.g2_beta, pk.g2_delta
    vk.g2_gamma = g2_mul(G2_GEN, tw.gamma)
    vk.g1_K = [g1_mul(G1_GEN, s) for s in vkK]
    # public committed wires as public-witness indexes (+1 for ONE), commitment
    # wires translated to their position after the public inputs (setup.go:295)
    vk.public_committed = [list(c.public_committed) for c in cinfo]
    vk.nb_public = nb_public
    return pk, vk


def solve_commitments(pk, w):
    """The solver's BSB22 hint for each commitment, in order (prove.go:83-110):
    the commitment point and its hash, written into w (in place)."""
    pts = []
    for j, c in enumerate(pk.cinfo):
        cp = pedersen_commit(pk.commitment_keys[j], [w[i] for i in c.private_committed])
        w[c.commitment_index] = commitment_hash(cp, [w[i] for i in c.public_committed])
        pts.append(cp)
    return pts


class ProofBsb22(Proof):
    def __init__(self, ar, bs, krs, commitments, pok):
        super().__init__(ar, bs, krs)
        self.commitments, self.pok = commitments, pok


def prove_bsb22(rcs, pk, w, commitments, r: int, s: int):
    """prove.go:63-322 with commitments (w already solved, commitment wires set)."""
    A, B, C = rcs.solution(w)
    dom = pk.domain
    h = compute_h(A, B, C, dom)
    wA = [w[i] for i in range(len(w)) if not pk.infinity_A[i]]
    wB = [w[i] for i in range(len(w)) if not pk.infinity_B[i]]
    ser = b"".join((w[c.commitment_index] % R).to_bytes(32, "big") for c in pk.cinfo)
    pok = batch_prove(pk.commitment_keys, [[w[i] for i in c.private_committed] for c in pk.cinfo], ser)
    kr = (-(r * s)) % R
    bs1 = g1_add(g1_add(msm_g1(pk.g1_B, wB), pk.g1_beta), g1_mul(pk.g1_delta, s))
    ar = g1_add(g1_add(msm_g1(pk.g1_A, wA), pk.g1_alpha), g1_mul(pk.g1_delta, r))
    n = dom.cardinality
    priv = filter_heap(w[rcs.nb_public:], rcs.nb_public, k_remove(pk.cinfo))
    krs = msm_g1(pk.g1_K, priv)
    krs = g1_add(krs, g1_mul(pk.g1_delta, kr))
    krs = g1_add(krs, msm_g1(pk.g1_Z, h[: n - 1]))
    krs = g1_add(krs, g1_mul(ar, s))
    krs = g1_add(krs, g1_mul(bs1, r))
    bs = g2_add(g2_add(msm_g2(pk.g2_B, wB), g2_mul(pk.g2_delta, s)), pk.g2_beta)
    return ProofBsb22(ar, bs, krs, list(commitments), pok)


def verify_bsb22(proof, vk, public_witness) -> bool:
    """verify.go:43-140 (public_witness excludes the ONE wire)."""
    pw = list(public_witness)
    ser = b""
    for j, pc in enumerate(vk.public_committed):
        hval = commitment_hash(proof.commitments[j], [pw[i - 1] for i in pc])
        pw.append(hval)
        ser += hval.to_bytes(32, "big")
    if proof.commitments:
        folded = fold_commitments(proof.commitments, ser)
        if not pedersen_verify(vk.commitment_key, folded, proof.pok):
            return False
    ksum = vk.g1_K[0]
    for x, k in zip(pw, vk.g1_K[1:]):
        ksum = g1_add(ksum, g1_mul(k, x))
    for c in proof.commitments:
        ksum = g1_add(ksum, c)
    neg = lambda q: (q[0], -q[1])
    from bn254_oracle import P
    na = (vk.g1_alpha[0], (-vk.g1_alpha[1]) % P)
    return pairing_check([(proof.Krs, neg(vk.g2_delta)), (proof.Ar, proof.Bs), (ksum, neg(vk.g2_gamma)),
                          (na, vk.g2_beta)])


def bsb22_test_circuit(nb_commitments: int = 1):
    """A small R1CS with BSB22 commitments, wire layout as the frontend builds it
    (public | secret | internal, the commitment wires are hint outputs, i.e.
    internal).  Wires: 0 ONE, 1 X (public), 2 a, 3 b, 4 c (secret), then the
    commitment wire(s) cw0 [cw1], then t1 = a b, t2 = t1 cw0, t3 = c cw_last,
    t4 = X a, t5 = (t2 + t3 + t4) X.
    Commitment 0: private (a, b), public (X); commitment 1: private (c)."""
    from bn254_oracle import R1CS
    cw = [5 + j for j in range(nb_commitments)]
    t1, t2, t3, t4, t5 = (5 + nb_commitments + k for k in range(5))
    cons = [
        ([(2, 1)], [(3, 1)], [(t1, 1)]),
        ([(t1, 1)], [(cw[0], 1)], [(t2, 1)]),
        ([(4, 1)], [(cw[-1], 1)], [(t3, 1)]),
        ([(1, 1)], [(2, 1)], [(t4, 1)]),
        ([(t2, 1), (t3, 1), (t4, 1)], [(1, 1)], [(t5, 1)]),
    ]
    rcs = R1CS(2, 3, nb_commitments + 5, cons)
    cinfo = [Commitment([2, 3], [1], cw[0])]
    if nb_commitments > 1:
        cinfo.append(Commitment([4], [], cw[1]))
    return rcs, cinfo


def bsb22_test_witness(rcs, pk, x, a, b, c):
    nb_c = len(pk.cinfo)
    w = [0] * rcs.nb_wires
    w[0], w[1], w[2], w[3], w[4] = 1, x % R, a % R, b % R, c % R
    pts = solve_commitments(pk, w)
    cw = [ci.commitment_index for ci in pk.cinfo]
    t1, t2, t3, t4, t5 = (5 + nb_c + k for k in range(5))
    w[t1] = w[2] * w[3] % R
    w[t2] = w[t1] * w[cw[0]] % R
    w[t3] = w[4] * w[cw[-1]] % R
    w[t4] = w[1] * w[2] % R
    w[t5] = (w[t2] + w[t3] + w[t4]) * w[1] % R
    return w, pts
