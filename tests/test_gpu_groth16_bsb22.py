"""Groth16 BN254 with BSB22 commitments (backend/groth16/bn254/prove.go:83-136,
238-248; setup.go:99-295; verify.go:43-140): the GPU prover (K MSM over the
filtered wires, Pedersen commitments and the batched proof of knowledge on
resident bases) against the restated oracle (oracle/bn254_bsb22.py), byte for
byte with injected r, s, and through the restated pairing verifier.  gnark-crypto's
pedersen / hash_to_field encodings are restated, so the byte-level parity of
the commitment hash and fold challenge is "parity unpinned" (see the oracle's
header); the pairing check pins the algebra."""
import pytest

import bn254_oracle as o
import bn254_bsb22 as bo

TW = dict(t=987654321, alpha=1111, beta=2222, gamma=3333, delta=4444)


def _setup(nc):
    rcs, cinfo = bo.bsb22_test_circuit(nc)
    pk, vk = bo.setup_bsb22(rcs, o.ToxicWaste(**TW), cinfo, sigma=424242, g_scalar=77)
    return rcs, cinfo, pk, vk


# ---------------------------------------------------------------- CPU (oracle, host logic)
@pytest.mark.parametrize("nc", [1, 2])
def test_oracle_bsb22_verifies_and_rejects(nc):
    rcs, cinfo, pk, vk = _setup(nc)
    w, pts = bo.bsb22_test_witness(rcs, pk, x=3, a=5, b=7, c=11)
    pr = bo.prove_bsb22(rcs, pk, w, pts, r=101, s=103)
    pub = w[1:rcs.nb_public]
    assert bo.verify_bsb22(pr, vk, pub)
    assert not bo.verify_bsb22(pr, vk, [4])  # other public input -> other commitment hash
    bad_pok = bo.ProofBsb22(pr.Ar, pr.Bs, pr.Krs, pr.commitments, o.g1_add(pr.pok, o.G1_GEN))
    assert not bo.verify_bsb22(bad_pok, vk, pub)
    bad_c = bo.ProofBsb22(pr.Ar, pr.Bs, pr.Krs, [o.g1_mul(pr.commitments[0], 2)] + pr.commitments[1:], pr.pok)
    assert not bo.verify_bsb22(bad_c, vk, pub)


def test_bsb22_host_logic_matches_oracle():
    from gnark_amd import pedersen
    rcs, cinfo, pk, vk = _setup(2)
    kidx = pedersen.k_wire_index(rcs.nb_public, rcs.nb_wires, [c.private_committed for c in cinfo],
                                 [c.commitment_index for c in cinfo])
    assert kidx == pk.k_wire_index
    # filterHeap KAT shape (utils_test.go:17-38): the removed wires are exactly the committed ones
    assert set(range(rcs.nb_public, rcs.nb_wires)) - set(kidx) == {2, 3, 4, 5, 6}
    msg = bytes(range(97))
    assert pedersen.hash_to_field(msg) == bo.hash_to_field(msg)
    assert pedersen.fold_challenge(msg) == bo.fold_challenge(msg)
    pt = o.g1_mul(o.G1_GEN, 99)
    assert pedersen.serialize_commitment(o.g1_to_bytes(pt), [3, 4]) == \
        o.g1_raw_encode(pt) + (3).to_bytes(32, "big") + (4).to_bytes(32, "big")
    # RFC 9380 K.1 (expand_message_xmd, SHA-256, len 0x20, msg "")
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    assert pedersen.expand_message_xmd(b"", dst, 0x20).hex() == \
        "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"


def test_bsb22_host_errors():
    from gnark_amd import pedersen
    with pytest.raises(ValueError):
        pedersen.batch_prove([], [[1]], b"")
    with pytest.raises(ValueError):
        pedersen.ProvingKey(bytes(64), bytes(128)).n and pedersen.DevicePedersenKey(
            pedersen.ProvingKey(bytes(64), bytes(128)))
    h = pedersen.Bsb22Hints([])
    assert h.complete() and h.pok() == bytes(64)
    h2 = pedersen.Bsb22Hints([None])  # a key whose hint never ran
    with pytest.raises(RuntimeError):
        h2.pok()
    assert pedersen.k_wire_index(2, 6, [[3]], [5]) == [2, 4]


# ---------------------------------------------------------------- GPU
def _pk_data(rcs, pk, cinfo):
    from gnark_amd import groth16, pedersen
    cat = lambda pts, f: b"".join(f(p) for p in pts)
    return groth16.ProvingKeyData(
        log_n=pk.domain.log_n, g1_A=cat(pk.g1_A, o.g1_to_bytes), g1_B=cat(pk.g1_B, o.g1_to_bytes),
        g1_Z=cat(pk.g1_Z, o.g1_to_bytes), g1_K=cat(pk.g1_K, o.g1_to_bytes),
        alpha1=o.g1_to_bytes(pk.g1_alpha), beta1=o.g1_to_bytes(pk.g1_beta), delta1=o.g1_to_bytes(pk.g1_delta),
        g2_B=cat(pk.g2_B, o.g2_to_bytes), beta2=o.g2_to_bytes(pk.g2_beta), delta2=o.g2_to_bytes(pk.g2_delta),
        infinity_A=bytes(int(x) for x in pk.infinity_A), infinity_B=bytes(int(x) for x in pk.infinity_B),
        nb_public=rcs.nb_public,
        k_wire_index=pedersen.k_wire_index(rcs.nb_public, rcs.nb_wires, [c.private_committed for c in cinfo],
                                           [c.commitment_index for c in cinfo]),
        commitment_keys=[pedersen.ProvingKey(cat(k.basis, o.g1_to_bytes), cat(k.basis_exp_sigma, o.g1_to_bytes))
                         for k in pk.commitment_keys])


@pytest.mark.gpu
@pytest.mark.parametrize("nc", [1, 2])
def test_gpu_bsb22_prove_bit_exact_and_verifies(nc):
    from gnark_amd import backend, fr, groth16, pedersen
    rcs, cinfo, pk, vk = _setup(nc)
    dpk = groth16.ProvingKey(_pk_data(rcs, pk, cinfo))
    try:
        # solve: the BSB22 hints on the GPU, then the rest of the circuit
        w_ref, pts_ref = bo.bsb22_test_witness(rcs, pk, x=3, a=5, b=7, c=11)
        hints = pedersen.Bsb22Hints(dpk.commitment_keys)
        for j, c in enumerate(cinfo):
            val = hints.hint(j, [w_ref[i] for i in c.public_committed], [w_ref[i] for i in c.private_committed])
            assert val == w_ref[c.commitment_index]
            assert hints.commitments[j] == o.g1_to_bytes(pts_ref[j])
        A, B, C = rcs.solution(w_ref)
        sol = groth16.Solution(o.fr_vec_to_bytes(w_ref), o.fr_vec_to_bytes(A), o.fr_vec_to_bytes(B),
                               o.fr_vec_to_bytes(C), len(w_ref), len(A))
        r, s = 101, 103
        pr = groth16.prove(dpk, sol, backend.with_amd_acceleration(), r=fr.fr_mont(r), s=fr.fr_mont(s),
                           bsb22=hints)
        ref = bo.prove_bsb22(rcs, pk, w_ref, pts_ref, r=r, s=s)
        assert pr.Ar == o.g1_to_bytes(ref.Ar)
        assert pr.Bs == o.g2_to_bytes(ref.Bs)
        assert pr.Krs == o.g1_to_bytes(ref.Krs)
        assert list(pr.Commitments) == [o.g1_to_bytes(p) for p in ref.commitments]
        assert pr.CommitmentPok == o.g1_to_bytes(ref.pok)
        got = bo.ProofBsb22(o.g1_from_bytes(pr.Ar), o.g2_from_bytes(pr.Bs), o.g1_from_bytes(pr.Krs),
                            [o.g1_from_bytes(c) for c in pr.Commitments], o.g1_from_bytes(pr.CommitmentPok))
        assert bo.verify_bsb22(got, vk, w_ref[1:rcs.nb_public])
        raw = pr.write_raw()
        assert len(raw) == 64 + 128 + 64 + 4 + 64 * nc + 64
        assert raw[256:260] == nc.to_bytes(4, "big")
        # without the hints the key refuses (prove.go needs the hint state)
        with pytest.raises(ValueError):
            groth16.prove(dpk, sol, backend.with_amd_acceleration(), r=fr.fr_mont(r), s=fr.fr_mont(s))
    finally:
        dpk.close()


@pytest.mark.gpu
def test_gpu_bsb22_random_randomness_verifies():
    """Random r, s (prove.go:180-185) and another witness: the proof verifies."""
    from gnark_amd import backend, groth16, pedersen
    rcs, cinfo, pk, vk = _setup(1)
    dpk = groth16.ProvingKey(_pk_data(rcs, pk, cinfo))
    try:
        w, _ = bo.bsb22_test_witness(rcs, pk, x=8, a=123456789, b=987654321, c=42)
        hints = pedersen.Bsb22Hints(dpk.commitment_keys)
        c = cinfo[0]
        hints.hint(0, [w[i] for i in c.public_committed], [w[i] for i in c.private_committed])
        A, B, C = rcs.solution(w)
        sol = groth16.Solution(o.fr_vec_to_bytes(w), o.fr_vec_to_bytes(A), o.fr_vec_to_bytes(B),
                               o.fr_vec_to_bytes(C), len(w), len(A))
        pr = groth16.prove(dpk, sol, backend.with_amd_acceleration(), bsb22=hints)
        got = bo.ProofBsb22(o.g1_from_bytes(pr.Ar), o.g2_from_bytes(pr.Bs), o.g1_from_bytes(pr.Krs),
                            [o.g1_from_bytes(x) for x in pr.Commitments], o.g1_from_bytes(pr.CommitmentPok))
        assert bo.verify_bsb22(got, vk, [8])
        assert not bo.verify_bsb22(got, vk, [9])
    finally:
        dpk.close()
