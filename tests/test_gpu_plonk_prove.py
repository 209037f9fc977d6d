"""End-to-end PlonK BLS12-381 prove through the C-ABI prover (gg_plonk_prove:
prove.go:116-1079 inside libgnark_amd.so) on synthetic sparse-R1CS circuits with
public inputs and BSB22 commitments (tests/plonk_circuits.py), checked by the
PlonK verifier (verify.go:45-290) restated in the oracle -- gnark's transcript
encodings (Marshal = RawBytes, uncompressed: groth16/bls12-381/verify.go:80-82,
plonk/bn254/solidity.go:407-536),
PI(zeta), the BSB22 terms -- with the SRS trapdoor in place of the pairing.
Witnesses that break a gate, a copy constraint, a public input or a commitment
must not verify.  BASELINE configs[4] size: a 2^22 circuit."""
import hashlib
import random
import time

import pytest

import bls12_381_oracle as bo
from plonk_circuits import Circuit, make_key, srs, to_oracle, check_gates

pytestmark = pytest.mark.gpu
R = bo.R


def _prove(pk, circ, seed, **kw):
    from gnark_amd import plonk_prover as pp
    L, Rv, O, pub, cmts = circ.solve(pk, seed, commit=pk.commit_lagrange)
    check_gates(circ, L, Rv, O, pub, cmts)
    proof = pp.prove(pk, L, Rv, O, rng=random.Random(seed), public=pub, commitments=cmts, **kw)
    return proof, pub


@pytest.mark.parametrize("log_n,nb_public,n_cmt", [(3, 0, 0), (5, 0, 0), (6, 3, 0), (7, 0, 1), (8, 2, 1), (8, 0, 2), (7, 0, 2), (8, 2, 2)])
def test_plonk_prove_verifies(log_n, nb_public, n_cmt):
    circ = Circuit(log_n, 11 + log_n, nb_public=nb_public, n_cmt=n_cmt)
    tau = random.Random(log_n).randrange(2, R)
    pk = make_key(circ, tau)
    proof, pub = _prove(pk, circ, 99 + log_n)
    pr, vk = to_oracle(pk, proof)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    # a tampered claimed value, commitment or public input is rejected
    bad = dict(pr)
    bad["claimed"] = list(pr["claimed"])
    bad["claimed"][2] = (bad["claimed"][2] + 1) % R
    assert not bo.plonk_verify_trapdoor(bad, vk, tau, public=pub)
    bad = dict(pr)
    bad["Z"] = bo.g1_add(pr["Z"], bo.G1_GEN)
    assert not bo.plonk_verify_trapdoor(bad, vk, tau, public=pub)
    if nb_public:
        assert not bo.plonk_verify_trapdoor(pr, vk, tau, public=[pub[0] + 1] + list(pub[1:]))
    if n_cmt:
        bad = dict(pr)
        bad["bsb22"] = [bo.g1_add(pr["bsb22"][0], bo.G1_GEN)] + pr["bsb22"][1:]
        assert not bo.plonk_verify_trapdoor(bad, vk, tau, public=pub)
    pk.close()


def test_plonk_prove_deterministic_and_hash_option():
    """Fixed blinding -> identical proofs; the transcript hash is the caller's
    (opts.ChallengeHash / KZGFoldingHash): explicit SHA-256 == the default, and a
    proof made with BLAKE2s verifies only under BLAKE2s."""
    from gnark_amd import plonk_prover as pp
    circ = Circuit(6, 5, nb_public=1, n_cmt=1)
    tau = 123456789
    pk = make_key(circ, tau)
    L, Rv, O, pub, cmts = circ.solve(pk, 7, commit=pk.commit_lagrange)
    p1 = pp.prove(pk, L, Rv, O, rng=random.Random(3), public=pub, commitments=cmts)
    p2 = pp.prove(pk, L, Rv, O, rng=random.Random(3), public=pub, commitments=cmts,
                  challenge_hash=hashlib.sha256, folding_hash=hashlib.sha256)
    assert p1 == p2
    p3 = pp.prove(pk, L, Rv, O, rng=random.Random(3), public=pub, commitments=cmts,
                  challenge_hash=hashlib.blake2s, folding_hash=hashlib.blake2s)
    pr, vk = to_oracle(pk, p3)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub, challenge_hash=hashlib.blake2s,
                                    folding_hash=hashlib.blake2s)
    assert not bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    pk.close()


@pytest.mark.parametrize("which", ["gate", "copy", "public", "commitment"])
def test_plonk_prove_rejects_bad_witness(which):
    from gnark_amd import plonk_prover as pp
    circ = Circuit(6, 7, nb_public=2, n_cmt=1)
    tau = random.Random(3).randrange(2, R)
    pk = make_key(circ, tau)
    L, Rv, O, pub, cmts = circ.solve(pk, 5, commit=pk.commit_lagrange)
    L, Rv, O = bytearray(L), bytearray(Rv), bytearray(O)
    n = circ.n
    if which == "gate":  # an output that no longer satisfies its gate
        O[32 * (n - 2)] ^= 1
    elif which == "copy":  # a gate input that differs from the wire it copies
        r = n - 3
        L[32 * r] ^= 1
        # keep the gate itself satisfied: recompute the output
        from plonk_circuits import MINV, MONT, K_ADD
        a = int.from_bytes(L[32 * r:32 * r + 32], "little")
        b = int.from_bytes(Rv[32 * r:32 * r + 32], "little")
        c = (a + b) % R if int(circ.kind[r]) == K_ADD else a * b % R * MINV % R
        O[32 * r:32 * r + 32] = c.to_bytes(32, "little")
    elif which == "public":  # proof for one public input, verified against another
        pub = [pub[0]] + [(pub[1] + 1) % R]
    else:  # a commitment that is not the hashed one
        vals, dig, hv = cmts[0]
        cmts = [(vals, bo.g1_to_bytes(bo.g1_add(bo.g1_from_bytes(dig), bo.G1_GEN)), hv)]
    proof = pp.prove(pk, bytes(L), bytes(Rv), bytes(O), rng=random.Random(5), public=pub, commitments=cmts)
    pr, vk = to_oracle(pk, proof)
    assert not bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    pk.close()


@pytest.mark.parametrize("world", [2, 3])
def test_plonk_prove_sharded_kzg_matches(world):
    """Multi-GPU layout rehearsed on one GPU: `world` key shards (a KZG-base slice
    each, one thread per rank, partial commitments summed by the reduce callback
    through an in-process all-gather) produce exactly the single-key proof."""
    import threading
    from gnark_amd import msm, plonk_prover as pp
    circ = Circuit(6, 21, nb_public=1, n_cmt=1)
    tau = random.Random(8).randrange(2, R)
    key_srs = srs(6, tau)
    pk0 = make_key(circ, tau, key_srs=key_srs)
    L, Rv, O, pub, cmts = circ.solve(pk0, 4, commit=pk0.commit_lagrange)
    ref = pp.prove(pk0, L, Rv, O, rng=random.Random(42), public=pub, commitments=cmts)
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
            keys[r] = make_key(circ, tau, shard=(r, world), reduce=reducer(r), key_srs=key_srs)
            proofs[r] = pp.prove(keys[r], L, Rv, O, rng=random.Random(42), public=pub, commitments=cmts)
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
    pr, vk = to_oracle(pk0, ref)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)


@pytest.mark.parametrize("curve,log_n,nb_public,n_cmt", [
    ("bls12-381", 3, 0, 0), ("bls12-381", 4, 1, 0), ("bls12-381", 5, 2, 1), ("bls12-381", 6, 0, 2),
    ("bls12-381", 7, 3, 1), ("bls12-381", 8, 2, 2), ("bls12-381", 10, 2, 1), ("bls12-381", 12, 1, 2),
    ("bls12-381", 14, 1, 1),
    ("bn254", 3, 0, 0), ("bn254", 4, 1, 0), ("bn254", 5, 2, 1), ("bn254", 6, 0, 2), ("bn254", 8, 2, 2),
    ("bn254", 10, 1, 1), ("bn254", 12, 2, 1)])
def test_plonk_proof_bytes_match_oracle_prover(curve, log_n, nb_public, n_cmt):
    """Byte-exact PlonK on both curves (backend/plonk/bls12-381 and
    backend/plonk/bn254): the GPU proof equals the oracle's restatement of
    prove.go:116-1391 (oracle/plonk_prover_oracle.py) on the same circuit, key
    (same SRS trapdoor), witness, BSB22 hint values and blinding -- every
    commitment, claimed value and opening, and the vk digests; the transcript
    order and encodings are those the reference's Solidity verifier hashes
    (plonk/bn254/solidity.go:407-536, 961-1024)."""
    import plonk_prover_oracle as po
    from test_oracle_plonk_prover import blinding, ints, oracle_key
    from gnark_amd import plonk_prover as pp
    circ = Circuit(log_n, 70 + log_n, nb_public=nb_public, n_cmt=n_cmt, curve=curve)
    F = circ.F
    tau = random.Random(100 + log_n).randrange(2, F.R)
    pk = make_key(circ, tau)
    key = oracle_key(circ, tau)
    g = F.g1_from_bytes
    vk = key["vk"]
    assert [g(x) for x in pk.vk.S] == vk["S"] and [g(x) for x in pk.vk.Qcp] == vk["Qcp"]
    assert [g(x) for x in (pk.vk.Ql, pk.vk.Qr, pk.vk.Qm, pk.vk.Qo, pk.vk.Qk)] == \
        [vk["Ql"], vk["Qr"], vk["Qm"], vk["Qo"], vk["Qk"]]
    L, Rv, O, pub, cmts = circ.solve(pk, 9, commit=pk.commit_lagrange)
    for v, d, _ in cmts:  # bsb22Hint's kzg.Commit on the GPU == the oracle's
        assert g(d) == po.commit_lagrange(key, ints(v, F))
    got = pp.prove(pk, L, Rv, O, rng=random.Random(5), public=pub, commitments=cmts)
    if log_n >= 12:  # the split-iDFT quotient path (2^14+ big domains) through 4 device parts, same bytes
        pkm = make_key(circ, tau, devices=[0] * 4)
        assert pp.prove(pkm, L, Rv, O, rng=random.Random(5), public=pub, commitments=cmts) == got
        pkm.close()
    want = po.prove(key, ints(L, F), ints(Rv, F), ints(O, F), pub, [(ints(v, F), g(d), h) for v, d, h in cmts],
                    blinding(5, F.R))
    assert po.verify_trapdoor(key, want, pub)
    assert [g(x) for x in got.LRO] == want["LRO"]
    assert g(got.Z) == want["Z"]
    assert [g(x) for x in got.H] == want["H"]
    assert [g(x) for x in got.bsb22] == want["bsb22"]
    assert list(got.claimed_values) == want["claimed"]
    assert got.z_shifted_value == want["zu"]
    assert g(got.z_shifted_H) == want["zs_H"]
    assert g(got.batched_H) == want["batched_H"]
    pk.close()


@pytest.mark.parametrize("log_n,parts,n_cmt", [(6, 2, 1), (7, 3, 2), (8, 4, 0), (8, 8, 1), (10, 2, 0),
                                               (11, 8, 1), (11, 16, 0), (12, 3, 1)])
def test_plonk_prove_multi_device_matches(log_n, parts, n_cmt):
    """One process, `parts` device parts (gg_plonk_pk_create_multi) rehearsed on
    this GPU: KZG-base slices per part (commitments split and summed in the
    library), the copy-constraint ratio scanned per KzgLagrange slice and
    chained, the quotient units (U = rho S classes of the big domain: cosets,
    half cosets at 8 parts, quarter cosets at 16; per-unit inverse DFT blocks
    and the tail stages from 2^12 big domains) with the blocks copied back --
    exactly the one-GPU proof, also through commit_lagrange (the BSB22 hint)
    and from device-resident L, R, O."""
    from gnark_amd import DeviceBuffer, plonk_prover as pp
    circ = Circuit(log_n, 31 + log_n, nb_public=1, n_cmt=n_cmt)
    tau = random.Random(log_n + parts).randrange(2, R)
    key_srs = srs(log_n, tau)
    pk0 = make_key(circ, tau, key_srs=key_srs)
    L, Rv, O, pub, cmts = circ.solve(pk0, 6, commit=pk0.commit_lagrange)
    ref = pp.prove(pk0, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    pkm = make_key(circ, tau, key_srs=key_srs, devices=[0] * parts)
    assert pkm.devices() == [0] * parts
    assert pkm.vk == pk0.vk
    L2, Rv2, O2, pub2, cmts2 = circ.solve(pkm, 6, commit=pkm.commit_lagrange)
    assert (L2, Rv2, O2, pub2, cmts2) == (L, Rv, O, pub, cmts)
    got = pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    assert got == ref
    dev = [DeviceBuffer.from_host(x) for x in (L, Rv, O)]
    got_d = pp.prove(pkm, *dev, rng=random.Random(17), public=pub, commitments=cmts)
    assert got_d == ref
    pr, vk = to_oracle(pk0, ref)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    pkm.close()
    pk0.close()


def test_plonk_prove_distinct_devices():
    """Device parts on distinct GPUs when the box has them (skipped on a one-GPU
    box): Z slices pushed into the Z owner's buffer, canonical-form
    pushes, the quotient units' blocks and the scalar slices cross devices for
    real; the proof equals the one-GPU proof, and peer access is reported."""
    from gnark_amd import device_count, plonk_prover as pp
    nd = device_count()
    if nd < 2:
        pytest.skip("one GPU visible")
    log_n, parts = 12, (4 if nd >= 4 else 2)
    circ = Circuit(log_n, 77, nb_public=1, n_cmt=1)
    tau = random.Random(log_n).randrange(2, R)
    key_srs = srs(log_n, tau)
    pk0 = make_key(circ, tau, key_srs=key_srs)
    L, Rv, O, pub, cmts = circ.solve(pk0, 6, commit=pk0.commit_lagrange)
    ref = pp.prove(pk0, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    pkm = make_key(circ, tau, key_srs=key_srs, devices=list(range(parts)))
    pa = pkm.peer_access()
    assert all(pa[i][j] in ("enabled", "unavailable", "enable_failed") for i in range(parts) for j in range(parts)
               if i != j)
    got = pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    assert got == ref
    pkm.close()
    pk0.close()


def test_plonk_peer_access_same_device():
    from gnark_amd import plonk_prover as pp  # noqa: F401
    circ = Circuit(6, 5, nb_public=1, n_cmt=0)
    tau = random.Random(6).randrange(2, R)
    pkm = make_key(circ, tau, devices=[0, 0, 0])
    assert pkm.peer_access() == [["same_device"] * 3] * 3
    pkm.close()


@pytest.mark.parametrize("log_n,nb_public,n_cmt,parts", [(12, 2, 1, 1), (14, 1, 0, 4), (12, 1, 1, 8)])
def test_plonk_bn254_prove_verifies(log_n, nb_public, n_cmt, parts):
    """backend/plonk/bn254 at sizes the Python oracle verifies in seconds: the GPU
    proof passes the verifier restatement (verify.go:45-290 over BN254), from a
    one-GPU key and from a key split over `parts` device parts."""
    import plonk_prover_oracle as po
    from test_oracle_plonk_prover import oracle_key
    from gnark_amd import plonk_prover as pp
    circ = Circuit(log_n, 90 + log_n, nb_public=nb_public, n_cmt=n_cmt, curve="bn254")
    F = circ.F
    tau = random.Random(log_n).randrange(2, F.R)
    pk = make_key(circ, tau, devices=[0] * parts if parts > 1 else None)
    L, Rv, O, pub, cmts = circ.solve(pk, 3, commit=pk.commit_lagrange)
    check_gates(circ, L, Rv, O, pub, cmts)
    proof = pp.prove(pk, L, Rv, O, rng=random.Random(8), public=pub, commitments=cmts)
    key = oracle_key(circ, tau)
    g = F.g1_from_bytes
    pr = {"LRO": [g(x) for x in proof.LRO], "Z": g(proof.Z), "H": [g(x) for x in proof.H],
          "batched_H": g(proof.batched_H), "claimed": list(proof.claimed_values), "zs_H": g(proof.z_shifted_H),
          "zu": proof.z_shifted_value, "bsb22": [g(x) for x in proof.bsb22]}
    assert po.verify_trapdoor(key, pr, pub)
    bad = dict(pr)
    bad["claimed"] = list(pr["claimed"])
    bad["claimed"][3] = (bad["claimed"][3] + 1) % F.R
    assert not po.verify_trapdoor(key, bad, pub)
    pk.close()


def test_plonk_prove_2p22_verifies():
    """BASELINE configs[4]: a satisfied 2^22 sparse-R1CS circuit (2 public inputs,
    one BSB22 commitment) proven on the GPU and verified (trapdoor KZG checks)."""
    t0 = time.time()

    def log(m):
        print(f"  [{time.time() - t0:6.1f}s] {m}", flush=True)
    log_n = 22
    circ = Circuit(log_n, 2022, nb_public=2, n_cmt=1)
    log("circuit")
    tau = random.Random(22).randrange(2, R)
    pk = make_key(circ, tau)
    log("key (SRS, trace, resident coset evaluations)")
    proof, pub = _prove(pk, circ, 4242)
    log("witness + prove")
    from gnark_amd import plonk_prover as pp
    L, Rv, O, pub2, cmts = circ.solve(pk, 4242, commit=pk.commit_lagrange)
    tim = {}
    t = time.perf_counter()
    p2 = pp.prove(pk, L, Rv, O, rng=random.Random(4242), public=pub2, commitments=cmts, timings=tim)
    log(f"prove again {1e3 * (time.perf_counter() - t):.1f} ms {tim}")
    assert p2 == proof
    pr, vk = to_oracle(pk, proof)
    assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    bad = dict(pr)
    bad["claimed"] = list(pr["claimed"])
    bad["claimed"][0] = (bad["claimed"][0] + 1) % R
    assert not bo.plonk_verify_trapdoor(bad, vk, tau, public=pub)
    log("verified")
    pk.close()
    # BASELINE configs[4] is "8xMI355X": the same proof from a key split over 8
    # device parts (one process; rehearsed here with every part on this GPU)
    pk8 = make_key(circ, tau, devices=[0] * 8)
    log("8-part key")
    tim = {}
    t = time.perf_counter()
    p8 = pp.prove(pk8, L, Rv, O, rng=random.Random(4242), public=pub2, commitments=cmts, timings=tim)
    log(f"8-part prove {1e3 * (time.perf_counter() - t):.1f} ms {tim}")
    assert p8 == proof
    pk8.close()


@pytest.mark.parametrize("weight", ["0.5", "1.7"])
def test_plonk_multi_device_part0_weight(weight, monkeypatch):
    """Part 0's share of the KZG slices is a weight (plonk_part0_weight;
    GG_PLONK_PART0_WEIGHT): uneven slice boundaries on both bases, the ratio
    slices and Z's slices follow them -- the proof is still the one-GPU one."""
    from gnark_amd import plonk_prover as pp
    log_n, parts = 9, 5
    circ = Circuit(log_n, 40, nb_public=1, n_cmt=1)
    tau = random.Random(5).randrange(2, R)
    key_srs = srs(log_n, tau)
    pk0 = make_key(circ, tau, key_srs=key_srs)
    L, Rv, O, pub, cmts = circ.solve(pk0, 6, commit=pk0.commit_lagrange)
    ref = pp.prove(pk0, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    monkeypatch.setenv("GG_PLONK_PART0_WEIGHT", weight)
    pkm = make_key(circ, tau, key_srs=key_srs, devices=[0] * parts)
    monkeypatch.delenv("GG_PLONK_PART0_WEIGHT")
    assert pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts) == ref
    pkm.close()
    pk0.close()


def test_plonk_rehearsal_mode():
    """gg_plonk_pk_set_rehearsal (bench.py's split_projection): the primary part
    of a multi-part key proves with its peers idle -- the library returns
    GG_REHEARSAL, prove() refuses the proof unless asked for a rehearsal, the
    proof is not the real one (the peers' MSM slices and cosets are missing),
    and switching it off gives the real proof again on the same key.  Part
    timings: every part ran MSM slices, the coset owners their cosets."""
    from gnark_amd import plonk_prover as pp, GnarkAmdError
    from gnark_amd._lib import GG_REHEARSAL
    log_n, parts = 7, 4
    circ = Circuit(log_n, 45, nb_public=1, n_cmt=0)
    tau = random.Random(99).randrange(2, R)
    pkm = make_key(circ, tau, devices=[0] * parts)
    L, Rv, O, pub, cmts = circ.solve(pkm, 6, commit=pkm.commit_lagrange)
    ref = pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    pt = pkm.part_timings()
    assert len(pt) == parts
    assert all(p["msm_slices"] == 10 and p["msm_ms"] > 0 for p in pt)  # the ten KZG commitments
    assert all(p["scalar_MB"] > 0 for p in pt[1:])
    assert all(p["ratio_ms"] > 0 for p in pt)  # every part scans its slice of the ratio
    assert [p["quotient_units"] for p in pt] == [1, 1, 1, 1]  # rho = 4 classes: one per part
    # canonical forms (L R O Qk, then Z) on the 3 peers, none on part 0
    assert [p["canon_tasks"] for p in pt] == [0, 2, 2, 1]
    assert all(p["canon_MB"] > 0 for p in pt[1:])
    pkm.set_rehearsal(True)
    with pytest.raises(GnarkAmdError) as ei:
        pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
    assert ei.value.code == GG_REHEARSAL
    solo = pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts, rehearsal_ok=True)
    assert solo != ref
    assert all(p["msm_slices"] == 0 and p["quotient_units"] == 0 and p["canon_tasks"] == 0
               for p in pkm.part_timings()[1:])
    # a peer alone: its MSM slices, unit and canonical-form tasks (R, then Z), nothing of the others
    pkm.set_rehearsal(True, part=2)
    assert pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts, rehearsal_ok=True) != ref
    pt = pkm.part_timings()
    assert [p["msm_slices"] for p in pt] == [0, 0, 10, 0]
    assert [p["quotient_units"] for p in pt] == [0, 0, 1, 0]
    assert [p["canon_tasks"] for p in pt] == [0, 0, 2, 0]
    with pytest.raises(GnarkAmdError):
        pkm.set_rehearsal(True, part=parts)
    pkm.set_rehearsal(False)
    assert pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts) == ref
    pkm.close()
