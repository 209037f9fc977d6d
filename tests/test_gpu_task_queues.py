"""Prove tasks on hardware queues of their own (common.h create_task_stream:
CU-masked streams, at most GG_TASK_QUEUES per device and process, later streams
from HIP's shared pool).  Proofs must not depend on where
a key's streams landed: dedicated queues, the shared pool, a budget that runs
out half-way through a key, budget returned by a closed key, and the timing
rehearsal handing the queues from shard to shard."""
import random

import pytest

import coracle

pytestmark = pytest.mark.gpu


def _case(log_n=12, n_wires=3000, seed=91):
    from gnark_amd import groth16
    from test_gpu_groth16 import synthetic_case
    d, wires, sa, sb, sc, ncons, r, s = synthetic_case(log_n, n_wires, 3, seed, k_inf_every=5)
    exp = coracle.groth16_prove(
        log_n, d["g1_A"], len(d["g1_A"]) // 64, d["g1_B"], len(d["g1_B"]) // 64, d["g1_Z"],
        d["g1_K"], len(d["g1_K"]) // 64, d["alpha1"], d["beta1"], d["delta1"], d["g2_B"],
        d["beta2"], d["delta2"], d["infinity_A"], d["infinity_B"], wires, n_wires, 3, sa, sb, sc,
        ncons, r, s)
    return groth16.ProvingKeyData(**d), groth16.Solution(wires, sa, sb, sc, n_wires, ncons), r, s, exp[:3]


@pytest.mark.parametrize("budget", ["0", "1", "3", "8"])
def test_groth16_any_queue_budget(budget, monkeypatch):
    """0: every task stream from the shared pool; 1 / 3: the budget runs out
    inside the key (G2 / computeH first); 8: all five dedicated."""
    from gnark_amd import backend, groth16
    monkeypatch.setenv("GG_TASK_QUEUES", budget)
    data, sol, r, s, exp = _case()
    pk = groth16.ProvingKey(data)
    pr = groth16.prove(pk, sol, backend.with_amd_acceleration(), r=r, s=s)
    assert (pr.Ar, pr.Bs, pr.Krs) == exp
    pk.close()


def test_groth16_keys_beyond_the_budget_and_back():
    """Three keys alive at once take 15 task streams against the default budget
    of 8 per device: the third key's streams all come from the pool.  Closing
    keys returns their queues; a key built afterwards proves the same."""
    from gnark_amd import backend, groth16
    data, sol, r, s, exp = _case()
    opt = backend.with_amd_acceleration()
    keys = [groth16.ProvingKey(data) for _ in range(3)]
    for pk in keys:
        pr = groth16.prove(pk, sol, opt, r=r, s=s)
        assert (pr.Ar, pr.Bs, pr.Krs) == exp
    for pk in keys:
        pk.close()
    pk = groth16.ProvingKey(data)
    pr = groth16.prove(pk, sol, opt, r=r, s=s)
    assert (pr.Ar, pr.Bs, pr.Krs) == exp
    pk.close()


def test_mpk_rehearsal_moves_the_queues():
    """set_rehearsal(r) re-creates the task streams of every shard on r's device
    (r's on dedicated queues, the others on the pool); solo shards 1, 3, 0 in
    turn, then the full proof again -- bit-exact with the single key."""
    from gnark_amd import backend, groth16
    data, sol, r, s, exp = _case(seed=93)
    opt = backend.with_amd_acceleration()
    mpk = groth16.MultiGpuProvingKey(data, [0] * 4)
    ref = mpk.prove(sol, opt, r=r, s=s)
    assert (ref.Ar, ref.Bs, ref.Krs) == exp
    for solo in (1, 3, 0):
        mpk.set_rehearsal(solo)
        mpk.prove(sol, opt, r=r, s=s, rehearsal_ok=True)
        assert mpk.shard_timings()[solo]["prove_ms"] > 0
    mpk.set_rehearsal(-1)
    assert mpk.prove(sol, opt, r=r, s=s) == ref
    mpk.close()


def test_plonk_one_device_key_any_queue_budget(monkeypatch):
    """A one-device PlonK key's four streams on dedicated queues (default) or
    the shared pool: the same proof for the same blinding, and it verifies."""
    import bls12_381_oracle as bo
    from gnark_amd import plonk_prover as pp
    from plonk_circuits import Circuit, make_key, to_oracle
    circ = Circuit(8, 19, nb_public=2, n_cmt=1)
    tau = 987654321
    proofs = []
    for budget in ("8", "0"):
        monkeypatch.setenv("GG_TASK_QUEUES", budget)
        pk = make_key(circ, tau)
        L, Rv, O, pub, cmts = circ.solve(pk, 17, commit=pk.commit_lagrange)
        proofs.append(pp.prove(pk, L, Rv, O, rng=random.Random(5), public=pub, commitments=cmts))
        if budget == "0":
            pr, vk = to_oracle(pk, proofs[-1])
            assert bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
        pk.close()
    assert proofs[0] == proofs[1]


@pytest.mark.parametrize("log_n", [12, 14])
def test_plonk_parts_on_dedicated_queues_rehearsal_handover(log_n, monkeypatch):
    """an 8-part PlonK key on this GPU with its parts' task
    streams on dedicated hardware queues (GG_PLONK_PART_QUEUES=1, GG_TASK_QUEUES=8:
    part 0 and part 1 take the device's eight at creation), the rehearsal handing
    the queues from part to part (re-created streams, r05k's configuration), then
    back to the creation layout -- the proof is byte-identical to the one-GPU
    proof before and after.  The library's waits are bounded (60 s here), so a
    stall fails with the wait named instead of hanging."""
    from gnark_amd import plonk_prover as pp
    from gnark_amd._lib import lib
    from plonk_circuits import Circuit, make_key, srs
    monkeypatch.setenv("GG_PLONK_PART_QUEUES", "1")
    monkeypatch.setenv("GG_TASK_QUEUES", "8")
    assert lib.gg_set_wait_timeout(60.0) == 0
    try:
        circ = Circuit(log_n, 31 + log_n, nb_public=1, n_cmt=1)
        tau = random.Random(log_n).randrange(2, pp.R)
        key_srs = srs(log_n, tau)
        pk0 = make_key(circ, tau, key_srs=key_srs)
        L, Rv, O, pub, cmts = circ.solve(pk0, 6, commit=pk0.commit_lagrange)
        ref = pp.prove(pk0, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts)
        pk0.close()
        pkm = make_key(circ, tau, key_srs=key_srs, devices=[0] * 8)
        assert pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts) == ref
        for part in (3, 0, 7, 5, 5, 1):
            pkm.set_rehearsal(True, part=part)
            for _ in range(2):
                pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts, rehearsal_ok=True)
            assert pkm.part_timings()[part]["msm_slices"] == 10
        pkm.set_rehearsal(False)
        assert pp.prove(pkm, L, Rv, O, rng=random.Random(17), public=pub, commitments=cmts) == ref
        pkm.close()
    finally:
        lib.gg_set_wait_timeout(0.0)
