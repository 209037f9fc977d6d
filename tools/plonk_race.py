"""Diagnostic: prove one small PlonK instance repeatedly and report which proof
components differ between runs (a race shows up as run-to-run differences)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "gnark-fork_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import bls12_381_oracle as bo  # noqa: E402
from plonk_circuits import Circuit, make_key, to_oracle  # noqa: E402
from gnark_amd import plonk_prover as pp  # noqa: E402

log_n, nbp, ncmt = (int(x) for x in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 6
circ = Circuit(log_n, 11 + log_n, nb_public=nbp, n_cmt=ncmt)
tau = random.Random(log_n).randrange(2, bo.R)
pk = make_key(circ, tau)
L, Rv, O, pub, cmts = circ.solve(pk, 99 + log_n, commit=pk.commit_lagrange)
proofs = [pp.prove(pk, L, Rv, O, rng=random.Random(5), public=pub, commitments=cmts) for _ in range(reps)]
for i, p in enumerate(proofs):
    pr, vk = to_oracle(pk, p)
    ok = bo.plonk_verify_trapdoor(pr, vk, tau, public=pub)
    diff = [f for f in ("LRO", "Z", "H", "bsb22", "batched_H", "claimed_values", "z_shifted_H", "z_shifted_value")
            if getattr(p, f) != getattr(proofs[0], f)]
    print(f"rep {i}: verifies={ok} differs_from_rep0={diff}", flush=True)
