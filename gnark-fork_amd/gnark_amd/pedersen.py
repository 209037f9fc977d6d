"""BSB22 commitments for Groth16 BN254 on MI355X: mirror of gnark-crypto's
ecc/bn254/fr/pedersen (ProvingKey.Commit / ProveKnowledge, BatchProve,
FoldCommitments; gnark-crypto v0.12.2-0.20231117165148-e77308824822, go.mod:10,
absent from the reference) with the MSMs on resident `MsmBase`s, and of the
BSB22 solver hint of backend/groth16/bn254/prove.go:83-110.

    keys  = [DevicePedersenKey(k) for k in pk_data.commitment_keys]  # with the key
    hints = Bsb22Hints(keys)                       # prove.go:76-81
    hints.hint(i, public_committed, private_committed) -> commitment wire value
    ...  solve the rest of the circuit with those values  ...
    proof = groth16.prove(pk, solution, opts, bsb22=hints)   # pok: prove.go:128-136

The hash of the hint (constraint.SerializeCommitment + hash_to_field.New(
"bsb22-commitment"), prove.go:99-108) and the fold challenge (fiat-shamir over
SHA-256, challenge "r") run on the host, as in gnark.  Their byte-level
encodings restate gnark-crypto and are "parity unpinned" (no fixture in the
reference); tests/test_gpu_groth16_bsb22.py checks every proof with the
restated pairing verifier (verify.go:43-140) and byte-for-byte against the
oracle's prover."""
from __future__ import annotations

import dataclasses
import hashlib
from typing import List, Optional, Sequence

from . import fr, msm

COMMITMENT_DST = b"bsb22-commitment"  # constraint/commitment.go:7


@dataclasses.dataclass
class ProvingKey:
    """pedersen.ProvingKey: Basis and BasisExpSigma, G1 affine in gnark's memory
    layout (64 B each)."""
    basis: bytes
    basis_exp_sigma: bytes

    @property
    def n(self) -> int:
        return len(self.basis) // 64


class DevicePedersenKey:
    """Both bases resident in HBM (built once with the Groth16 key)."""

    def __init__(self, key: ProvingKey):
        if len(key.basis) != len(key.basis_exp_sigma) or len(key.basis) % 64:
            raise ValueError("pedersen key: basis and basisExpSigma must have the same length")
        self.key, self.n = key, key.n
        self.basis = msm.MsmBase(msm.G1, key.basis, self.n) if self.n else None
        self.basis_exp_sigma = msm.MsmBase(msm.G1, key.basis_exp_sigma, self.n) if self.n else None

    def _msm(self, base, values: Sequence[int]) -> bytes:
        if len(values) != self.n:
            raise ValueError("pedersen: %d values for a basis of %d" % (len(values), self.n))
        if not self.n:
            return bytes(64)
        return base.msm(b"".join(fr.fr_mont(v % fr.R) for v in values), self.n)

    def commit(self, values: Sequence[int]) -> bytes:
        """ProvingKey.Commit: sum v_i Basis_i (affine, gnark layout)."""
        return self._msm(self.basis, values)

    def prove_knowledge(self, values: Sequence[int]) -> bytes:
        """ProvingKey.ProveKnowledge: sum v_i BasisExpSigma_i."""
        return self._msm(self.basis_exp_sigma, values)

    def close(self):
        for b in (self.basis, self.basis_exp_sigma):
            if b is not None:
                b.close()
        self.basis = self.basis_exp_sigma = None


def expand_message_xmd(msg: bytes, dst: bytes, n: int) -> bytes:
    """RFC 9380 5.3.1 with SHA-256 (gnark-crypto ecc/hash.ExpandMsgXmd)."""
    ell = (n + 31) // 32
    if ell > 255 or len(dst) > 255:
        raise ValueError("expand_message_xmd: output or DST too long")
    dst_prime = dst + bytes([len(dst)])
    b0 = hashlib.sha256(bytes(64) + msg + n.to_bytes(2, "big") + b"\x00" + dst_prime).digest()
    out, bi = b"", bytes(32)
    for i in range(1, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:n]


def hash_to_field(msg: bytes, dst: bytes = COMMITMENT_DST) -> int:
    """hash_to_field.New(dst): fr.Hash(msg, dst, 1) -> one element; the hint
    then reads back its 32 big-endian bytes with SetBytes (prove.go:100-107)."""
    return int.from_bytes(expand_message_xmd(msg, dst, 48), "big") % fr.R


def serialize_commitment(commitment_aff: bytes, public_committed: Sequence[int]) -> bytes:
    """constraint.SerializeCommitment(Marshal(C), publicCommitted, 32)."""
    return fr.g1_raw(commitment_aff) + b"".join((v % fr.R).to_bytes(32, "big") for v in public_committed)


def fold_challenge(commitments_serialized: bytes) -> int:
    """pedersen getChallenge: fiat-shamir transcript (SHA-256), challenge "r"
    bound to the serialized commitment wire values."""
    return int.from_bytes(hashlib.sha256(b"r" + commitments_serialized).digest(), "big") % fr.R


def batch_prove(keys: Sequence[DevicePedersenKey], values: Sequence[Sequence[int]],
                commitments_serialized: bytes) -> bytes:
    """pedersen.BatchProve: one key -> ProveKnowledge; several -> the values of
    key i scaled by r^i, one MSM per key on its resident BasisExpSigma, summed."""
    if len(keys) != len(values):
        raise ValueError("BatchProve: %d keys, %d value vectors" % (len(keys), len(values)))
    if not keys:
        return bytes(64)
    if len(keys) == 1:
        return keys[0].prove_knowledge(values[0])
    r = fold_challenge(commitments_serialized)
    acc, ri = None, 1
    for k, v in zip(keys, values):
        jac = k.basis_exp_sigma.msm_jac(b"".join(fr.fr_mont(x * ri % fr.R) for x in v), k.n) \
            if k.n else None
        if jac is not None:
            acc = jac if acc is None else msm.jac_add(msm.G1, acc, jac)
        ri = ri * r % fr.R
    return msm.jac_to_affine(msm.G1, acc) if acc is not None else bytes(64)


class Bsb22Hints:
    """The state prove.go's BSB22 hint override fills while the circuit is
    solved (prove.go:76-110): per commitment, the Pedersen commitment, the
    private committed values and the hint's output (the commitment wire)."""

    def __init__(self, keys: Sequence[DevicePedersenKey]):
        self.keys = list(keys)
        n = len(self.keys)
        self.commitments: List[Optional[bytes]] = [None] * n
        self.private_values: List[Optional[List[int]]] = [None] * n
        self.wire_values: List[Optional[int]] = [None] * n

    def hint(self, i: int, public_committed: Sequence[int], private_committed: Sequence[int]) -> int:
        """in = [i, publicAndCommitmentCommitted..., privateCommitted...] -> out[0]."""
        self.private_values[i] = [v % fr.R for v in private_committed]
        c = self.keys[i].commit(self.private_values[i])
        self.commitments[i] = c
        self.wire_values[i] = hash_to_field(serialize_commitment(c, public_committed))
        return self.wire_values[i]

    def complete(self) -> bool:
        return all(v is not None for v in self.wire_values)

    def pok(self) -> bytes:
        """pedersen.BatchProve(pk.CommitmentKeys, privateCommittedValues,
        commitmentsSerialized) (prove.go:128-136)."""
        if not self.complete():
            raise RuntimeError("BSB22: not every commitment hint was solved")
        ser = b"".join(v.to_bytes(32, "big") for v in self.wire_values)
        return batch_prove(self.keys, self.private_values, ser)


def k_wire_index(nb_public: int, n_wires: int, private_committed: Sequence[Sequence[int]],
                 commitment_indexes: Sequence[int]):
    """Absolute wire id of every pk.G1.K point: filterHeap(wires[nbPublic:],
    nbPublic, privateCommitted ++ commitmentIndexes) (prove.go:238-248)."""
    rm = set(commitment_indexes)
    for pc in private_committed:
        rm.update(pc)
    return [i for i in range(nb_public, n_wires) if i not in rm]
